#!/bin/bash
# GPU box: the GAE scan under several libraries (PRL_HIP_LIB=...), interleaved, on fixed 500 /
# 200-step segments (trained CartPole / Pendulum) and on random 5 % breaks.
# Usage: gae_ab.sh "PRL_HIP_LIB=tools/exp/lib_a.so" "X=1" ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for rep in 1 2; do
  for args in "--gae-n 32764206 --gae-seg 500" "--gae-n 8269824 --gae-seg 500" "--gae-n 13107200 --gae-seg 200" "--gae-n 32764206"; do
    for cfg in "$@"; do
      out=$(env $cfg timeout -k 10 120 python -u tools/kernel_bench.py $args) || { echo "fail $cfg $args"; exit 1; }
      echo "$cfg $args $out"
    done
  done
done
