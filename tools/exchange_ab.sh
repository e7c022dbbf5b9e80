#!/bin/bash
# GPU box: A/B of two engine builds (PRL_HIP_LIB) at mb 512, with the tile (PRL_UPD_PROFILE=1) and
# without it (=2: the exchange + AdamW alone).  Usage: tools/exchange_ab.sh lib_a.so lib_b.so
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for lib in "$@"; do
  for mode in 1 2; do
    PRL_HIP_LIB=$PWD/$lib PRL_UPD_PROFILE=$mode timeout -k 10 120 python -u tools/engine_profile.py 262144 512 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    echo "$lib mode=$mode $(grep '"mb"' gpurun_out/ab.log)"
  done
done
