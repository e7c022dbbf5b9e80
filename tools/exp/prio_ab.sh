#!/bin/bash
# GPU box: engine tests, then mb 512 A/B (engine_ab.sh, PROF=0) and mb 65,536 CartPole / Pendulum
# learn() timings for the libraries named (PRL_HIP_LIB=...; "X=1" for the in-tree one).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py tests/test_tp_learn_gpu.py tests/test_wide_gpu.py > gpurun_out/prio_tests.log 2>&1 || { tail -30 gpurun_out/prio_tests.log; exit 1; }
tail -1 gpurun_out/prio_tests.log
PROF=0 bash tools/exp/engine_ab.sh "$@" || exit 1
for rep in 1 2; do for cfg in "$@"; do for net in cartpole pendulum; do
  env $cfg PRL_UPD_PROFILE=0 timeout -k 10 120 python -u tools/engine_profile.py 1048576 65536 $net > gpurun_out/pab.log 2>&1 || { tail -3 gpurun_out/pab.log; exit 1; }
  echo "$cfg $net #$rep $(grep '"mb"' gpurun_out/pab.log | cut -c1-120)"
done; done; done
