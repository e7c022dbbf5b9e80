#!/bin/bash
# GPU box: the update-engine tests, then tools/engine_profile.py at mb 512 with the tile
# (PRL_UPD_PROFILE=1) and without it (=2: the exchange + AdamW alone).  Stops at the first failure.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_stack_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/engine_tests.log 2>&1; rc=$?
tail -3 gpurun_out/engine_tests.log; [ $rc -eq 0 ] || exit $rc
for mode in 1 2; do
  PRL_UPD_PROFILE=$mode timeout -k 10 180 python -u tools/engine_profile.py 262144 ${MBS:-512} \
    > gpurun_out/eprof$mode.log 2>&1 || { tail -5 gpurun_out/eprof$mode.log; exit 1; }
  echo "mode=$mode $(grep '"mb"' gpurun_out/eprof$mode.log)"
done
