#!/bin/bash
# GPU box: PRL_UPD_SPL_DIRECT=1 (dW1 stored from the MFMA accumulators into the partial mid-tile,
# the per-wave publish skipping those quads) — engine tests under it, then mb-512 step time
# interleaved against the default (in-tree library, HEAD).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
K="split or reproducible or off_policy or matches_autograd or dpx or learn_c1 or reference_learn or persistent"
PRL_UPD_SPL_DIRECT=1 timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_stack_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "$K" > gpurun_out/direct_tests.log 2>&1 || { echo "DIRECT tests FAILED"; tail -40 gpurun_out/direct_tests.log; exit 1; }
echo "DIRECT tests ok: $(tail -1 gpurun_out/direct_tests.log)"
PROF=0 tools/exp/engine_ab.sh "PRL_X=default" "PRL_UPD_SPL_DIRECT=1" || exit 1
PROF=1 tools/exp/engine_ab.sh "PRL_X=default" "PRL_UPD_SPL_DIRECT=1"
