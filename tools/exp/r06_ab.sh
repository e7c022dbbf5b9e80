#!/bin/bash
# GPU box: engine + data-parallel tests on the in-tree library, then engine_ab.sh's interleaved
# mb-512 timing of the given settings (e.g. PRL_HIP_LIB=tools/exp/lib_X.so for the previous build).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_stack_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "split or reproducible or off_policy or matches_autograd or dpx or learn_c1 or reference_learn" > gpurun_out/ab_tests.log 2>&1 \
  || { echo "tests FAILED"; tail -40 gpurun_out/ab_tests.log; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/ab_tests.log)"
exec tools/exp/engine_ab.sh "$@"
