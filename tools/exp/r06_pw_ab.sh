#!/bin/bash
# GPU box: per-wave publish (no barrier before the publish) — engine / stack / data-parallel tests on the
# in-tree library, then mb-512 step time, interleaved against tools/exp/lib_wb.so (HEAD before).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_stack_gpu.py tests/test_distributed_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "split or reproducible or off_policy or matches_autograd or dpx or learn_c1 or reference_learn or persistent" > gpurun_out/pw_tests.log 2>&1 \
  || { echo "tests FAILED"; tail -40 gpurun_out/pw_tests.log; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/pw_tests.log)"
PROF=0 tools/exp/engine_ab.sh "PRL_HIP_LIB=tools/exp/lib_wb.so" "PRL_X=pw" || exit 1
PROF=1 tools/exp/engine_ab.sh "PRL_HIP_LIB=tools/exp/lib_wb.so" "PRL_X=pw"
