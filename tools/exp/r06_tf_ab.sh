#!/bin/bash
# GPU box: the next tile's trunk forward inside AdamW (split.h WB + PRE) on the in-tree library —
# engine / stack / data-parallel tests, then mb-512 step time interleaved against
# tools/exp/lib_wb.so (wave-block AdamW) and tools/exp/lib_pw.so (+ per-wave publish).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_stack_gpu.py tests/test_distributed_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "split or reproducible or off_policy or matches_autograd or dpx or learn_c1 or reference_learn or persistent" > gpurun_out/tf_tests.log 2>&1 \
  || { echo "tests FAILED"; tail -40 gpurun_out/tf_tests.log; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/tf_tests.log)"
PROF=0 tools/exp/engine_ab.sh "PRL_HIP_LIB=tools/exp/lib_wb.so" "PRL_HIP_LIB=tools/exp/lib_pw.so" "PRL_X=tf" || exit 1
PROF=1 tools/exp/engine_ab.sh "PRL_HIP_LIB=tools/exp/lib_wb.so" "PRL_HIP_LIB=tools/exp/lib_pw.so" "PRL_X=tf"
