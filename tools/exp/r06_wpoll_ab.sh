#!/bin/bash
# GPU box: the in-tree library (WB + the next tile's trunk forward inside AdamW) — engine / stack /
# data-parallel tests, the engine tests again with PRL_UPD_SPL_WPOLL=1 (every wave polls counter
# B itself), then mb-512 step time interleaved: lib_wb.so (WB only), in-tree, in-tree + WPOLL.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
K="split or reproducible or off_policy or matches_autograd or dpx or learn_c1 or reference_learn or persistent"
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_stack_gpu.py tests/test_distributed_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "$K" > gpurun_out/tf_tests.log 2>&1 || { echo "tests FAILED"; tail -40 gpurun_out/tf_tests.log; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/tf_tests.log)"
PRL_UPD_SPL_WPOLL=1 timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_stack_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "$K" > gpurun_out/wpoll_tests.log 2>&1 || { echo "WPOLL tests FAILED"; tail -40 gpurun_out/wpoll_tests.log; exit 1; }
echo "WPOLL tests ok: $(tail -1 gpurun_out/wpoll_tests.log)"
PROF=0 tools/exp/engine_ab.sh "PRL_HIP_LIB=tools/exp/lib_wb.so" "PRL_X=tf" "PRL_UPD_SPL_WPOLL=1" || exit 1
PROF=1 tools/exp/engine_ab.sh "PRL_HIP_LIB=tools/exp/lib_wb.so" "PRL_X=tf" "PRL_UPD_SPL_WPOLL=1"
