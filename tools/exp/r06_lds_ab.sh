#!/bin/bash
# GPU box: dF / dW1 operand reads batched (one LDS round trip each instead of one per MFMA pair),
# on the in-tree
# library — the engine / stack / data-parallel tests and the reference learn() fixtures, then
# mb-512 step time interleaved against tools/exp/lib_loss.so (HEAD before).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
K="split or reproducible or off_policy or matches_autograd or dpx or learn_c1 or reference_learn or persistent or evaluate or fixture or throughput"
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py tests/test_stack_gpu.py tests/test_distributed_gpu.py tests/test_tp_learn_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "$K" > gpurun_out/lds_tests.log 2>&1 || { echo "tests FAILED"; tail -40 gpurun_out/lds_tests.log; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/lds_tests.log)"
PROF=0 tools/exp/engine_ab.sh "PRL_HIP_LIB=tools/exp/lib_loss.so" "PRL_X=lds" || exit 1
PROF=1 tools/exp/engine_ab.sh "PRL_HIP_LIB=tools/exp/lib_loss.so" "PRL_X=lds"
