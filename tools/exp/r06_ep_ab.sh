#!/bin/bash
# GPU box: each wave's publish split — the entries final after dW1 (W1 rows, γ1 / β1, W2) stored
# right after dW1, the rest (W0 block, γ0 / β0, output biases) at the tile's end — tests, then
# mb-512 step time interleaved x3 against tools/exp/lib_ep0.so (HEAD before).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
K="split or reproducible or off_policy or matches_autograd or dpx or learn_c1 or reference_learn or persistent or evaluate or fixture"
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py tests/test_stack_gpu.py tests/test_distributed_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "$K" > gpurun_out/ep_tests.log 2>&1 || { echo "tests FAILED"; tail -40 gpurun_out/ep_tests.log; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/ep_tests.log)"
PROF=0 tools/exp/engine_ab.sh "PRL_HIP_LIB=tools/exp/lib_ep0.so" "PRL_X=ep" || exit 1
PROF=1 tools/exp/engine_ab.sh "PRL_HIP_LIB=tools/exp/lib_ep0.so" "PRL_X=ep"
