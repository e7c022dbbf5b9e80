cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python -u tools/exp/engine_determinism2.py 262144 > gpurun_out/d2.log 2>&1; echo "d2 rc=$?"; grep inputs gpurun_out/d2.log | cut -c1-200
timeout -k 10 200 python -u tools/exp/learn_determinism2.py 262144 > gpurun_out/l2.log 2>&1; echo "l2 rc=$?"; grep sync gpurun_out/l2.log
timeout -k 10 300 python -u tools/exp/xcd_check.py 262144 0,1,0,1 > gpurun_out/x.log 2>&1; echo "x rc=$?"; grep mode gpurun_out/x.log
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_stack_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/engine_tests.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/engine_tests.log
