cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_stack_gpu.py tests/test_rnd_learn_gpu.py -m gpu -x -q -k "rnd or RND" --timeout 120 --timeout-method thread > gpurun_out/rt.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/rt.log
RND_D=348 timeout -k 10 300 python -u tools/rnd_bench.py 1000 1001 323584 1048576 > gpurun_out/rnd.log 2>&1; grep fast gpurun_out/rnd.log
RND_D=4 timeout -k 10 300 python -u tools/rnd_bench.py 1000 70001 > gpurun_out/rnd4.log 2>&1; grep fast gpurun_out/rnd4.log
