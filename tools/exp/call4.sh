cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1; rc=$?; tail -1 gpurun_out/gputest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo smoke rc=$rc; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_benchprof.sh > gpurun_out/benchprof.out 2>&1; rc=$?; grep "rc=" gpurun_out/benchprof.out; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_subprof.sh > gpurun_out/subprof.out 2>&1; rc=$?; grep "rc=" gpurun_out/subprof.out; exit $rc
