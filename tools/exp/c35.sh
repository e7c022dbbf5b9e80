cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --config c5 --steps 2 --warmup 1 > gpurun_out/c5.log 2>&1; echo "c5 rc=$?"; tail -1 gpurun_out/c5.log | cut -c1-300
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o c5 --output-format csv -- python bench.py --config c5 --steps 1 --warmup 1 > gpurun_out/prof_c5.log 2>&1; echo "prof c5 rc=$?"
python tools/rocprof_summary.py stats gpurun_out/prof_c5/c5_kernel_stats.csv --top 30 > gpurun_out/c5_kernel_stats.md; rm -f gpurun_out/prof_c5/c5_kernel_trace.csv
timeout -k 10 500 python -u bench.py --config c3 --steps 2 --warmup 1 > gpurun_out/c3.log 2>&1; echo "c3 rc=$?"; tail -1 gpurun_out/c3.log | cut -c1-300
