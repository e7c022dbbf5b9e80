#!/bin/bash
# GPU box (round 6): the -m gpu suite + smoke, then the default bench line with its rocprofv3
# summary and GAE counters (tools/gpu_benchprof.sh), then C5 standalone under rocprofv3 stats.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
tools/gpu_round.sh r06f "timeout -k 10 240 python __graft_entry__.py smoke" || exit $?
tools/gpu_benchprof.sh || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o c5 --output-format csv -- python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c5.log 2>&1; rc=$?
echo "[prof_c5] rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/prof_c5.log; exit $rc; }
python tools/rocprof_summary.py stats gpurun_out/prof_c5/c5_kernel_stats.csv --top 30 > gpurun_out/c5_kernel_stats.md
rm -f gpurun_out/prof_c5/c5_kernel_trace.csv
grep '"metric"' gpurun_out/prof_c5.log | tail -1 > gpurun_out/c5_under_rocprof.json
