#!/bin/bash
# GPU box: wide tests, then the rollout kernel time (rocprofv3) and C5 bench lines for the
# libraries named (PRL_HIP_LIB=...; X=1 = in-tree), interleaved
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_wide_gpu.py > gpurun_out/team_tests.log 2>&1 || { tail -30 gpurun_out/team_tests.log; exit 1; }
tail -1 gpurun_out/team_tests.log
i=0
for cfg in "$@"; do i=$((i+1))
  env $cfg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tp$i -o t --output-format csv -- python bench.py --config c5 --no-cpu-baseline --no-learn-fixed > gpurun_out/tp$i.log 2>&1 || { tail -5 gpurun_out/tp$i.log; exit 1; }
  python tools/rocprof_summary.py stats gpurun_out/tp$i/t_kernel_stats.csv --top 12 > gpurun_out/tp$i.md; rm -f gpurun_out/tp$i/t_kernel_trace.csv
  echo "$cfg $(grep -i rollout gpurun_out/tp$i.md)"
done
for rep in 1 2; do for cfg in "$@"; do
  env $cfg timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > gpurun_out/team_c5.log 2>&1 || { tail -5 gpurun_out/team_c5.log; exit 1; }
  echo "$cfg #$rep $(tail -1 gpurun_out/team_c5.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["rollout_env_steps_per_s"], d["learn_ms_per_1M"])')"
done; done
