#!/bin/bash
# GPU box: wide tests, the rollout kernel's time under rocprofv3 for the team form off / on, then
# C5 bench lines off / on (interleaved, 2 rounds)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_wide_gpu.py > gpurun_out/team_tests.log 2>&1 || { tail -30 gpurun_out/team_tests.log; exit 1; }
tail -1 gpurun_out/team_tests.log
for v in 0 1; do
  PRL_WIDE_ROLLOUT_TEAM=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tprof$v -o t --output-format csv -- python bench.py --config c5 --no-cpu-baseline --no-learn-fixed > gpurun_out/tprof$v.log 2>&1 || { tail -5 gpurun_out/tprof$v.log; exit 1; }
  python tools/rocprof_summary.py stats gpurun_out/tprof$v/t_kernel_stats.csv --top 12 > gpurun_out/tprof$v.md; rm -f gpurun_out/tprof$v/t_kernel_trace.csv
  grep -i "rollout" gpurun_out/tprof$v.md
done
for rep in 1 2; do for v in 0 1; do
  PRL_WIDE_ROLLOUT_TEAM=$v timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > gpurun_out/team_c5.log 2>&1 || { tail -5 gpurun_out/team_c5.log; exit 1; }
  echo "TEAM=$v #$rep $(tail -1 gpurun_out/team_c5.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["rollout_env_steps_per_s"], d["learn_ms_per_1M"], d.get("vector_steps_per_rollout"))')"
done; done
