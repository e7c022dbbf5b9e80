#!/bin/bash
# GPU box: the team rollout test under both team widths, then the rollout kernel's time
# (rocprofv3) and C5 bench lines for PRL_WIDE_ROLLOUT_TEAM=1 (4 waves) vs 8, interleaved
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in 1 8; do
  PRL_WIDE_ROLLOUT_TEAM=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_wide_gpu.py -k "persistent_wide_rollout" > gpurun_out/t8_tests$v.log 2>&1 || { tail -30 gpurun_out/t8_tests$v.log; exit 1; }
  echo "TEAM=$v tests: $(tail -1 gpurun_out/t8_tests$v.log)"
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k flatten > gpurun_out/t8_fl.log 2>&1 || { tail -30 gpurun_out/t8_fl.log; exit 1; }
echo "flatten: $(tail -1 gpurun_out/t8_fl.log)"
for v in 1 8; do
  PRL_WIDE_ROLLOUT_TEAM=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/t8p$v -o t --output-format csv -- python bench.py --config c5 --no-cpu-baseline --no-learn-fixed > gpurun_out/t8p$v.log 2>&1 || { tail -5 gpurun_out/t8p$v.log; exit 1; }
  python tools/rocprof_summary.py stats gpurun_out/t8p$v/t_kernel_stats.csv --top 14 > gpurun_out/t8p$v.md; rm -f gpurun_out/t8p$v/t_kernel_trace.csv
  echo "TEAM=$v $(grep -i 'rollout\|flatten' gpurun_out/t8p$v.md | cut -c1-120)"
done
for rep in 1 2; do for v in 1 8; do
  PRL_WIDE_ROLLOUT_TEAM=$v timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > gpurun_out/t8_c5.log 2>&1 || { tail -5 gpurun_out/t8_c5.log; exit 1; }
  echo "TEAM=$v #$rep $(tail -1 gpurun_out/t8_c5.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["rollout_env_steps_per_s"], d["learn_ms_per_1M"])')"
done; done
