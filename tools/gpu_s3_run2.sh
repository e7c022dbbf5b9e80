set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_wide_gpu.py tests/test_stack_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/s3_wide.log 2>&1 || { tail -30 $O/s3_wide.log; exit 1; }
tail -2 $O/s3_wide.log
for v in 0 1; do
  PRL_ROLLOUT_DIST_AT=$v timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-learn-fixed --no-subconfigs --steps 3 > $O/s3_c5_at$v.log 2>&1 || { tail -20 $O/s3_c5_at$v.log; exit 1; }
  grep '"metric"' $O/s3_c5_at$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('at=$v', d['value'], d['ms_per_step'], d.get('rollout_env_steps_per_s'), d.get('learn_ms_per_1M'))"
done
