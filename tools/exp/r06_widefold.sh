#!/bin/bash
# GPU box: the wide step's fold past the W0 block — wide / RND-learn / 2-rank wide tests, then the
# wide step (tools/wide_bench.py) and the C5 bench, previous library vs this one, interleaved.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_wide_gpu.py tests/test_rnd_learn_gpu.py tests/test_distributed_gpu.py -x -q \
    --timeout 200 --timeout-method thread -k "not eight and not four and not persistent and not rccl and not dpx" > gpurun_out/wf_tests.log 2>&1 \
  || { echo "tests FAILED"; tail -30 gpurun_out/wf_tests.log; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/wf_tests.log)"
for rep in 1 2; do
  for cfg in "PRL_HIP_LIB=tools/exp/lib_main.so" "X=1"; do
    env $cfg timeout -k 10 120 python tools/wide_bench.py --reps 20 > gpurun_out/wf_wb.log 2>&1 || { tail -3 gpurun_out/wf_wb.log; exit 1; }
    echo "$cfg wide_bench: $(tail -1 gpurun_out/wf_wb.log | cut -c1-200)"
    env $cfg timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/wf_c5.log 2>&1 || { tail -3 gpurun_out/wf_c5.log; exit 1; }
    grep '"metric"' gpurun_out/wf_c5.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'"$cfg"' c5:", d["value"], d["learn_ms_per_1M"], d["rollout_env_steps_per_s"], d["roofline"]["avg_launch_us"], d["roofline"]["warm_launch_us"])'
  done
done
