#!/bin/bash
# GPU box: the C5 bench at the round-5 sub-record's timing (2 steps after 1 warm-up) and at this
# round's (5 after 2), back to back on one box: is the driver's round-5 C5 gap the short timing?
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for sw in "2 1" "5 2" "2 1"; do
  set -- $sw
  timeout -k 10 300 python bench.py --config c5 --steps $1 --warmup $2 --no-cpu-baseline > gpurun_out/c5warm_$1_$2.log 2>&1 || { echo "c5 $sw failed"; tail -5 gpurun_out/c5warm_$1_$2.log; exit 1; }
  grep '"metric"' gpurun_out/c5warm_$1_$2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("steps %d warmup %d:" % (d["steps"], d["warmup"]), d["value"], d["rollout_env_steps_per_s"], d["learn_ms_per_1M"], d["transitions_per_step"])'
done
