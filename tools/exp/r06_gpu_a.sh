#!/bin/bash
# GPU box (round 6): the 8-rank tests, the changed GPU tests, then the split engine's per-step
# time against the number of tile groups (mb 64 .. 2048: G = 2 mb / 16 workgroups).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
run() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "[$name] rc=$rc $(tail -1 gpurun_out/$name.log)"; return $rc; }
run t_stack 300 python -u -m pytest tests/test_stack_gpu.py -x -q --timeout 200 --timeout-method thread -k "persistent_rollout" || exit 1
run t_wide 300 python -u -m pytest tests/test_wide_gpu.py -x -q --timeout 200 --timeout-method thread -k "flat_adamw" || exit 1
run t_eight 900 python -u -m pytest tests/test_distributed_gpu.py -x -v --timeout 400 --timeout-method thread -k "eight" || exit 1
for mb in 64 128 256 512 1024 2048; do
  run prof_mb$mb 120 python -u tools/engine_profile.py 262144 $mb || exit 1
  grep '"mb"' gpurun_out/prof_mb$mb.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d["phases_us"]; print(d["mb"], d["us_per_step"], {k: p[k] for k in list(p)[:7]})'
done
