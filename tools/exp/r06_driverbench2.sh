#!/bin/bash
# GPU box: the driver's bench command on the final tree (python bench.py --gpus 1 --steps 20
# --warmup 5), with a heartbeat file under gpurun_out/ (bench.py prints only its final line).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/driverbench.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 30; date +%T >> gpurun_out/heartbeat.txt; done
wait $pid; rc=$?
echo "[bench 20/5] rc=$rc"; grep '"metric"' gpurun_out/driverbench.log | tail -1 > gpurun_out/driverbench.json; cut -c1-300 gpurun_out/driverbench.json
exit $rc
