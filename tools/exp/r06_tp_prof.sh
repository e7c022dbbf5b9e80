#!/bin/bash
# GPU box: the throughput form's phase split at mb 65,536 (CartPole, Pendulum), then the
# 8-rank bench rehearsal (8 ranks on this one GPU, gloo for the host exchange).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for net in cartpole pendulum; do
  timeout -k 10 180 python -u tools/engine_profile.py 1048576 65536 $net > gpurun_out/tp_$net.log 2>&1 || { tail -5 gpurun_out/tp_$net.log; exit 1; }
  grep '"mb"' gpurun_out/tp_$net.log
done
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 8 --steps 2 --warmup 1 --dist-backend gloo --no-cpu-baseline > gpurun_out/bench8_gloo.log 2>&1; rc=$?
echo "[bench 8 ranks, one GPU] rc=$rc"; grep '"metric"' gpurun_out/bench8_gloo.log | tail -1 | cut -c1-600
