#!/bin/bash
# GPU box: the 8-rank bench rehearsal on this one GPU (gloo for the host exchange; the ranks'
# co-residency vote picks the 8-wave data-parallel kernel) on the final tree.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 8 --steps 2 --warmup 1 --dist-backend gloo --no-cpu-baseline > gpurun_out/bench8_gloo.log 2>&1; rc=$?
echo "[bench 8 ranks, one GPU] rc=$rc"; grep '"metric"' gpurun_out/bench8_gloo.log | tail -1 > gpurun_out/bench8.json; cut -c1-400 gpurun_out/bench8.json
exit $rc
