#!/bin/bash
# GPU box: which program exits with SIGSEGV under rocprofv3 --kernel-trace (round-1 verdict:
# the profiled bench crashed inside exit() after the profiler's finalisation)?
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
PKG=$PWD/parallel-reinforcement-learning_amd
run() { local name=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace -d /tmp/tp_$name -o t --output-format csv -- "$@" > gpurun_out/tp_$name.log 2>&1
  echo "[$name] rc=$?"; }
run learn_fused python tools/learn_bench.py --n 65536 --mb 512 --k 1
#run learn_graph python tools/learn_bench.py --n 65536 --mb 512 --k 1 --no-fused
#run learn_eager python tools/learn_bench.py --n 65536 --mb 512 --k 1 --no-fused --eager
run coop python -c "
import sys; sys.path.insert(0, '$PKG'); import torch, prl_native
from PPO import PPO
p = PPO(False, 4, 2, mini_batch_size=512)
eng = p._fused_engine()
S = torch.randn(4096, 4, device='cuda'); A = (torch.rand(4096, device='cuda') < 0.5).float()
z = torch.zeros(4096, device='cuda')
eng.run(S, A, z, z, z, 1); torch.cuda.synchronize(); print('coop ok')"
#run evaluate python -c "
import sys; sys.path.insert(0, '$PKG'); import torch, prl_native
from PPO import PPO
p = PPO(False, 4, 2, mini_batch_size=512)
eng = p._fused_engine()
S = torch.randn(4096, 4, device='cuda'); A = (torch.rand(4096, device='cuda') < 0.5).float()
print(eng.evaluate(p.policy_old, S, A)[0].sum().item())"
