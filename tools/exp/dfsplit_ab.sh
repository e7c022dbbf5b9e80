#!/bin/bash
# GPU box: dF split over the head groups (in-tree library) against HEAD before it
# (PRL_HIP_LIB=tools/exp/lib_base.so): engine / TP / distributed tests, then CartPole learn()
# per optimizer step at mb 512 and 65,536, interleaved over 3 rounds (box noise).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py tests/test_tp_learn_gpu.py tests/test_distributed_gpu.py > gpurun_out/df_tests.log 2>&1 || { tail -30 gpurun_out/df_tests.log; exit 1; }
tail -1 gpurun_out/df_tests.log
for rep in 1 2 3; do for cfg in "PRL_HIP_LIB=tools/exp/lib_base.so" "X=1"; do
  env $cfg PRL_UPD_PROFILE=0 timeout -k 10 120 python -u tools/engine_profile.py 1048576 512,65536 cartpole > gpurun_out/df.log 2>&1 || { tail -3 gpurun_out/df.log; exit 1; }
  grep '"mb"' gpurun_out/df.log | while read -r line; do echo "$cfg #$rep $(echo "$line" | cut -c1-110)"; done
done; done
env PRL_UPD_PROFILE=1 timeout -k 10 120 python -u tools/engine_profile.py 1048576 512,65536 cartpole > gpurun_out/df_phases.log 2>&1 && grep '"mb"' gpurun_out/df_phases.log
