#!/bin/bash
# GPU box: group 1 skips the trunk forward (PRL_HIP_LIB=tools/exp/lib_trunk.so) and, in-tree,
# also Pendulum's loss hand-off, against HEAD before both (lib_base.so): engine / TP /
# distributed tests, then learn() per optimizer step at mb 512 and 65,536, 3 interleaved rounds.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py tests/test_tp_learn_gpu.py tests/test_distributed_gpu.py > gpurun_out/fw_tests.log 2>&1 || { tail -30 gpurun_out/fw_tests.log; exit 1; }
tail -1 gpurun_out/fw_tests.log
for rep in 1 2 3; do for cfg in "PRL_HIP_LIB=tools/exp/lib_base.so" "PRL_HIP_LIB=tools/exp/lib_trunk.so" "X=1"; do for net in cartpole pendulum; do
  env $cfg PRL_UPD_PROFILE=0 timeout -k 10 120 python -u tools/engine_profile.py 1048576 512,65536 $net > gpurun_out/fw.log 2>&1 || { tail -3 gpurun_out/fw.log; exit 1; }
  grep '"mb"' gpurun_out/fw.log | while read -r line; do echo "$cfg #$rep $(echo "$line" | cut -c1-100)"; done
done; done; done
