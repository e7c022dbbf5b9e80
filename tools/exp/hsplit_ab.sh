#!/bin/bash
# GPU box: the three-head net's third head on head group 1 (in-tree library) against group 0
# (PRL_HIP_LIB=tools/exp/lib_base.so): engine / TP tests, then Pendulum learn() per optimizer
# step at mb 65,536 (C3's minibatch) and 512, interleaved over 3 rounds (box noise).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py tests/test_tp_learn_gpu.py > gpurun_out/hs_tests.log 2>&1 || { tail -30 gpurun_out/hs_tests.log; exit 1; }
tail -1 gpurun_out/hs_tests.log
for rep in 1 2 3; do for cfg in "PRL_HIP_LIB=tools/exp/lib_base.so" "X=1"; do for mb in 65536 512; do
  env $cfg PRL_UPD_PROFILE=0 timeout -k 10 120 python -u tools/engine_profile.py 1048576 $mb pendulum > gpurun_out/hs.log 2>&1 || { tail -3 gpurun_out/hs.log; exit 1; }
  echo "$cfg mb $mb #$rep $(grep '"mb"' gpurun_out/hs.log | cut -c1-140)"
done; done; done
