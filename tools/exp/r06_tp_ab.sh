#!/bin/bash
# GPU box: the 8-wave / throughput tile's MFMA operand reads batched (dF / dW1 / dW2 / dW0, as the
# split tile's) — tests (engine / tp / stack / distributed + reference fixtures), then interleaved
# timing against tools/exp/lib_fin.so (HEAD before): the throughput form at mb 65,536 (CartPole
# C2, Pendulum C3) x2, and the 8-wave latency form at mb 512 (PRL_UPD_SPLIT=0) x2.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
K="split or reproducible or off_policy or matches_autograd or dpx or learn_c1 or reference_learn or persistent or evaluate or fixture or throughput or tp"
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py tests/test_stack_gpu.py tests/test_distributed_gpu.py tests/test_tp_learn_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "$K" > gpurun_out/tpab_tests.log 2>&1 || { echo "tests FAILED"; tail -40 gpurun_out/tpab_tests.log; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/tpab_tests.log)"
for rep in 1 2; do
  for net in cartpole pendulum; do
    for cfg in "PRL_HIP_LIB=tools/exp/lib_fin.so" "PRL_X=tpb"; do
      env $cfg PRL_UPD_PROFILE=0 timeout -k 10 180 python -u tools/engine_profile.py 1048576 65536 $net > gpurun_out/tp.log 2>&1 || { tail -3 gpurun_out/tp.log; exit 1; }
      echo "tp $net $cfg #$rep $(grep '"mb"' gpurun_out/tp.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["us_per_step"])')"
    done
  done
  for cfg in "PRL_HIP_LIB=tools/exp/lib_fin.so" "PRL_X=tpb"; do
    env $cfg PRL_UPD_SPLIT=0 PRL_UPD_PROFILE=0 timeout -k 10 120 python -u tools/engine_profile.py 262144 512 > gpurun_out/w8.log 2>&1 || { tail -3 gpurun_out/w8.log; exit 1; }
    echo "8-wave mb512 $cfg #$rep $(grep '"mb"' gpurun_out/w8.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["us_per_step"])')"
  done
done
