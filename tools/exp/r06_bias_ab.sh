#!/bin/bash
# GPU box: the output-bias row sums' 16 LDS reads in flight together (split tile: wave 1; the
# 8-wave / throughput tile: wave NW - 1) — tests, then interleaved timing against
# tools/exp/lib_lds.so (HEAD before): mb 512 (split form), and the throughput form at mb 65,536
# for CartPole (C2) and Pendulum (C3).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
K="split or reproducible or off_policy or matches_autograd or dpx or learn_c1 or reference_learn or persistent or evaluate or fixture or throughput"
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py tests/test_stack_gpu.py tests/test_distributed_gpu.py tests/test_tp_learn_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "$K" > gpurun_out/bias_tests.log 2>&1 || { echo "tests FAILED"; tail -40 gpurun_out/bias_tests.log; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/bias_tests.log)"
PROF=0 tools/exp/engine_ab.sh "PRL_HIP_LIB=tools/exp/lib_lds.so" "PRL_X=bias" || exit 1
for rep in 1 2; do
  for net in cartpole pendulum; do
    for cfg in "PRL_HIP_LIB=tools/exp/lib_lds.so" "PRL_X=bias"; do
      env $cfg PRL_UPD_PROFILE=0 timeout -k 10 180 python -u tools/engine_profile.py 1048576 65536 $net > gpurun_out/tp.log 2>&1 || { tail -3 gpurun_out/tp.log; exit 1; }
      echo "$net $cfg #$rep $(grep '"mb"' gpurun_out/tp.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["us_per_step"])')"
    done
  done
done
