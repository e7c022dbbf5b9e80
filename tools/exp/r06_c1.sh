#!/bin/bash
# GPU box: (1) tests on the in-tree library; (2) mb-512 step time interleaved against
# tools/exp/lib_lds.so (HEAD before the output-bias row-read batching); (3) the throughput form at
# mb 65,536 (CartPole C2 / Pendulum C3), one rep each; (4) the update engine's HBM traffic
# (FETCH_SIZE / WRITE_SIZE, engine_profile 262144 512, k 11: 5,632 optimizer steps per dispatch);
# (5) workgroup 0's phase marks at mb 512.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/tpmc; export TMPDIR=/tmp
K="split or reproducible or off_policy or matches_autograd or dpx or learn_c1 or reference_learn or persistent or evaluate or fixture or throughput"
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py tests/test_stack_gpu.py tests/test_distributed_gpu.py tests/test_tp_learn_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "$K" > gpurun_out/c1_tests.log 2>&1 || { echo "tests FAILED"; tail -40 gpurun_out/c1_tests.log; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/c1_tests.log)"
PROF=0 tools/exp/engine_ab.sh "PRL_HIP_LIB=tools/exp/lib_lds.so" "PRL_X=bias" || exit 1
for net in cartpole pendulum; do
  for cfg in "PRL_HIP_LIB=tools/exp/lib_lds.so" "PRL_X=bias"; do
    env $cfg PRL_UPD_PROFILE=0 timeout -k 10 180 python -u tools/engine_profile.py 1048576 65536 $net > gpurun_out/tp.log 2>&1 || { tail -3 gpurun_out/tp.log; exit 1; }
    echo "tp $net $cfg $(grep '"mb"' gpurun_out/tp.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["us_per_step"])')"
  done
done
O=$GRAFT_REPO_ROOT/gpurun_out/tpmc
for C in FETCH_SIZE WRITE_SIZE; do
  PRL_UPD_PROFILE=0 timeout -s KILL 120 rocprofv3 --pmc $C -d $O/upd_$C -o p --output-format csv -- python tools/engine_profile.py 262144 512 > $O/upd_$C.log 2>&1
  rc=$?; echo "[upd $C] rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/upd_$C.log; exit $rc; }
done
python tools/rocprof_summary.py pmc $(ls $O/upd_*/p_counter_collection.csv $O/upd_*/*/p_counter_collection.csv 2>/dev/null) --match ppo_update_split_kernel > $O/update_pmc.json
echo "update_pmc: $(head -c 400 $O/update_pmc.json)"
rm -rf $O/upd_FETCH_SIZE $O/upd_WRITE_SIZE
PRL_UPD_PROFILE=1 timeout -k 10 120 python -u tools/engine_profile.py 262144 512 > gpurun_out/prof512.log 2>&1 && grep '"mb"' gpurun_out/prof512.log > gpurun_out/engine_phases_mb512.json
for net in cartpole pendulum; do
  PRL_UPD_PROFILE=1 timeout -k 10 180 python -u tools/engine_profile.py 1048576 65536 $net > gpurun_out/tp_$net.log 2>&1 && grep '"mb"' gpurun_out/tp_$net.log >> gpurun_out/tp_engine_phases.jsonl
done
echo done
