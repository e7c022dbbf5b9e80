#!/bin/bash
# GPU box (round 6, final state after the wave-block / latency-trim work): the -m gpu suite +
# smoke, the default bench line with its rocprofv3 summary and GAE counters, the update engine's
# HBM traffic (FETCH_SIZE / WRITE_SIZE at mb 512, k 11: 5,632 optimizer steps per dispatch) and
# workgroup 0's phase marks (mb 512; throughput form at mb 65,536 for CartPole and Pendulum).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/tpmc; export TMPDIR=/tmp
tools/gpu_round.sh r06g "timeout -k 10 240 python __graft_entry__.py smoke" || exit $?
tools/gpu_benchprof.sh || exit $?
O=$GRAFT_REPO_ROOT/gpurun_out/tpmc
for C in FETCH_SIZE WRITE_SIZE; do
  PRL_UPD_PROFILE=0 timeout -s KILL 120 rocprofv3 --pmc $C -d $O/upd_$C -o p --output-format csv -- python tools/engine_profile.py 262144 512 > $O/upd_$C.log 2>&1
  rc=$?; echo "[upd $C] rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/upd_$C.log; exit $rc; }
done
python tools/rocprof_summary.py pmc $(ls $O/upd_*/p_counter_collection.csv $O/upd_*/*/p_counter_collection.csv 2>/dev/null) --match ppo_update_split_kernel > $O/update_pmc.json
echo "update_pmc: $(head -c 300 $O/update_pmc.json)"
rm -rf $O/upd_FETCH_SIZE $O/upd_WRITE_SIZE
PRL_UPD_PROFILE=1 timeout -k 10 120 python -u tools/engine_profile.py 262144 512 > gpurun_out/prof512.log 2>&1 && grep '"mb"' gpurun_out/prof512.log > gpurun_out/engine_phases_mb512.json
for net in cartpole pendulum; do
  PRL_UPD_PROFILE=1 timeout -k 10 180 python -u tools/engine_profile.py 1048576 65536 $net > gpurun_out/tp_$net.log 2>&1 && grep '"mb"' gpurun_out/tp_$net.log >> gpurun_out/tp_engine_phases.jsonl
done
echo done
