#!/bin/bash
# GPU box: HBM bytes of the kernels bench.py's roofline objects name, from separate rocprofv3
# --pmc FETCH_SIZE / WRITE_SIZE runs (tools/rocprof_summary.py doubles FETCH_SIZE for gfx950):
#   update engine   tools/engine_profile.py 262144 512 (k 11: 5,632 optimizer steps per dispatch)
#   rollout step    tools/kernel_bench.py --env-e 65536 (every dispatch 65,536 env-steps from reset)
#   CartPole rollout tools/rollout_once.py 65536 (ONE cp_rollout_kernel dispatch; its env-steps printed)
# -> gpurun_out/tpmc/{update,env,cprollout}_pmc.json (+ the runs' logs)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/tpmc; export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/tpmc
pass() {   # pass NAME COUNTER LIMIT cmd...
  local name=$1 c=$2 lim=$3; shift 3
  timeout -s KILL $lim rocprofv3 --pmc $c -d $O/${name}_$c -o p --output-format csv -- "$@" > $O/${name}_$c.log 2>&1
  local rc=$?; echo "[$name $c] rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/${name}_$c.log; exit $rc; }
}
for C in FETCH_SIZE WRITE_SIZE; do
  PRL_UPD_PROFILE=0 pass upd $C 120 python tools/engine_profile.py 262144 512
  pass env $C 90 python tools/kernel_bench.py --env-e 65536 --reps 5
  pass cpr $C 90 python tools/rollout_once.py 65536
done
sum() { python tools/rocprof_summary.py pmc $(ls $O/$1_*/p_counter_collection.csv $O/$1_*/*/p_counter_collection.csv 2>/dev/null) --match $2 > $O/$3; echo "$3: $(head -c 400 $O/$3)"; }
sum upd ppo_update_split_kernel update_pmc.json
sum env rollout_step_kernel env_pmc.json
sum cpr cp_rollout_kernel cprollout_pmc.json
grep -h '"env_steps"' $O/cpr_*.log | head -2
