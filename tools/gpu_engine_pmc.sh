#!/bin/bash
# GPU box: list the PMC counters, then SQ instruction-mix passes over the fused update engine
# (learn() on 2^16 synthetic CartPole transitions, mb 512, k 2 = 256 optimizer steps in one launch;
# LB_ARGS overrides learn_bench.py's arguments).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out"
timeout -s KILL 60 rocprofv3 -L > $O/pmc_list.txt 2>&1 || echo "list rc=$?"
P=1
for C in "${@}"; do
  timeout -s KILL 90 rocprofv3 --pmc $C -d $O/epmc$P -o p --output-format csv -- python tools/learn_bench.py ${LB_ARGS:---n 65536 --mb 512 --k 2} > $O/epmc$P.log 2>&1
  rc=$?; echo "[pass $P: $C] rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/epmc$P.log; exit $rc; }
  python tools/rocprof_summary.py pmc $O/epmc$P/p_counter_collection.csv --match ppo_update_kernel > $O/epmc$P.json 2>&1 || true
  P=$((P+1))
done
