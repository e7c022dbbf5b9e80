#!/bin/bash
# GPU box: SQ counter passes (one per argument, each its own run under its own limit) over the C5
# bench's persistent team rollout (wide_rollout4_kernel), condensed to gpurun_out/rpmc<N>.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out"
P=1
for C in "${@}"; do
  timeout -s KILL 200 rocprofv3 --pmc $C -d $O/rpmc$P -o p --output-format csv -- python bench.py --config c5 --no-cpu-baseline --no-learn-fixed --steps 1 --warmup 1 > $O/rpmc$P.log 2>&1
  rc=$?; echo "[pass $P: $C] rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/rpmc$P.log; exit $rc; }
  python tools/rocprof_summary.py pmc $O/rpmc$P/p_counter_collection.csv --match wide_rollout4 > $O/rpmc$P.json 2>&1 || true
  rm -f $O/rpmc$P/p_counter_collection.csv
  P=$((P+1))
done
