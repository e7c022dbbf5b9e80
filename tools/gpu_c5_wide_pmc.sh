#!/bin/bash
# GPU box: HBM bytes of C5's wide-step launches (tile kernel, dW0 + fold, dW0's fold, flat AdamW)
# from separate rocprofv3 --pmc passes (FETCH_SIZE, then WRITE_SIZE) over a short C5 bench run.
# Outputs under gpurun_out/c5pmc/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out/c5pmc"; mkdir -p "$O"
RX='ppo_wide|flat_adamw'
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" -d $O/fetch -o fetch --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" -d $O/write -o write --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline > $O/write.log 2>&1 || { tail -5 $O/write.log; exit 1; }
for k in ppo_wide_grad_kernel ppo_wide_dw0_kernel ppo_wide_reduce_kernel flat_adamw_kernel; do
  python3 tools/rocprof_summary.py pmc $O/fetch/fetch_counter_collection.csv $O/write/write_counter_collection.csv --match $k > $O/$k.json
done
cat $O/*.json
