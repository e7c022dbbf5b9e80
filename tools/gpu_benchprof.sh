#!/bin/bash
# GPU box: default bench line, the rocprofv3 kernel-trace summary of the SAME command, and the
# GAE scan's HBM traffic (separate --pmc passes for FETCH_SIZE and WRITE_SIZE) at the bench's
# transition count.  Stops at the first failing step.  Outputs under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out"
step() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
         echo "[$name] rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$O/$name.log"; exit $rc; }; }
BENCH="bench.py ${BENCH_ARGS:-}"
step bench 600 python $BENCH --dump-gae /tmp/gae_inputs.pt
tail -1 $O/bench.log
N=$(python -c "import torch; print(torch.load('/tmp/gae_inputs.pt', weights_only=True)['V'].numel())")
step prof_bench 900 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o bench --output-format csv -- python $BENCH --no-cpu-baseline --no-learn-fixed --no-subconfigs
grep '"metric"' $O/prof_bench.log | tail -1 > $O/bench_under_rocprof.json
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o fetch --output-format csv -- python tools/kernel_bench.py --gae-file /tmp/gae_inputs.pt --reps 3
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o write --output-format csv -- python tools/kernel_bench.py --gae-file /tmp/gae_inputs.pt --reps 3
# condense on the box (the raw kernel trace of a full bench run is far above gpurun's pull limit)
python tools/rocprof_summary.py stats $O/prof_bench/bench_kernel_stats.csv --top 40 > $O/bench_kernel_stats.md
python tools/rocprof_summary.py pmc $O/pmc_fetch/fetch_counter_collection.csv $O/pmc_write/write_counter_collection.csv --match gae_kernel --n $N > $O/gae_pmc.json
python tools/rocprof_summary.py trace $O/prof_bench/bench_kernel_trace.csv --match gae_kernel > $O/gae_trace.json
# the update engine's launches of the timed steps (bench.py's default --steps 3 after 1 warm-up)
python tools/rocprof_summary.py trace $O/prof_bench/bench_kernel_trace.csv --match ${UPD_KERNEL:-ppo_update_split_kernel} --last 3 > $O/update_trace.json
python tools/rocprof_summary.py trace $O/prof_bench/bench_kernel_trace.csv --match rollout_step_kernel > $O/env_trace.json
python tools/rocprof_summary.py trace $O/prof_bench/bench_kernel_trace.csv --match cp_rollout_kernel > $O/cp_rollout_trace.json
rm -f $O/prof_bench/bench_kernel_trace.csv
cat $O/gae_pmc.json $O/gae_trace.json $O/update_trace.json $O/cp_rollout_trace.json
