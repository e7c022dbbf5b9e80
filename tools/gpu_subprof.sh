#!/bin/bash
# GPU box: rocprofv3 kernel-trace summaries of the bench's sub-records (C2 at mini_batch 65,536,
# C3, C5), each as its own bench.py run of that config (2 timed steps after 1 warm-up), condensed
# to <name>_kernel_stats.md + the bench line under gpurun_out/.  Stops at the first failing step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out"
step() { local name=$1 to=$2; shift 2; timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1; local rc=$?
         echo "[$name] rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$O/$name.log"; exit $rc; }; }
prof() { local name=$1; shift
  step prof_$name 420 rocprofv3 --kernel-trace --stats -d $O/prof_$name -o $name --output-format csv -- \
       python bench.py "$@" --no-cpu-baseline --no-learn-fixed --no-subconfigs --steps 2
  grep '"metric"' $O/prof_$name.log | tail -1 > $O/${name}_bench_under_rocprof.json
  python tools/rocprof_summary.py stats $O/prof_$name/${name}_kernel_stats.csv --top 25 > $O/${name}_kernel_stats.md
  rm -f $O/prof_$name/${name}_kernel_trace.csv
}
prof c2_mb65536 --config c2 --mb 65536
prof c3 --config c3
prof c5 --config c5
head -12 $O/c2_mb65536_kernel_stats.md $O/c3_kernel_stats.md $O/c5_kernel_stats.md
