#!/bin/bash
# GPU box: rocprofv3 kernel trace of a short C5 bench run; the timeline of its last learn()
# (from the rollout's env-major flatten to bench.py's first re-timing sleep) condensed to
# gpurun_out/c5_learn_timeline.md.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out"
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/prof_c5tl -o c5tl --output-format csv -- \
    python bench.py --config c5 --no-cpu-baseline --no-learn-fixed --no-subconfigs --steps 1 \
    > $O/c5tl.log 2>&1 || { tail -5 $O/c5tl.log; exit 1; }
python tools/rocprof_summary.py timeline $O/prof_c5tl/c5tl_kernel_trace.csv --match flatten_wide \
    --upto spin_kernel > $O/c5_learn_timeline.md
rm -f $O/prof_c5tl/c5tl_kernel_trace.csv
head -40 $O/c5_learn_timeline.md
