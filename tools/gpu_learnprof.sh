#!/bin/bash
# learn() timing + a rocprofv3 kernel trace of a short learn (k=1, 32K transitions).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out"
timeout -k 10 300 python tools/learn_bench.py > $O/lb.log 2>&1; rc=$?; echo "lb rc=$rc"; tail -1 $O/lb.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python tools/learn_bench.py --mb 65536 > $O/lb2.log 2>&1; rc=$?; echo "lb2 rc=$rc"; tail -1 $O/lb2.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_learn -o learn --output-format csv -- python tools/learn_bench.py --n 32768 --k 1 > $O/prof_learn.log 2>&1; echo "prof rc=$?"
