#!/bin/bash
# GPU box: the -m gpu suite (one process, per-test time limit), then optional extra steps, each
# under its own time limit.  A test FAILURE (pytest rc 1) still runs the extra steps; a crash,
# abort or time limit (any other rc) ends the script there.
# Usage: tools/gpu_round.sh TAG ["cmd" ...]
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; shift
timeout -k 10 840 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_gputests.log 2>&1
rc=$?
tail -4 gpurun_out/${TAG}_gputests.log; grep -E "FAILED|ERROR" gpurun_out/${TAG}_gputests.log | head -20
echo "pytest rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
i=0
for c in "$@"; do
  i=$((i+1))
  timeout -k 10 300 bash -c "$c" > gpurun_out/${TAG}_step$i.log 2>&1
  r=$?; echo "[step $i rc=$r] $c"; tail -12 gpurun_out/${TAG}_step$i.log
  [ $r -eq 0 ] || exit $r
done
exit $rc
