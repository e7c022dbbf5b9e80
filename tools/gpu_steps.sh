#!/bin/bash
# GPU box: run each step under its own time limit, stop at the first step that fails (a crash,
# abort, time limit or test failure ends the script there: nothing more touches the GPU).
# Usage: tools/gpu_steps.sh TAG SECONDS "cmd" [SECONDS "cmd" ...]
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; shift
i=0
while [ $# -ge 2 ]; do
  lim=$1; c=$2; shift 2
  i=$((i+1))
  timeout -k 10 "$lim" bash -c "$c" > gpurun_out/${TAG}_step$i.log 2>&1
  r=$?; echo "[step $i rc=$r] $c"; tail -15 gpurun_out/${TAG}_step$i.log
  [ $r -eq 0 ] || exit $r
done
