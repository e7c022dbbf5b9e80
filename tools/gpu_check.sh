#!/bin/bash
# GPU-box check: gpu tests, smoke, short bench (outputs under gpurun_out/).
# Every GPU step has its own time limit; the script stops at the first failing step.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step pytest timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x ${PYTEST_ARGS} \
  > gpurun_out/gpu_tests.log 2>&1
tail -3 gpurun_out/gpu_tests.log
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
tail -2 gpurun_out/smoke.log
step bench timeout -k 10 600 python bench.py --steps 1 --warmup 1 > gpurun_out/bench1.log 2>&1
tail -3 gpurun_out/bench1.log
