#!/bin/bash
# GPU-box check: gpu tests, smoke, short bench (outputs under gpurun_out/).
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > gpurun_out/gpu_tests.log 2>&1; echo "pytest rc=$?"
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps 1 --warmup 1 > gpurun_out/bench1.log 2>&1; echo "bench rc=$?"; tail -3 gpurun_out/bench1.log
