#!/bin/bash
# GPU-box quick loop: gpu tests + kernel micro-bench (+ optional extra command in $1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 700 python -m pytest tests -m gpu -q -rf > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/gpu_tests.log
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 300 python tools/kernel_bench.py > gpurun_out/kb.log 2>&1; rc=$?; echo "kb rc=$rc"; grep kernel gpurun_out/kb.log
if [ $rc -ge 124 ]; then exit $rc; fi
if [ -n "$1" ]; then eval "$1"; fi
