#!/bin/bash
# GPU-box loop for the update engine: engine/stack parity tests, then the per-phase profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_engine_gpu.py tests/test_stack_gpu.py ${PYTEST_ARGS} > gpurun_out/engine_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAIL|Error" gpurun_out/engine_tests.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/engine_profile.py > gpurun_out/engine_profile.log 2>&1; rc=$?
echo "profile rc=$rc"; cat gpurun_out/engine_profile.log | tail -5
exit $rc
