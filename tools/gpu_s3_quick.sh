#!/bin/bash
# GPU box: the rollout / wide-net GPU tests and smoke() (quick validation of the captured step).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_stack_gpu.py tests/test_wide_gpu.py tests/test_kernels_gpu.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > $O/s3q_tests.log 2>&1 || { tail -30 $O/s3q_tests.log; exit 1; }
tail -2 $O/s3q_tests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/s3q_smoke.log 2>&1 \
    || { tail -20 $O/s3q_smoke.log; exit 1; }
tail -2 $O/s3q_smoke.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > $O/s3q_all.log 2>&1 || { tail -30 $O/s3q_all.log; exit 1; }
tail -2 $O/s3q_all.log
