#!/bin/bash
# GPU box: the full tests/test_kernels_gpu.py, then the C5 graphed-rollout NaN diagnostic
# (tools/diag_graph_nan_test.py) in the same process.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q -s --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tools/diag_graph_nan_test.py > gpurun_out/bis_diag.log 2>&1
echo "rc=$?"; grep -E "^k=|^capture|^replay|^it0|^saved|passed|failed" gpurun_out/bis_diag.log | head -12
