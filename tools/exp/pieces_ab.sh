#!/bin/bash
# GPU box: the split form's clip-norm pieces (PRL_UPD_SPL_PIECES): engine + data-parallel tests
# under the default, then engine_ab.sh's interleaved mb-512 timing for the settings given.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "split or reproducible or off_policy or matches_autograd or dpx" > gpurun_out/pieces_tests.log 2>&1 \
  || { echo "tests FAILED"; tail -40 gpurun_out/pieces_tests.log; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/pieces_tests.log)"
timeout -k 10 300 python -u -m pytest tests/test_distributed_gpu.py -x -q --timeout 200 --timeout-method thread \
    -k "persistent" > gpurun_out/pieces_dist.log 2>&1 \
  || { echo "dist tests FAILED"; tail -40 gpurun_out/pieces_dist.log; exit 1; }
echo "dist tests ok: $(tail -1 gpurun_out/pieces_dist.log)"
exec tools/exp/engine_ab.sh "$@"
