#!/bin/bash
# GPU box: the split form's phase-B helpers (PRL_UPD_SPL_HELP).  Engine tests under the default
# (all free CUs as helpers), then engine_ab.sh's interleaved mb-512 timing for the settings given.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "split or reproducible or off_policy or matches_autograd or dpx" > gpurun_out/help_ab_tests.log 2>&1 \
  || { echo "tests FAILED"; tail -40 gpurun_out/help_ab_tests.log; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/help_ab_tests.log)"
exec tools/exp/engine_ab.sh "$@"
