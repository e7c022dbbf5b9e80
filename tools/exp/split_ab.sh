#!/bin/bash
# GPU box: the head-split form's variants, correctness first (engine tests under each setting),
# then engine_ab.sh's interleaved mb-512 timing.  Usage: split_ab.sh "ENV=a" "ENV=b" ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for cfg in "$@"; do
  env $cfg timeout -k 10 150 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread \
      -k "split or reproducible or off_policy or matches_autograd" > gpurun_out/split_ab_tests.log 2>&1 \
    || { echo "tests FAILED under $cfg"; tail -30 gpurun_out/split_ab_tests.log; exit 1; }
  echo "tests ok under $cfg: $(tail -1 gpurun_out/split_ab_tests.log)"
done
exec tools/exp/engine_ab.sh "$@"
