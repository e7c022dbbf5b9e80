#!/bin/bash
# GPU box: which earlier GPU test file leaves state that makes the C5 per-step rollout's reward
# score NaN in test_wide_graphed_rollout_equals_eager_rollout (passes alone).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=tests/test_wide_gpu.py::test_wide_graphed_rollout_equals_eager_rollout
for f in test_kernels_gpu test_stack_gpu test_rnd_learn_gpu test_tp_learn_gpu test_engine_gpu test_distributed_gpu; do
  timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/$f.py $T > gpurun_out/bis_$f.log 2>&1
  echo "$f rc=$? $(tail -1 gpurun_out/bis_$f.log)"
done
