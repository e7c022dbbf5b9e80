#!/bin/bash
# GPU box: which test function of tests/test_kernels_gpu.py, run before it, makes the C5 graphed
# rollout's reward score NaN in test_wide_graphed_rollout_equals_eager_rollout (passes alone).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=tests/test_wide_gpu.py::test_wide_graphed_rollout_equals_eager_rollout
for f in $(grep -o "^def test_[a-z0-9_]*" tests/test_kernels_gpu.py | cut -c5-); do
  timeout -k 10 200 python -u -m pytest -q --timeout 100 --timeout-method thread "tests/test_kernels_gpu.py::$f" $T > gpurun_out/bis_$f.log 2>&1
  echo "$f rc=$? $(tail -1 gpurun_out/bis_$f.log)"
done
