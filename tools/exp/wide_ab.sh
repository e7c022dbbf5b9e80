#!/bin/bash
# GPU box: wide tests, then prl_ppo_wide_grad at C5's shape (tools/wide_bench.py) for the
# libraries named (PRL_HIP_LIB=...; X=1 = in-tree), 3 interleaved rounds
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_wide_gpu.py tests/test_rnd_learn_gpu.py > gpurun_out/wab_tests.log 2>&1 || { tail -30 gpurun_out/wab_tests.log; exit 1; }
tail -1 gpurun_out/wab_tests.log
for rep in 1 2 3; do for cfg in "$@"; do
  env $cfg timeout -k 10 120 python -u tools/wide_bench.py > gpurun_out/wb.log 2>&1 || { tail -3 gpurun_out/wb.log; exit 1; }
  echo "$cfg #$rep $(tail -1 gpurun_out/wb.log | cut -c60-400)"
done; done
