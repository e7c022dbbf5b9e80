#!/bin/bash
# GPU box: the 2-rank wide-step test with and without prl_flat_adamw's counter memset
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for m in 1 0 1; do
  PRL_FA_MEMSET=$m timeout -k 10 300 python -u -m pytest tests/test_distributed_gpu.py -x -q --timeout 200 --timeout-method thread \
    -k "wide_step_equal" > gpurun_out/wide2_$m.log 2>&1; echo "memset=$m rc=$? $(tail -1 gpurun_out/wide2_$m.log)"; grep -h "AssertionError: (" gpurun_out/wide2_$m.log | head -2
done
timeout -k 10 300 python -u -m pytest tests/test_tp_learn_gpu.py tests/test_wide_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/wide2_tp.log 2>&1; echo "tp/wide rc=$? $(tail -1 gpurun_out/wide2_tp.log)"
