#!/bin/bash
# GPU box: C5's dW0 pass with its B operands read one K step ahead (double-buffered registers; the
# same MFMAs in the same order) — the wide-step tests, then the wide gradient step
# (tools/wide_bench.py, D 348, mb 65,536) interleaved x3 and the C5 bench line against
# tools/exp/lib_w0.so (HEAD before).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_wide_gpu.py tests/test_rnd_learn_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/dw0_tests.log 2>&1 || { echo "tests FAILED"; tail -40 gpurun_out/dw0_tests.log; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/dw0_tests.log)"
for rep in 1 2 3; do
  for cfg in "PRL_HIP_LIB=tools/exp/lib_w0.so" "PRL_X=dw0"; do
    env $cfg timeout -k 10 120 python -u tools/wide_bench.py > gpurun_out/wb.log 2>&1 || { tail -3 gpurun_out/wb.log; exit 1; }
    echo "wide $cfg #$rep $(tail -1 gpurun_out/wb.log | cut -c1-160)"
  done
done
for cfg in "PRL_HIP_LIB=tools/exp/lib_w0.so" "PRL_X=dw0"; do
  env $cfg timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-learn-fixed > gpurun_out/c5.log 2>&1 || { tail -3 gpurun_out/c5.log; exit 1; }
  echo "c5 $cfg $(grep '"metric"' gpurun_out/c5.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("learn_ms_per_1M"), d["roofline"].get("avg_launch_us"))')"
done
