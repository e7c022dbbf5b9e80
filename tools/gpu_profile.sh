#!/bin/bash
# GPU-box: numerics diagnostic, gpu tests, kernel micro-bench, rocprofv3 kernel trace and
# separate PMC passes.  Stops at the first step that dies by signal / timeout (GPU trouble).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O="$GRAFT_REPO_ROOT/gpurun_out"
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"
  if [ $rc -ge 124 ] && [ $rc -ne 255 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step diag 300 python tools/diag_numerics.py
step gpu_tests 900 python -m pytest tests -m gpu -q -rf
tail -4 "$O/gpu_tests.log"
step kb 400 python tools/kernel_bench.py
grep kernel "$O/kb.log"
step prof_kb 400 rocprofv3 --kernel-trace --stats -d "$O/prof_kb" -o kb --output-format csv -- python tools/kernel_bench.py --quick
step pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o fetch --output-format csv -- python tools/kernel_bench.py --quick --reps 3
step pmc_write 400 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o write --output-format csv -- python tools/kernel_bench.py --quick --reps 3
find "$O" -name "*.csv" | head -20
