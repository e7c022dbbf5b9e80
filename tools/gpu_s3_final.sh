#!/bin/bash
# GPU box: the whole GPU test suite, smoke(), then the default bench line (C2 + sub-records).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > $O/s3f_gputests.log 2>&1 || { tail -30 $O/s3f_gputests.log; exit 1; }
tail -2 $O/s3f_gputests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/s3f_smoke.log 2>&1 \
    || { tail -20 $O/s3f_smoke.log; exit 1; }
tail -2 $O/s3f_smoke.log
timeout -k 10 600 python bench.py > $O/s3f_bench.log 2>&1 || { tail -20 $O/s3f_bench.log; exit 1; }
grep '"metric"' $O/s3f_bench.log | tail -1 > $O/s3f_bench.json
python - <<'P'
import json
d = json.load(open("gpurun_out/s3f_bench.json"))
print("C2", d["value"], d["ms_per_step"], d["roofline"]["us_per_optimizer_step"], d["rollout_env_steps_per_s"])
for k, v in d["subconfigs"].items():
    print(k, v["value"], v["ms_per_step"], v.get("rollout_env_steps_per_s"), v.get("learn_ms_per_1M"))
P
