"""Wrap a tools/rocprof_summary.py pmc list into {"meta": {...}, "kernels": [...]} for profiles/:
the workload the counters were taken on, so bench.py scales them per unit and refuses a shape
they were not taken at.  Usage: pmc_meta.py IN.json OUT.json key=value ... (ints / floats parsed)"""
import json
import subprocess
import sys


def _val(v):
    for f in (int, float):
        try:
            return f(v)
        except ValueError:
            pass
    return v


kernels = json.load(open(sys.argv[1]))
meta = dict(kv.split("=", 1) for kv in sys.argv[3:])
meta = {k: (v if k in ("commit", "workload") else _val(v)) for k, v in meta.items()}
try:
    meta.setdefault("commit", subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True,
                                             text=True).stdout.strip() or None)
except OSError:
    pass
json.dump({"meta": meta, "kernels": kernels}, open(sys.argv[2], "w"), indent=1)
