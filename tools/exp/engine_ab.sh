#!/bin/bash
# GPU box: engine_profile at mb 512 for several env settings (e.g. PRL_HIP_LIB=tools/exp/lib_x.so,
# PRL_UPD_EARLY=0), interleaved over 3 rounds (box noise).  Usage: engine_ab.sh "ENV=a" "ENV=b" ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for rep in 1 2 3; do
  for cfg in "$@"; do
    env $cfg PRL_UPD_PROFILE=${PROF:-1} timeout -k 10 120 python -u tools/engine_profile.py 262144 512 > gpurun_out/ab.log 2>&1 || { tail -3 gpurun_out/ab.log; exit 1; }
    echo "$cfg #$rep $(grep '"mb"' gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d["phases_us"]; print(d["us_per_step"], {k: p[k] for k in list(p)[:7]})')"
  done
done
