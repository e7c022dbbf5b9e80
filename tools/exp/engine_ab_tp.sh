#!/bin/bash
# GPU box: engine_profile at mb 65,536 (throughput form) for CartPole and Pendulum under several
# env settings, interleaved over 2 rounds.  Usage: engine_ab_tp.sh "ENV=a" "ENV=b" ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for rep in 1 2; do
  for net in cartpole pendulum; do
    for cfg in "$@"; do
      env $cfg PRL_UPD_PROFILE=1 timeout -k 10 120 python -u tools/engine_profile.py 1048576 65536 $net > gpurun_out/abtp.log 2>&1 || { tail -3 gpurun_out/abtp.log; exit 1; }
      echo "$net $cfg #$rep $(grep '"mb"' gpurun_out/abtp.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d["phases_us"]; print(d["us_per_step"], {k: p[k] for k in list(p)[:7]})')"
    done
  done
done
