cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for d in 0,0 50,0 100,0 0,50 0,100 100,100 150,150; do
  for mode in 1 2; do
    PRL_UPD_POLL_DELAY=$d PRL_UPD_PROFILE=$mode timeout -k 10 120 python -u tools/engine_profile.py 262144 512 > gpurun_out/sw.log 2>&1 || { tail -3 gpurun_out/sw.log; exit 1; }
    echo "delay=$d mode=$mode $(grep '"mb"' gpurun_out/sw.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d["phases_us"]; print(d["us_per_step"], {k: p[k] for k in list(p)[:7]})')"
  done
done
