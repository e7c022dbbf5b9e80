#!/bin/bash
# GPU box (round 6, final): r06_full.sh (suite + smoke, bench + rocprofv3 + GAE counters, C5 under
# rocprofv3), then C5's wide-step counters (tools/gpu_c5_wide_pmc.sh).
cd "$GRAFT_REPO_ROOT"
tools/exp/r06_full.sh || exit $?
tools/gpu_c5_wide_pmc.sh > gpurun_out/c5pmc.log 2>&1; rc=$?; echo "[c5pmc] rc=$rc"; exit $rc
