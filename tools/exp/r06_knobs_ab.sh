#!/bin/bash
# GPU box: the split engine's runtime knobs re-measured on the final kernel (mb 512, interleaved
# x3): phase B's trunk / loss quad weight (PRL_UPD_SPL_TW4, default 8), the counter waits'
# s_sleep (PRL_UPD_SPL_POLL, default 0 = s_sleep 1), phase B's threads per quad (PRL_UPD_SPL_FILL).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
PROF=0 tools/exp/engine_ab.sh "PRL_X=default" "PRL_UPD_SPL_TW4=6" "PRL_UPD_SPL_TW4=10" "PRL_UPD_SPL_POLL=2" "PRL_UPD_SPL_FILL=0"
