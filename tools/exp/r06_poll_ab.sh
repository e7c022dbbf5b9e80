#!/bin/bash
# GPU box: the counter waits' polling on the final kernel (mb 512, interleaved x3): default (one
# poll in flight, s_sleep 1), PRL_UPD_SPL_POLL=1 (four polls in flight), 3 / 4 (s_sleep 4 / 8).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
PROF=0 tools/exp/engine_ab.sh "PRL_X=default" "PRL_UPD_SPL_POLL=1" "PRL_UPD_SPL_POLL=3" "PRL_UPD_SPL_POLL=4"
