#!/bin/bash
# GPU box (round 6, final tree): the -m gpu suite + smoke, then the default bench line with its
# rocprofv3 summary and GAE counters (tools/gpu_benchprof.sh).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
tools/gpu_round.sh r06h "timeout -k 10 240 python __graft_entry__.py smoke" || exit $?
tools/gpu_benchprof.sh
