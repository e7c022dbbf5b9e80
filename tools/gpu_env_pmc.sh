#!/bin/bash
# GPU box: the CartPole rollout-step kernel at 2^22 envs under rocprofv3 counter passes (one pass
# per counter group, each under its own time limit): instruction mix, VALU activity, occupancy.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/env_pmc; export TMPDIR=/tmp
O=gpurun_out/env_pmc
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1; echo "list rc=$?"
run() { local name=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" -d $O/$name -o $name --output-format csv -- python tools/kernel_bench.py --env-e 4194304 --reps 3 > $O/$name.log 2>&1; echo "$name rc=$?"; }
run mix SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS GRBM_GUI_ACTIVE
run busy SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_COUNT
run derived VALUBusy
run occ MeanOccupancyPerCU
