#!/bin/bash
# Build libprl_hip.so from git HEAD's prl_ppo_update.hip (+ this tree's other objects) into
# tools/exp/lib_head.so, for same-box A/B runs (PRL_HIP_LIB=tools/exp/lib_head.so).
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
T=$(mktemp -d)
mkdir -p $T/include $T/a/b
git -C $R show HEAD:parallel-reinforcement-learning_amd/csrc/prl_ppo_update.hip > $T/a/b/prl_ppo_update.hip
git -C $R show HEAD:parallel-reinforcement-learning_amd/csrc/prl_common.h > $T/a/b/prl_common.h
git -C $R show HEAD:include/prl_abi.h > $T/include/prl_abi.h
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -ffp-contract=off -fno-gpu-rdc -c $T/a/b/prl_ppo_update.hip -o $T/upd.o
B=$R/parallel-reinforcement-learning_amd/csrc/build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/tools/exp/lib_head.so $B/prl_abi.o $B/prl_envs.o $B/prl_buffers.o $B/prl_gae.o $B/prl_loss.o $B/prl_rnd.o $B/prl_gn.o $B/prl_update.o $T/upd.o
rm -rf $T
