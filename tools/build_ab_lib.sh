#!/bin/bash
# Build libprl_hip.so from another git revision (for same-box A/Bs): tools/build_ab_lib.sh REV NAME
# -> tools/exp/lib_NAME.so (git-ignored; travels to the GPU box).  Run it with
# PRL_HIP_LIB=tools/exp/lib_NAME.so (the source-stamp check is skipped for an explicit library).
set -e
REV=$1; NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/prl_ab_XXXX)
git -C "$ROOT" worktree add -q --detach "$WT" "$REV"
python "$WT/parallel-reinforcement-learning_amd/csrc/build.py" > /dev/null
mkdir -p "$ROOT/tools/exp"
cp "$WT/parallel-reinforcement-learning_amd/libprl_hip.so" "$ROOT/tools/exp/lib_$NAME.so"
git -C "$ROOT" worktree remove --force "$WT"
echo "tools/exp/lib_$NAME.so from $(git -C "$ROOT" rev-parse --short "$REV")"
