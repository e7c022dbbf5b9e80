#!/bin/bash
# Build a libprl_hip.so variant into tools/exp/lib_<name>.so for same-box A/B runs
# (PRL_HIP_LIB=tools/exp/lib_<name>.so): this tree's objects, with ONE source recompiled —
# from git HEAD when REV=HEAD, else from the tree — with extra compiler flags.
#   build_variant_lib.sh <name> <source basename, e.g. prl_gae.hip> [extra hipcc flags...]
set -e
NAME=$1; SRC=$2; shift 2
R=$(cd "$(dirname "$0")/../.." && pwd)
C=$R/parallel-reinforcement-learning_amd/csrc
T=$(mktemp -d)
mkdir -p $T/include $T/a/b
cp $C/prl_common.h $T/a/b/; cp $R/include/prl_abi.h $T/include/
if [ "${REV:-}" = HEAD ]; then git -C $R show HEAD:parallel-reinforcement-learning_amd/csrc/$SRC > $T/a/b/$SRC
else cp $C/$SRC $T/a/b/$SRC; fi
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -ffp-contract=off -fno-gpu-rdc "$@" -c $T/a/b/$SRC -o $T/v.o
OBJS=""
for o in $C/build/*.o; do [ "$(basename $o .o)" = "$(basename $SRC .hip)" ] || OBJS="$OBJS $o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/tools/exp/lib_$NAME.so $OBJS $T/v.o
rm -rf $T
