#!/bin/bash
# Build an A/B variant of libcosnet_hip.so with extra defines: bash tools/build_variant.sh NAME "-DX=1 ..."
set -e
NAME=$1; DEFS=$2
D=cosnet_amd/_lib/var_$NAME
mkdir -p $D
make -s -C cosnet_amd/csrc OUT=../_lib/var_$NAME/libcosnet_hip.so OBJDIR=../_lib/var_$NAME/obj FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -Wall -Wno-unused-function $DEFS" -j8
