#!/bin/bash
# Build _abx/libogbx_<name>.so: libogbx with $SRC.hip (default locomaze) compiled under
# extra flags (the other objects from build/obj, built by `make`).  Run here.
# usage: scripts/build_maze_variant.sh <name> [-DFLAG ...]
# (-D macros the sources do not reference are rejected: scripts/check_macros.sh)
set -eu
cd "$(dirname "$0")/.."
name=$1; shift
make -s -C ogbench_amd/csrc >/dev/null
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -Wno-unused-function -Wno-unused-variable -Wno-bitwise-instead-of-logical"
mkdir -p build/var
SRC=${SRC:-locomaze}
scripts/check_macros.sh ogbench_amd/csrc/$SRC.hip "$@"
# the Makefile's per-file flags (FLAGS_<src>), then the variant's
PF=$(make -s -C ogbench_amd/csrc -p 2>/dev/null | sed -n "s/^FLAGS_$SRC := //p")
$H $F $PF "$@" -c ogbench_amd/csrc/$SRC.hip -o build/var/${SRC}_$name.o
objs=$(ls build/obj/*.o | grep -v "/$SRC\.o" | tr '\n' ' ')
mkdir -p _abx
$H --offload-arch=gfx950 -shared -fPIC -o _abx/libogbx_$name.so $objs build/var/${SRC}_$name.o
echo _abx/libogbx_$name.so
