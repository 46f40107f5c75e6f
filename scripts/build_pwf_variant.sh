#!/bin/bash
# Build _abx/libogbx_pwf_<name>.so: libogbx with powder.hip compiled under
# extra flags (the other objects from build/obj, built by `make`).  Run here.
# usage: scripts/build_pwf_variant.sh <name> [-DOGBX_PWF_RULE_STAMPS ...]
# (-D macros the sources do not reference are rejected: scripts/check_macros.sh)
set -eu
cd "$(dirname "$0")/.."
name=$1; shift
make -s -C ogbench_amd/csrc >/dev/null
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -w"
mkdir -p build/var
scripts/check_macros.sh ogbench_amd/csrc/powder.hip "$@"
$H $F "$@" -c ogbench_amd/csrc/powder.hip -o build/var/powder_$name.o
objs=$(ls build/obj/*.o | grep -v '/powder' | tr '\n' ' ')
mkdir -p _abx
$H --offload-arch=gfx950 -shared -fPIC -o _abx/libogbx_pwf_$name.so $objs build/var/powder_$name.o
echo _abx/libogbx_pwf_$name.so
