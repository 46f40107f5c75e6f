#!/bin/bash
# Build _abx/libogbx_<name>.so: libogbx with $SRC.hip (default locomaze) compiled
# from the working tree's csrc with the files $FILES (csrc-relative, default
# point_contact.h) taken from git revision <rev> (the other objects from
# build/obj), for A/B runs of a kernel change against the revision it started
# from.  usage: FILES="a.h b.h" scripts/build_rev_variant.sh <name> <rev> [-DFLAG ...]
set -eu
cd "$(dirname "$0")/.."
name=$1; rev=$2; shift 2
make -s -C ogbench_amd/csrc >/dev/null
SRC=${SRC:-locomaze}
d=build/rev_$name
rm -rf $d && mkdir -p $d/ogbench_amd $d/include
cp -r ogbench_amd/csrc $d/ogbench_amd/ && cp include/ogbx.h $d/include/
for f in ${FILES:-point_contact.h}; do git show "$rev:ogbench_amd/csrc/$f" > $d/ogbench_amd/csrc/$f; done
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -Wno-unused-function -Wno-unused-variable -Wno-bitwise-instead-of-logical"
PF=$(make -s -C ogbench_amd/csrc -p 2>/dev/null | sed -n "s/^FLAGS_$SRC := //p")
$H $F $PF "$@" -c $d/ogbench_amd/csrc/$SRC.hip -o $d/$SRC.o
objs=$(ls build/obj/*.o | grep -v "/$SRC\.o" | tr '\n' ' ')
mkdir -p _abx
$H --offload-arch=gfx950 -shared -fPIC -o _abx/libogbx_$name.so $objs $d/$SRC.o
echo _abx/libogbx_$name.so
