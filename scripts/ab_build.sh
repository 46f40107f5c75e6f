#!/bin/bash
# A/B builds of libogbx (diagnostic only, never shipped): each argument is
# name:flags; outputs _variants/libogbx_<name>.so.
set -e
cd "$(dirname "$0")/../ogbench_amd/csrc"
mkdir -p ../../_variants
for v in "$@"; do
  name=${v%%:*}; flags=${v#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -shared $flags \
     common.hip locomaze.hip gcsample.hip powder.hip eval.hip loader.hip comm.hip -o ../../_variants/libogbx_$name.so &
done
wait
ls ../../_variants
