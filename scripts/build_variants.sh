#!/bin/bash
# Diagnostic/ablation builds of libogbx (timing and counters only; never shipped).
set -e
cd "$(dirname "$0")/../ogbench_amd/csrc"
mkdir -p ../../build/variants
for v in "base:" "nonewton:-DOGBX_ABLATE_NEWTON" "stage1:-DOGBX_ABLATE_STAGES=1" "nocollide:-DOGBX_ABLATE_COLLIDE" "stats:-DOGBX_PHYS_STATS" "stamps:-DOGBX_PHYS_STAMPS"; do
  name=${v%%:*}; flags=${v#*:}
  out=../../build/variants/libogbx_$name.so
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -shared $flags \
     common.hip locomaze.hip -o $out &
done
wait
ls -la ../../build/variants
