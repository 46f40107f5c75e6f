#!/bin/bash
# Ablation / tuning builds of the full powderworld forward (timing only; never shipped).
# OGBX_PWF_RULES bits: 1 stone, 4 sand, 8 fluid, 16 ice, 32 water, 64 fire, 128 plant, 256 velocity.
# OGBX_PWF_WAVES: waves per SIMD the register budget is sized for.
set -e
cd "$(dirname "$0")/../ogbench_amd/csrc"
mkdir -p ../../build/variants
rm -f ../../build/variants/libogbx_pwf_*.so
for v in ${VARIANTS:-"w4:" "w2:-DOGBX_PWF_WAVES=2" "w1:-DOGBX_PWF_WAVES=1"}; do
  name=${v%%:*}; flags=${v#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -shared $flags \
     common.hip powder.hip -o ../../build/variants/libogbx_pwf_$name.so &
done
wait
