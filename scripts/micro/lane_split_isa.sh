#!/bin/bash
# ISA instructions per lean stage of the two forms of scripts/micro/lane_split.hip
# (compiled with the product kernel's flags; run here, no GPU needed).
set -eu
cd "$(dirname "$0")/../.."
mkdir -p _ab/lane_split_isa && cd _ab/lane_split_isa
hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -mllvm -amdgpu-sched-strategy=max-ilp \
  ../../scripts/micro/lane_split.hip -o lane_split --save-temps 2>/dev/null
for k in k_one k_pair; do python ../../scripts/micro/isa_stage_count.py lane_split-hip-amdgcn-amd-amdhsa-gfx950.s $k; done
