#!/bin/bash
# Device-side launch floor (verdict r04 #3): scripts/micro/launch_cost.hip
# built on the box, run plain (device-paced vs host-paced spans) and under
# rocprofv3 --kernel-trace --stats (per-dispatch durations of the empty
# kernels at the maze / GC / powder grids).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/floor
export TMPDIR=/tmp
/opt/rocm/bin/hipcc -O3 -w --offload-arch=gfx950 scripts/micro/launch_cost.hip -o gpurun_out/floor/launch_cost || exit 2
timeout -k 10 120 gpurun_out/floor/launch_cost > gpurun_out/floor/launch_cost.txt 2>&1 || exit $?
cat gpurun_out/floor/launch_cost.txt
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/floor/prof -o run --output-format csv -- \
  gpurun_out/floor/launch_cost > gpurun_out/floor/launch_cost_prof.txt 2>&1 || exit $?
rm -f gpurun_out/floor/launch_cost
