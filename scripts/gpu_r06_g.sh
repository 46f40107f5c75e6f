#!/bin/bash
# Round 6: whole GPU suite; lean-loop layout-independence fix, two forms
# (in-tree: restore the pre-loop values after the loop; v1: selects every
# iteration) against HEAD's; GC/HGC half-size column tables vs 32-column
# (gc32); host costs; antmaze wrapper with the bound step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
true
true
true
LIBS="ogbench_amd/libogbx.so _abx/libogbx_v1.so _abx/libogbx_head.so" ROUNDS=3 bash scripts/gpu_maze_ab.sh || exit 4
LIBS="ogbench_amd/libogbx.so _abx/libogbx_gc32.so" ROUNDS=3 WLS="gcsample hgcsample antmaze" bash scripts/gpu_lib_ab.sh || exit 5
timeout -k 10 200 python scripts/probe_gc_host.py > gpurun_out/r06_gc_host4.log 2>&1 || { tail -20 gpurun_out/r06_gc_host4.log; exit 6; }
tail -1 gpurun_out/r06_gc_host4.log
