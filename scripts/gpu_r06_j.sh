#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OGBX_LIB=$PWD/_abx/libogbx_masks.so timeout -k 10 200 python scripts/probe_mask_trace.py > gpurun_out/r06_mask_trace.log 2>&1 || { tail -20 gpurun_out/r06_mask_trace.log; exit 2; }
tail -1 gpurun_out/r06_mask_trace.log
