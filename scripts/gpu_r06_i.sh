#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OGBX_LIB=$PWD/_abx/libogbx_stages.so timeout -k 10 200 python scripts/probe_window_clock.py > gpurun_out/r06_window_clock.log 2>&1 || { tail -20 gpurun_out/r06_window_clock.log; exit 2; }
tail -1 gpurun_out/r06_window_clock.log
