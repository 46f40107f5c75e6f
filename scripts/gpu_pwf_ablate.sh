#!/bin/bash
# Powder medium forward ablations (GPU box): bench each _ab/libogbx_pwf_*.so
# (scripts/build_pwf_variant.sh), then the per-env phase stamps
# (_ab/libogbx_pwfst.so, scripts/probe_pwf_stamps.py).  Tuning only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_pwf_variant_bench.sh || exit $?
if [ -f _ab/libogbx_pwfst.so ]; then
  OGBX_LIB=_ab/libogbx_pwfst.so timeout -k 10 200 python scripts/probe_pwf_stamps.py > gpurun_out/pwf_stamps.log 2>&1
  rc=$?; tail -3 gpurun_out/pwf_stamps.log; exit $rc
fi
