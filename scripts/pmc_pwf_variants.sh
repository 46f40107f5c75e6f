#!/bin/bash
# SQ instruction counters of pwf_forward_kernel for every build/variants/libogbx_pwf_*.so on the same worlds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OGBX_LIB=build/variants/libogbx_pwf_all.so timeout -k 10 120 python scripts/probe_pwf.py > gpurun_out/probe.log 2>&1 || exit $?
for f in build/variants/libogbx_pwf_*.so; do
  v=$(basename $f .so)
  OGBX_LIB=$f timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_LDS -d gpurun_out/pmcv_$v -o run --output-format csv -- python3 scripts/probe_pwf_pmc.py > gpurun_out/pmcv_$v.log 2>&1 || exit $?
done
rm -f gpurun_out/pwf_worlds_*.pt
