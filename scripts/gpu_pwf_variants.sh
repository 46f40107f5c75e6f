#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for f in build/variants/libogbx_pwf_*.so; do
  OGBX_LIB=$f timeout -k 10 120 python scripts/probe_pwf.py 2>&1 | grep -v amdgpu.ids
  rc=${PIPESTATUS[0]}; if [ $rc -ne 0 ]; then exit $rc; fi
done
