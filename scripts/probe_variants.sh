#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in base nonewton stage1 nocollide stats; do
  OGBX_LIB=build/variants/libogbx_$v.so timeout -k 10 120 python scripts/probe_locomaze.py 2>&1 | grep -v amdgpu.ids
  rc=$?; if [ $rc -gt 1 ]; then exit $rc; fi
done
