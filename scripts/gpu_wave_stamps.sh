#!/bin/bash
# Per-wave duration distributions (scripts/probe_wave_stamps.py) of each
# stamp-built library in $LIBS at each N in $NS (GPU box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for lib in $LIBS; do for N in ${NS:-65536 8192}; do
  echo "== $lib"
  OGBX_LIB=$PWD/$lib timeout -k 10 120 python3 scripts/probe_wave_stamps.py $N 2>&1 | grep -v amdgpu.ids || exit 3
done; done
