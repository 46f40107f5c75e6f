bash scripts/probe_variants.sh > gpurun_out/variants.log 2>&1; rc=$?; cat gpurun_out/variants.log; [ $rc -le 1 ] || exit $rc
OGBX_LIB=build/variants/libogbx_stamps.so timeout -k 10 120 python scripts/probe_stamps.py 2>&1 | grep -v amdgpu.ids
