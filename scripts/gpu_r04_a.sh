export TMPDIR=/tmp
OGBX_WRITE_PINS=gpurun_out/pins.json timeout -k 10 500 python -u -m pytest tests/test_locomaze_gpu.py tests/test_contact_pin_gpu.py tests/test_shard_boundary_gpu.py tests/test_gc_gpu.py tests/test_periodic_gpu.py tests/test_antmaze_gpu.py tests/test_stream_pin_gpu.py tests/test_hgc_gpu.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu2.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" gpurun_out/pytest_gpu2.log | tail -15; cat gpurun_out/pins.json; echo pytest rc=$rc
[ $rc -le 1 ] || exit $rc
ROUNDS=2 bash scripts/gpu_maze_ab.sh
