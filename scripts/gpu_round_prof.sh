set -u
timeout -k 10 300 python -m pytest tests/test_eval_gpu.py -x -q > gpurun_out/eval_tests.log 2>&1; rc=$?; tail -4 gpurun_out/eval_tests.log; [ $rc -eq 0 ] || exit $rc
WL=powder KERNEL=pw_step_kernel STEPS=600 bash scripts/gpu_prof.sh || exit $?
WL=pointmaze KERNEL=maze_step_kernel STEPS=300 bash scripts/gpu_prof.sh || exit $?
WL=gcsample KERNEL=gc_sample_kernel STEPS=300 bash scripts/gpu_prof.sh || exit $?
