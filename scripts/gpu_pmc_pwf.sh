#!/bin/bash
# Issue-side counters of pwf_step_kernel (powderworld medium) in the bench setting.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--workload ${WL:-powder-medium} --steps 150 --warmup 30 --no-cpu-baseline --no-extras"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES \
  -d gpurun_out/pmc_pwf_sq -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_pwf_sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT \
  -d gpurun_out/pmc_pwf_sq2 -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_pwf_sq2.log 2>&1 || exit $?
