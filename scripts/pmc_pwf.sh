#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_LDS -d gpurun_out/pmc_pwf1 -o run --output-format csv -- python3 scripts/probe_pwf_pmc.py > gpurun_out/pmc_pwf1.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_BUSY_CYCLES SQ_INSTS_FLAT -d gpurun_out/pmc_pwf2 -o run --output-format csv -- python3 scripts/probe_pwf_pmc.py > gpurun_out/pmc_pwf2.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc_pwf0 -o run --output-format csv -- python3 scripts/probe_pwf_pmc.py > gpurun_out/pmc_pwf0.log 2>&1
