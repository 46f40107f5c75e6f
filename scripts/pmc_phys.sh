export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_SMEM -d gpurun_out/pmc_phys1 -o run --output-format csv -- python3 scripts/probe_phys_pmc.py > gpurun_out/pmc_phys1.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_INSTS_BRANCH -d gpurun_out/pmc_phys2 -o run --output-format csv -- python3 scripts/probe_phys_pmc.py > gpurun_out/pmc_phys2.log 2>&1
echo rc2=$?
