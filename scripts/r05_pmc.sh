#!/bin/bash
# Round-5 counter passes: the GAS fit kernels (C3) and the C5 combined kernel, each pass its
# own rocprofv3 run.  Output: gpurun_out/pk_gas/, gpurun_out/pk_c5/ (prof_kernels.sh)
set -u
cd "$(dirname "$0")/.."
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_INSTS_SMEM"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA"
P3="SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_LDS"
timeout -k 10 400 bash scripts/prof_kernels.sh gas "$P1" "$P2" > gpurun_out/r05_pmc_gas.txt 2>&1
rc=$?; cat gpurun_out/r05_pmc_gas.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 bash scripts/prof_kernels.sh c5 "$P3" > gpurun_out/r05_pmc_c5.txt 2>&1
rc=$?; cat gpurun_out/r05_pmc_c5.txt; exit $rc
