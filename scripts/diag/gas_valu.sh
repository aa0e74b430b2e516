cd /root/repo
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_INSTS_SMEM"
timeout -k 10 400 bash scripts/prof_kernels.sh gas "$P1" > gpurun_out/pmc_gas64.txt 2>&1; rc=$?
grep -E "rfit" gpurun_out/pmc_gas64.txt | grep -E "INSTS_VALU|INSTS_LDS|WAVE_CYCLES"; exit $rc
