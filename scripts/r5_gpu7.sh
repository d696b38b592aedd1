#!/bin/bash
# round 5: why the fused wide Gram runs at 1/4 of its MFMA bound and the fused
# DL step kernel at 1/6 -- timings + PMC passes (kernel-trace-free)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/wide_gram_mb.py > gpurun_out/r5_wide_gram_mb.txt 2>&1 || { tail -20 gpurun_out/r5_wide_gram_mb.txt; exit 1; }
cat gpurun_out/r5_wide_gram_mb.txt
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmc_wide1 -o p -- python3 scripts/wide_gram_mb.py 3000000 > gpurun_out/r5_pmc_wide1.log 2>&1 || { tail -20 gpurun_out/r5_pmc_wide1.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum \
  --output-format csv -d gpurun_out/pmc_wide2 -o p -- python3 scripts/wide_gram_mb.py 3000000 > gpurun_out/r5_pmc_wide2.log 2>&1 || { tail -20 gpurun_out/r5_pmc_wide2.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmc_dl1 -o p -- python3 bench.py --algo dl --rows 2000000 --batch 1024 --steps 50 --warmup 5 > gpurun_out/r5_pmc_dl1.log 2>&1 || { tail -20 gpurun_out/r5_pmc_dl1.log; exit 1; }
find gpurun_out/pmc_wide1 gpurun_out/pmc_wide2 gpurun_out/pmc_dl1 -name "*.csv" | head
