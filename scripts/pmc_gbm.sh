# PMC passes over the GBM tree kernels at 100M x 100 (3 trees): HBM bytes,
# L2 hit rate, LDS / VALU / wait counters per kernel.  Summaries ->
# gpurun_out/pmc_gbm/summary.txt
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_gbm
R=${ROWS:-100000000}
B="python3 bench.py --rows $R --steps 3 --warmup 1 --no-glm"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_gbm/a -o run --output-format csv -- $B > gpurun_out/pmc_gbm/a.log 2>&1
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_gbm/b -o run --output-format csv -- $B > gpurun_out/pmc_gbm/b.log 2>&1 || true
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_VMEM_RD -d gpurun_out/pmc_gbm/c -o run --output-format csv -- $B > gpurun_out/pmc_gbm/c.log 2>&1
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE -d gpurun_out/pmc_gbm/d -o run --output-format csv -- $B > gpurun_out/pmc_gbm/d.log 2>&1 || true
python3 scripts/pmc_summary.py gpurun_out/pmc_gbm > gpurun_out/pmc_gbm/summary.txt
find gpurun_out/pmc_gbm -name '*.csv' -size +20M -delete
cat gpurun_out/pmc_gbm/summary.txt
ROWS=12500000 bash scripts/prof_gbm_rows.sh
ROWS=100000000 bash scripts/prof_gbm_rows.sh
