# PMC passes over the root-level histogram kernels (row vs quad).
set -e
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_hist
for K in row quad; do
  export KERNEL=$K
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS -d gpurun_out/pmc_hist/$K.a -o run --output-format csv -- python3 scripts/hist_one_mb.py
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum -d gpurun_out/pmc_hist/$K.b -o run --output-format csv -- python3 scripts/hist_one_mb.py
done
