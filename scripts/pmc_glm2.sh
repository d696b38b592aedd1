# PMC passes over the GLM IRLS pass (bench.py --algo glm, 100M x 100, 5 iterations).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_glm
B="python3 bench.py --algo glm --steps 4 --warmup 1"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_glm/a -o run --output-format csv -- $B > gpurun_out/pmc_glm/a.log 2>&1
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA -d gpurun_out/pmc_glm/c -o run --output-format csv -- $B > gpurun_out/pmc_glm/c.log 2>&1
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_SALU -d gpurun_out/pmc_glm/d -o run --output-format csv -- $B > gpurun_out/pmc_glm/d.log 2>&1 || true
python3 scripts/pmc_summary.py gpurun_out/pmc_glm > gpurun_out/pmc_glm/summary.txt
find gpurun_out/pmc_glm -name '*.csv' -size +20M -delete
head -20 gpurun_out/pmc_glm/summary.txt
