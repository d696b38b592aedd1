set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/avail.txt 2>&1 || true
N=20000000 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc/kt -o run --output-format csv -- python3 scripts/glm_mb.py > gpurun_out/pmc/kt.log 2>&1
N=20000000 timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc/c1 -o run --output-format csv -- python3 scripts/glm_mb.py > gpurun_out/pmc/c1.log 2>&1
N=20000000 timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA -d gpurun_out/pmc/c2 -o run --output-format csv -- python3 scripts/glm_mb.py > gpurun_out/pmc/c2.log 2>&1 || true
