# LDS bank-conflict / VALU survey of the other hot kernels (K-Means, DRF, DL).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_algos
run() {
  name=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_LDS_IDX_ACTIVE -d gpurun_out/pmc_algos/$name/a -o run --output-format csv -- python3 bench.py "$@" > gpurun_out/pmc_algos/$name.log 2>&1 || true
  python3 scripts/pmc_summary.py gpurun_out/pmc_algos/$name > gpurun_out/pmc_algos/$name.txt || true
  find gpurun_out/pmc_algos/$name -name '*.csv' -size +20M -delete
  echo "== $name"; grep -B1 -A3 "bank-conflict" gpurun_out/pmc_algos/$name.txt | head -40
}
run kmeans --algo kmeans --rows 20000000 --steps 5 --warmup 1
run drf --algo drf --rows 2000000 --cols 50 --steps 3 --warmup 1
run dl --algo dl --rows 2000000 --steps 50 --warmup 5
