# DRF config of BASELINE.json (mixed numeric/categorical, high-cardinality
# categoricals) at reduced rows on one GPU, plus the 100-numeric GBM check.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
H2O3_PROFILE=1 timeout -k 10 400 python bench.py --algo drf --rows ${ROWS:-10000000} --cols 500 --cat-cols 100 --cat-card 1000 \
  --steps 5 --warmup 1 > gpurun_out/drf_bench.log 2>&1
grep '"metric"' gpurun_out/drf_bench.log | cut -c1-400
grep phases gpurun_out/drf_bench.log | cut -c1-500 || true
