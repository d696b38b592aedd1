# DRF config of BASELINE.json at its full row count on ONE GPU:
# 50M x 500 (400 numeric + 100 categorical of cardinality 1000), ntrees=1000 model, depth 20.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
H2O3_PROFILE=1 timeout -k 10 900 python -u bench.py --algo drf --rows ${ROWS:-50000000} --cols 500 --cat-cols 100 \
  --cat-card 1000 --steps ${STEPS:-4} --warmup 1 > gpurun_out/drf_50m_bench.log 2>&1
grep '"metric"' gpurun_out/drf_50m_bench.log | cut -c1-600
grep phases gpurun_out/drf_50m_bench.log | cut -c1-800 || true
