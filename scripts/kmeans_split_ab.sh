# K-Means Lloyd iteration at 100M x 100: fused kernel vs the large-k split path
# (assignment pass + fixed-point sums pass), k = 16 / 64 / 128; then the GPU tests.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kmeans.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/km_tests.log 2>&1 || { tail -30 gpurun_out/km_tests.log; exit 1; }
tail -n 2 gpurun_out/km_tests.log
for k in ${KS:-16 64 128}; do
  for s in 0 1; do
    H2O3_KM_SPLIT=$s timeout -k 10 300 python bench.py --algo kmeans --k $k --steps 10 --warmup 2 > gpurun_out/km_${k}_${s}.log 2>&1
    echo "k=$k split=$s $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/km_${k}_${s}.log)"
  done
done
