# K-Means: GPU tests, 100M x 100 Lloyd iteration rate for several k, rocprof stats.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kmeans.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_kmeans.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_kmeans.log; exit 1; }
tail -n 3 gpurun_out/pytest_kmeans.log
for K in ${KS:-4 16 64 128}; do
  timeout -k 10 300 python bench.py --algo kmeans --k $K --steps 10 --warmup 2 > gpurun_out/kmeans_k$K.log 2>&1
  echo "k=$K $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/kmeans_k$K.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kmeans -o kmeans --output-format csv -- python bench.py --algo kmeans --k 16 --steps 10 --warmup 2 > gpurun_out/kmeans_prof.log 2>&1
find gpurun_out/prof_kmeans -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/kmeans_kernel_stats.csv
head -8 gpurun_out/kmeans_kernel_stats.csv | cut -c1-220
