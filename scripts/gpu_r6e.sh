set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6e
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_kmeans.py tests/test_deeplearning.py tests/test_ua_fold_gpu.py "tests/test_linalg_gpu.py::test_xv_kernel_matches_fp64" \
  "tests/test_linalg_gpu.py::test_pca_methods_on_gram_kernel_match_fp64" > gpurun_out/r6e/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r6e/tests.log; exit 1; }
echo "tests ok"
for k in 128 64 16; do
timeout -k 10 300 python bench.py --algo kmeans --k $k --steps 10 --warmup 2 > gpurun_out/r6e/kmeans_k$k.json 2> gpurun_out/r6e/kmeans_k$k.err || { echo "kmeans bench failed"; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/profkm -o km --output-format csv -- python bench.py --algo kmeans --k 128 --steps 5 --warmup 1 \
  > gpurun_out/r6e/km_prof.log 2>&1 && cp $(find /tmp/profkm -name "*kernel_stats.csv" | head -1) gpurun_out/r6e/kmeans_k128_kernel_stats.csv || { echo "km prof failed"; exit 1; }
timeout -k 10 300 python bench.py --algo dl --rows 2000000 --hidden 1024,1024 --batch 1024 --steps 200 --warmup 20 \
  > gpurun_out/r6e/dl_h1024.json 2> gpurun_out/r6e/dl_h1024.err || { echo "dl bench failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/profdl -o dl --output-format csv -- python bench.py --algo dl --rows 2000000 --hidden 1024,1024 --batch 1024 --steps 50 --warmup 5 \
  > gpurun_out/r6e/dl_prof.log 2>&1 && cp $(find /tmp/profdl -name "*kernel_stats.csv" | head -1) gpurun_out/r6e/dl_h1024_kernel_stats.csv || { echo "dl prof failed"; exit 1; }
timeout -k 10 300 python bench.py --rows 12500000 --histogram-type UniformAdaptive --nbins 20 --steps 6 --warmup 2 --no-glm \
  > gpurun_out/r6e/gbm_ua_12m5.json 2> gpurun_out/r6e/gbm_ua_12m5.err || { echo "ua bench failed"; exit 1; }
echo "done"
