set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6c
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6c/gpu_tests.log 2>&1
rc=$?
tail -30 gpurun_out/r6c/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for k in 16 64 128; do
  timeout -k 10 300 python bench.py --algo kmeans --k $k --steps 10 --warmup 2 > gpurun_out/r6c/kmeans_k$k.json 2> gpurun_out/r6c/kmeans_k$k.err || exit $?
done
timeout -k 10 300 python bench.py --algo pca --k 10 --steps 5 --warmup 1 > gpurun_out/r6c/pca_k10.json 2> gpurun_out/r6c/pca_k10.err
timeout -k 10 400 python bench.py --histogram-type UniformAdaptive --nbins 20 --steps 8 --warmup 2 --no-glm > gpurun_out/r6c/gbm_ua_100m.json 2> gpurun_out/r6c/gbm_ua_100m.err
