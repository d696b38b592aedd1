set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6i
timeout -k 10 200 python -u -m pytest -x -q --timeout 100 --timeout-method thread -m gpu tests/test_kmeans.py > gpurun_out/r6i/tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/r6i/tests.log; exit 1; }
timeout -k 10 200 python scripts/km_dl_mb.py 20000000 > gpurun_out/r6i/mb.txt 2>&1 || { echo "mb failed"; exit 1; }
for k in 128 64; do
timeout -k 10 300 python bench.py --algo kmeans --k $k --steps 10 --warmup 2 > gpurun_out/r6i/kmeans_k$k.json 2> gpurun_out/r6i/kmeans_k$k.err || { echo "kmeans bench failed"; exit 1; }
done
timeout -k 10 400 python bench.py --histogram-type UniformAdaptive --nbins 20 --steps 3 --warmup 1 --no-glm > gpurun_out/r6i/gbm_ua_100m.json 2> gpurun_out/r6i/gbm_ua_100m.err || { echo "ua bench failed"; exit 1; }
echo done
