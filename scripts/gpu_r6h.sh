set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6h
H2O3_KM_NW=6 timeout -k 10 200 python -u -m pytest -x -q --timeout 100 --timeout-method thread -m gpu tests/test_kmeans.py > gpurun_out/r6h/tests_nw6.log 2>&1 || { echo "tests nw6 failed"; tail -20 gpurun_out/r6h/tests_nw6.log; exit 1; }
timeout -k 10 200 python scripts/km_dl_mb.py 20000000 > gpurun_out/r6h/mb_nw4.txt 2>&1 || { echo "mb failed"; exit 1; }
H2O3_KM_NW=6 timeout -k 10 200 python scripts/km_dl_mb.py 20000000 > gpurun_out/r6h/mb_nw6.txt 2>&1 || { echo "mb6 failed"; exit 1; }
for ch in 65536 262144 524288; do
H2O3_HIST_CHUNK=$ch timeout -k 10 300 python bench.py --rows 12500000 --histogram-type UniformAdaptive --nbins 20 --steps 4 --warmup 2 --no-glm \
  > gpurun_out/r6h/ua_chunk$ch.json 2> gpurun_out/r6h/ua_chunk$ch.err || { echo "ua bench failed"; exit 1; }
done
for nw in 4 6; do
H2O3_KM_NW=$nw timeout -k 10 300 python bench.py --algo kmeans --k 128 --steps 10 --warmup 2 > gpurun_out/r6h/kmeans_k128_nw$nw.json 2> gpurun_out/r6h/kmeans_k128_nw$nw.err || { echo "kmeans bench failed"; exit 1; }
done
echo done
