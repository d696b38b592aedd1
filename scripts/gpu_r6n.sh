set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6n
H2O3_KM_RT=2 timeout -k 10 200 python -u -m pytest -x -q --timeout 100 --timeout-method thread -m gpu tests/test_kmeans.py > gpurun_out/r6n/tests_rt2.log 2>&1 || { echo "tests rt2 failed"; tail -20 gpurun_out/r6n/tests_rt2.log; exit 1; }
for rt in 1 2; do
H2O3_KM_RT=$rt timeout -k 10 200 python scripts/km_dl_mb.py 20000000 > gpurun_out/r6n/mb_rt$rt.txt 2>&1 || { echo "mb failed"; exit 1; }
for k in 128 64; do
H2O3_KM_RT=$rt timeout -k 10 300 python bench.py --algo kmeans --k $k --steps 10 --warmup 2 > gpurun_out/r6n/kmeans_k${k}_rt$rt.json 2> gpurun_out/r6n/kmeans_k${k}_rt$rt.err || { echo "kmeans bench failed"; exit 1; }
done
done
echo done
