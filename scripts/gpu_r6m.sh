set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6m
timeout -k 10 200 python -u -m pytest -x -q --timeout 100 --timeout-method thread -m gpu tests/test_deeplearning.py > gpurun_out/r6m/tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/r6m/tests.log; exit 1; }
for t in 64x64 64x128 128x128; do
H2O3_DL_GEMM_TILE=$t timeout -k 10 120 python -u -m pytest -x -q --timeout 100 --timeout-method thread -m gpu "tests/test_deeplearning.py::test_dl_gemm_kernel_matches_fp64" > gpurun_out/r6m/gemm_test_$t.log 2>&1 || { echo "gemm test $t failed"; tail -20 gpurun_out/r6m/gemm_test_$t.log; exit 1; }
H2O3_DL_GEMM_TILE=$t timeout -k 10 200 python scripts/km_dl_mb.py 1000000 > gpurun_out/r6m/mb_$t.txt 2>&1 || { echo "mb $t failed"; exit 1; }
H2O3_DL_GEMM_TILE=$t timeout -k 10 300 python bench.py --algo dl --rows 2000000 --hidden 1024,1024 --batch 1024 --steps 200 --warmup 20 \
  > gpurun_out/r6m/dl_h1024_$t.json 2> gpurun_out/r6m/dl_h1024_$t.err || { echo "dl bench $t failed"; exit 1; }
done
echo done
