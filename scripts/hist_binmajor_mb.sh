set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_tree_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "packed or hist" > gpurun_out/pytest_hist.log 2>&1 || { tail -30 gpurun_out/pytest_hist.log; exit 1; }
tail -n 1 gpurun_out/pytest_hist.log
for BM in 0 1; do
  H2O3_HIST_BINMAJOR=$BM H2O3_PROFILE=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bm_$BM.log 2>&1
  echo "binmajor=$BM $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bm_$BM.log)"
  grep phases gpurun_out/bm_$BM.log | cut -c1-300
done
