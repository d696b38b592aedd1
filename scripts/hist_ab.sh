# Histogram kernel A/B: one launch, fewest groups (3 x 36 at F=100); LW=1 vs 2; then the GBM bench.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_tree_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tk.log 2>&1 || { tail -30 gpurun_out/tk.log; exit 1; }
tail -1 gpurun_out/tk.log
for LW in 1 2; do
  echo "== LW=$LW"; H2O3_HIST_LW=$LW KERNELS=quad timeout -k 10 200 python scripts/hist_fsweep_mb.py
done
echo "== LW=1 FGW=32"; H2O3_HIST_FGW=32 KERNELS=quad timeout -k 10 200 python scripts/hist_fsweep_mb.py
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1
tail -1 gpurun_out/bench_default.log | cut -c1-300
