# Histogram kernel A/B: 2 x 512-thread WGs per CU (80 KB LDS each) vs 1 x 1024-thread WG (156 KB); then the GBM bench both ways.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_tree_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tk.log 2>&1 || { tail -30 gpurun_out/tk.log; exit 1; }
tail -1 gpurun_out/tk.log
echo "== default"; KERNELS=quad timeout -k 10 200 python scripts/hist_fsweep_mb.py
echo "== BIG"; H2O3_HIST_BIG=1 KERNELS=quad timeout -k 10 200 python scripts/hist_fsweep_mb.py
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1
tail -1 gpurun_out/bench_default.log | cut -c1-200
H2O3_HIST_BIG=1 timeout -k 10 400 python bench.py > gpurun_out/bench_big.log 2>&1
tail -1 gpurun_out/bench_big.log | cut -c1-200
