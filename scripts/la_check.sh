# Look-ahead level histograms: GPU tests, then per-tree timeline at 12.5M rows and the default bench.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_tree_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tk.log 2>&1 || { tail -40 gpurun_out/tk.log; exit 1; }
tail -1 gpurun_out/tk.log
bash scripts/prof_gbm_rows.sh > gpurun_out/prof_rows.log 2>&1
head -16 gpurun_out/prof_rows.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1
tail -1 gpurun_out/bench_default.log | cut -c1-200
H2O3_LOOKAHEAD=0 timeout -k 10 400 python bench.py > gpurun_out/bench_nola.log 2>&1
tail -1 gpurun_out/bench_nola.log | cut -c1-200
