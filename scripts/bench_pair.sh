# Default bench at 100M and 12.5M rows (GBM + companion GLM).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1
tail -1 gpurun_out/bench_default.log | cut -c1-700
timeout -k 10 300 python bench.py --rows 12500000 --steps 20 --warmup 3 > gpurun_out/bench_12m5.log 2>&1
grep -o '"ms_per_step": [0-9.]*\|"glm_ms_per_iter": [0-9.]*' gpurun_out/bench_12m5.log
