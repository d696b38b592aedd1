set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --algo drf --rows 2000000 --cols 50 --steps 10 --warmup 2 > gpurun_out/drf2m.log 2>&1
echo "drf 2Mx50: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/drf2m.log)"
timeout -k 10 400 python bench.py --algo drf --rows 10000000 --cols 500 --cat-cols 100 --cat-card 1000 --steps 3 \
  --warmup 1 > gpurun_out/drf10m.log 2>&1
echo "drf 10Mx500: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/drf10m.log)"
BENCH_ARGS="--algo drf --rows 2000000 --cols 50 --steps 6 --warmup 1" timeout -k 10 400 python scripts/grow_line_sampler.py > gpurun_out/drf_lines3.txt 2>&1
head -22 gpurun_out/drf_lines3.txt | tail -20
