# GPU tests + smoke + row sweep (1M / 12.5M / 100M) with phase timers.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 2 gpurun_out/pytest_gpu.log
for R in ${ROWS:-1000000 12500000 100000000}; do
  H2O3_PROFILE=${PROF:-0} timeout -k 10 300 python bench.py --rows $R --steps 10 --warmup 2 > gpurun_out/sweep_$R.log 2>&1
  echo "rows=$R $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sweep_$R.log) $(grep -o '"train_logloss_after": [0-9.]*' gpurun_out/sweep_$R.log)"
  grep phases gpurun_out/sweep_$R.log | cut -c1-400 || true
done
