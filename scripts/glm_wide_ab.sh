set -e
export TMPDIR=/tmp
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_linalg_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_wide.log 2>&1 || { tail -30 gpurun_out/pytest_wide.log; exit 1; }
tail -n 1 gpurun_out/pytest_wide.log
for M in bf3; do
  H2O3_WIDE_GRAM=$M H2O3_PROFILE=1 timeout -k 10 500 python bench.py --algo glm --rows 12500000 --cols 1000 --steps 5 --warmup 1 > gpurun_out/glm_wide_$M.log 2>&1
  echo "$M $(grep '"metric"' gpurun_out/glm_wide_$M.log | cut -c1-200)"
  grep -o '"train_dev.*' gpurun_out/glm_wide_$M.log || true
  grep phases gpurun_out/glm_wide_$M.log | cut -c1-300 || true
done
