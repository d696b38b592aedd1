set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tree_kernels_gpu.py \
  -k "pair or direct" > gpurun_out/pytest_kp.log 2>&1
tail -2 gpurun_out/pytest_kp.log
for KP in 1 4; do
  H2O3_PAIR_KP=$KP timeout -k 10 400 python bench.py --algo drf --rows 10000000 --cols 500 --cat-cols 100 \
    --cat-card 1000 --steps 3 --warmup 1 > gpurun_out/kp_drf.log 2>&1
  echo "kp=$KP drf 10Mx500: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/kp_drf.log)"
done
