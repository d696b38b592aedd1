set -e
export TMPDIR=/tmp
timeout -k 10 200 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; }
for f in 0 20 25 32 50 10; do
  if [ "$f" = "0" ]; then unset H2O3_HIST_FGL; else export H2O3_HIST_FGL=$f; fi
  H2O3_PROFILE=1 timeout -k 10 200 python bench.py --rows 10000000 --steps 3 --warmup 1 > gpurun_out/ab_fgl_$f.log 2>&1
  echo "FGL=$f"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_fgl_$f.log; grep phases gpurun_out/ab_fgl_$f.log | cut -c1-200
done
