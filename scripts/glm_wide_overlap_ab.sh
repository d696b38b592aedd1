# A/B of the double-buffered split / GEMM pipeline of the wide GLM pass
# (12.5M x 1000, the per-GPU share of the 100M x 1000 config at 8 GPUs).
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_linalg_gpu.py -x -q --timeout 120 --timeout-method thread -k "wide or bf3" > gpurun_out/pytest_wide_overlap.log 2>&1 || { tail -30 gpurun_out/pytest_wide_overlap.log; exit 1; }
tail -n 1 gpurun_out/pytest_wide_overlap.log
for M in 0 1; do
  H2O3_WIDE_OVERLAP=$M timeout -k 10 400 python bench.py --algo glm --rows 12500000 --cols 1000 --steps 5 --warmup 1 > gpurun_out/glm_wide_overlap_$M.log 2>&1
  echo "overlap=$M $(grep '"metric"' gpurun_out/glm_wide_overlap_$M.log | cut -c1-220)"
done
