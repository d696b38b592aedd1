# bf16x3 vs f32 MFMA A/B for the fused GLM IRLS kernel (P = 100 -> padded 128).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_linalg_gpu.py tests/test_gpu_algos.py -k "glm or gram or GLM" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_glm.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_glm.log; exit 1; }
tail -n 2 gpurun_out/pytest_glm.log
for B in 1 0; do
  H2O3_GLM_BF3=$B timeout -k 10 300 python bench.py --algo glm --steps 10 --warmup 2 > gpurun_out/glm_bf3_$B.log 2>&1
  echo "bf3=$B $(tail -n 1 gpurun_out/glm_bf3_$B.log | cut -c1-400)"
done
cd /tmp && H2O3_GLM_BF3=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_glm_bf3 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --algo glm --steps 5 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_glm_bf3.log 2>&1
find $GRAFT_REPO_ROOT/gpurun_out/prof_glm_bf3 -name "*kernel_stats.csv" | head -1 | xargs head -8 | cut -c1-200
