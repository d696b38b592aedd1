# GLM IRLSM at 1000 columns (the per-GPU share of the 100M x 1000 config at 8 GPUs).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
H2O3_PROFILE=1 timeout -k 10 500 python bench.py --algo glm --rows ${ROWS:-12500000} --cols 1000 --steps 3 --warmup 1 > gpurun_out/glm_wide.log 2>&1
grep '"metric"' gpurun_out/glm_wide.log | cut -c1-260
grep phases gpurun_out/glm_wide.log | cut -c1-400 || true
