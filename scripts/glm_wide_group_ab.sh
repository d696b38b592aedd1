# Row chunks per batched bf16 Gram GEMM (H2O3_WIDE_GROUP) at 12.5M x 1000:
# 32 output tiles of 256 x 256 per chunk, so the group sets how many tiles
# are in flight on the 256 CUs.
set -e
mkdir -p gpurun_out
for G in 4 8 16; do
  H2O3_WIDE_GROUP=$G timeout -k 10 400 python bench.py --algo glm --rows 12500000 --cols 1000 --steps 5 --warmup 1 > gpurun_out/glm_wide_g$G.log 2>&1
  echo "group=$G $(grep '"metric"' gpurun_out/glm_wide_g$G.log | cut -c1-140)"
done
