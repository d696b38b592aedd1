# Per-tree time vs rows on one GPU: 12.5M rows = the per-GPU share of the
# 100M benchmark at 8 GPUs, so this bounds the strong-scaling curve from the
# compute side (host overhead shows up as the floor at 1M rows).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for R in 100000000 25000000 12500000 1000000; do
  H2O3_PROFILE=1 timeout -k 10 300 python bench.py --rows $R --steps 10 --warmup 2 > gpurun_out/sweep_$R.log 2>&1
  echo "rows=$R $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sweep_$R.log)"
  grep phases gpurun_out/sweep_$R.log | cut -c1-600
done
