# Histogram workgroup-count sweep (H2O3_HIST_TB) at the root and a deep level,
# 100M and 12.5M rows, then the GBM bench at 12.5M for the best candidates.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for N in 12500000 100000000; do
  for TB in 512 1024 2048 4096; do
    H2O3_HIST_TB=$TB N=$N ONLY=1 timeout -k 10 200 python scripts/hist_tb_mb.py >> gpurun_out/hist_tb.txt 2>&1
  done
done
cat gpurun_out/hist_tb.txt
