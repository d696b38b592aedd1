# bm kernel: work-item count A/B (H2O3_HIST_TB = total workgroups target) at 100M and 12.5M rows.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for R in 100000000 12500000; do
  for TB in default 512 1024 4096; do
    if [ "$TB" = default ]; then unset H2O3_HIST_TB; else export H2O3_HIST_TB=$TB; fi
    timeout -k 10 300 python bench.py --rows $R --steps 10 --warmup 2 --no-glm > gpurun_out/bmtb_${TB}_$R.log 2>&1
    echo "rows=$R TB=$TB $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bmtb_${TB}_$R.log) $(grep -o '"train_logloss_after": [0-9.]*' gpurun_out/bmtb_${TB}_$R.log)"
  done
done
