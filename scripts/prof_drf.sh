# Kernel-level profile of the DRF config (10M x 500, 100 categoricals of
# cardinality 1000), row-direct pair histograms at every sampled level.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/rocprof_drf
H2O3_PAIR_DIRECT=${D:-1} timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- \
  python3 bench.py --algo drf --rows 10000000 --cols 500 --cat-cols 100 --cat-card 1000 --steps 2 --warmup 1 > $OUT.log 2>&1
grep '"metric"' $OUT.log | cut -c1-200
python3 - "$OUT/run_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:18]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):7d} calls {float(r["Percentage"]):5.1f}%  {r["Name"][:100]}')
PY
