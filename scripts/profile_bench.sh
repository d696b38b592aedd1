set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/rocprof_gbm100m}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 bench.py --rows 100000000 --steps 5 --warmup 1 > $OUT.log 2>&1
tail -n 1 $OUT.log
python3 - "$OUT/run_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):6d} calls {float(r["Percentage"]):5.1f}%  {r["Name"][:90]}')
PY
