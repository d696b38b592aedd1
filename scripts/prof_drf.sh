# Kernel statistics of the DRF BASELINE config shape at 10M rows (500 cols, 100 categorical of card 1000)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/rocprof_drf
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 bench.py --algo drf --rows ${ROWS:-10000000} --cols 500 --cat-cols 100 --cat-card 1000 --steps 3 --warmup 1 > $OUT.log 2>&1
grep '"metric"' $OUT.log | cut -c1-200
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/rocprof_drf/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.1f} ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:18]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.1f} ms {int(r["Calls"]):7d}x  {r["Name"][:90]}')
PY
rm -f gpurun_out/rocprof_drf/*/*kernel_trace.csv gpurun_out/rocprof_drf/*kernel_trace.csv 2>/dev/null || true
