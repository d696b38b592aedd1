set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/rocprof_1m
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 bench.py --rows ${ROWS:-1000000} --steps 20 --warmup 2 > $OUT.log 2>&1
tail -n 1 $OUT.log | cut -c1-200
python3 - "$OUT/run_kernel_stats.csv" "$OUT/run_kernel_trace.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.1f} ms over {sum(int(r['Calls']) for r in rows)} launches")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):6d} calls {float(r["Percentage"]):5.1f}%  {r["Name"][:100]}')
tr = list(csv.DictReader(open(sys.argv[2])))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
# last 20 trees ~ the timed window: take the final 60% of the trace
n = len(tr); sub = tr[int(n*0.5):]
span = (int(sub[-1]["End_Timestamp"]) - int(sub[0]["Start_Timestamp"]))/1e6
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in sub)/1e6
print(f"second half of trace: span {span:.1f} ms, kernel busy {busy:.1f} ms, launches {len(sub)}")
PY
