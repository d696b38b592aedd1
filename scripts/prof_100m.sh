# rocprofv3 kernel stats of the headline bench (100M x 100, depth 8) + GLM, and
# per-tree kernel time breakdown from the trace.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/rocprof_gbm100m
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 > $OUT.log 2>&1
tail -n 1 $OUT.log | cut -c1-300
python3 - "$OUT/run_kernel_trace.csv" <<'PY'
import csv, sys, collections
tr = list(csv.DictReader(open(sys.argv[1])))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(tr) if "hist_quad" in r["Kernel_Name"]]
st = idx[::8]
a, b = st[-9], st[-1]
sub = tr[a:b]
tot = collections.defaultdict(float); cnt = collections.Counter()
for r in sub:
    k = r["Kernel_Name"][:70]; tot[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 / 8; cnt[k] += 1
span = (int(tr[b]["Start_Timestamp"]) - int(tr[a]["Start_Timestamp"])) / 1e6 / 8
print(f"per tree (last 8 trees): span {span:.2f} ms, kernel busy {sum(tot.values()):.2f} ms, launches {len(sub)/8:.0f}")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:14]:
    print(f"{v:8.3f} ms {cnt[k]/8:6.1f}x  {k}")
PY
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof_glm100m -o run --output-format csv -- python3 bench.py --algo glm --steps 10 --warmup 2 > gpurun_out/rocprof_glm100m.log 2>&1
tail -n 1 gpurun_out/rocprof_glm100m.log | cut -c1-300
