# Per-tree kernel breakdown of DRF at the BASELINE shape (50M x 500, 100
# categorical of cardinality 1000, depth 20) from a rocprofv3 kernel trace:
# only kernels after the first tree's first pair histogram are counted.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROWS:-50000000}
OUT=gpurun_out/rocprof_drf_$R
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 -u bench.py --algo drf \
  --rows $R --cols 500 --cat-cols 100 --cat-card 1000 --steps ${STEPS:-2} --warmup 1 > $OUT.log 2>&1
grep '"metric"' $OUT.log | cut -c1-300
python3 - "$(ls $OUT/*/run_kernel_trace.csv $OUT/run_kernel_trace.csv 2>/dev/null | head -1)" "${STEPS:-2}" > gpurun_out/drf_${R}_pertree.txt <<'PY'
import csv, sys, collections
tr = list(csv.DictReader(open(sys.argv[1])))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
first = next(i for i, r in enumerate(tr) if "pair_hist" in r["Kernel_Name"] or "hist_build" in r["Kernel_Name"])
sub = tr[first:]
ntree = int(sys.argv[2]) + 1
span = (int(sub[-1]["End_Timestamp"]) - int(sub[0]["Start_Timestamp"])) / 1e6 / ntree
tot = collections.defaultdict(float); cnt = collections.Counter()
busy = 0
for r in sub:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    k = r["Kernel_Name"][:80]
    tot[k] += d / ntree; cnt[k] += 1
    busy += d
print(f"per tree ({ntree} trees incl. warmup): span {span:.1f} ms, kernel busy {busy / ntree:.1f} ms")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:25]:
    print(f"{v:9.2f} ms {cnt[k] / ntree:8.1f}x  {k}")
PY
cat gpurun_out/drf_${R}_pertree.txt
