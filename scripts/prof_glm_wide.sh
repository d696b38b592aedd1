set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof_glm_wide -o run --output-format csv -- python3 bench.py --algo glm --rows 12500000 --cols 1000 --steps 3 --warmup 1 > gpurun_out/rocprof_glm_wide.log 2>&1
python3 - <<'PY' > gpurun_out/rocprof_glm_wide_summary.txt
import csv, collections
r = list(csv.DictReader(open("gpurun_out/rocprof_glm_wide/run_kernel_stats.csv")))
for x in r[:10]:
    print(x["Calls"], round(float(x["AverageNs"]) / 1e6, 3), "ms avg", round(float(x["TotalDurationNs"]) / 1e6, 1), "ms tot", x["Name"][:110])
tr = list(csv.DictReader(open("gpurun_out/rocprof_glm_wide/run_kernel_trace.csv")))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(tr) if "glm_wide_split" in r["Kernel_Name"]]
n = len(idx) // 4
a, b = idx[2 * n], idx[3 * n]
t0 = int(tr[a]["Start_Timestamp"])
busy = 0; prev = t0; gaps = []
for x in tr[a:b]:
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    if s > prev:
        gaps.append((s - prev, x["Kernel_Name"][:70]))
    busy += e - s; prev = max(prev, e)
print("pass 3: span ms", (int(tr[b]["Start_Timestamp"]) - t0) / 1e6, "busy ms", busy / 1e6, "kernels", b - a)
gaps.sort(reverse=True)
for g in gaps[:10]:
    print("gap", round(g[0] / 1e6, 3), "before", g[1])
c = collections.Counter(x["Kernel_Name"][:90] for x in tr[a:b])
for k, v in c.most_common(12):
    print(v, k)
PY
rm -f gpurun_out/rocprof_glm_wide/run_kernel_trace.csv
cat gpurun_out/rocprof_glm_wide_summary.txt
