# Per-tree GPU busy time vs wall span from a kernel trace (ROWS rows, depth 8).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
R=${ROWS:-12500000}
OUT=gpurun_out/rocprof_gbm_$R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 bench.py --rows $R --steps 10 --warmup 2 --no-glm > $OUT.log 2>&1
python3 - "$OUT/run_kernel_trace.csv" > gpurun_out/gbm_${R}_pertree.txt <<'PY'
import csv, sys, collections
tr = list(csv.DictReader(open(sys.argv[1])))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(tr) if "hist_quad" in r["Kernel_Name"] or "hist_bm_kernel" in r["Kernel_Name"]]
st = idx[::8]
a, b = st[-9], st[-1]
sub = tr[a:b]
tot = collections.defaultdict(float); cnt = collections.Counter()
busy = 0; prev = int(sub[0]["Start_Timestamp"]); gaps = []; gapk = []; last_k = ""
for r in sub:
    s_, e_ = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    k = r["Kernel_Name"][:60]; tot[k] += (e_ - s_) / 1e6 / 8; cnt[k] += 1
    if s_ > prev: gaps.append(s_ - prev); gapk.append((s_ - prev, last_k, r["Kernel_Name"][:50]))
    last_k = r["Kernel_Name"][:50]
    busy += e_ - s_; prev = max(prev, e_)
span = (int(tr[b]["Start_Timestamp"]) - int(tr[a]["Start_Timestamp"])) / 1e6 / 8
print(f"per tree (last 8 trees): span {span:.2f} ms, kernel busy {busy/1e6/8:.2f} ms, launches {len(sub)/8:.0f}, idle gaps {sum(gaps)/1e6/8:.2f} ms in {len(gaps)/8:.0f} gaps")
gaps.sort(reverse=True)
print("largest gaps (us):", [round(g / 1e3) for g in gaps[:12]])
gapk.sort(reverse=True)
for g, a_, b_ in gapk[:10]:
    print(f"  gap {g/1e3:7.0f} us after {a_} -> before {b_}")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:14]:
    print(f"{v:8.3f} ms {cnt[k]/8:6.1f}x  {k}")
# per-level times of the level kernels (mean over the 8 trees, in launch order)
for name in ("hist_bm_kernel", "hist_bm_reduce", "hist_quad", "part_flags", "part_compact", "hist_sibling", "split_kernel"):
    ks = [r for r in sub if name in r["Kernel_Name"]]
    per = len(ks) // 8
    if per == 0:
        continue
    lv = [sum((int(ks[t * per + i]["End_Timestamp"]) - int(ks[t * per + i]["Start_Timestamp"])) for t in range(8)) / 8e3
          for i in range(per)]
    print(f"{name:14s} per level (us):", [round(x) for x in lv])
PY
rm -f $OUT/run_kernel_trace.csv
cat gpurun_out/gbm_${R}_pertree.txt
