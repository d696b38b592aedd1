"""Sum rocprofv3 --pmc counter CSVs per kernel name (all passes under a dir)."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
dur = collections.defaultdict(float)
for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:70]
        vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add((f, r["Dispatch_Id"]))
for f in sorted(glob.glob(os.path.join(root, "a", "**", "*kernel_trace.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        dur[r["Kernel_Name"][:70]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
order = sorted(vals, key=lambda k: -dur.get(k, 0))
for k in order[:16]:
    v = vals[k]
    ms = dur.get(k, 0.0)
    print(f"== {k}  time {ms:.2f} ms (pass a, all dispatches)")
    line = []
    for c in sorted(v):
        line.append(f"{c}={v[c]:.4g}")
    print("   " + "  ".join(line))
    if "FETCH_SIZE" in v and ms > 0:
        print(f"   HBM read {v['FETCH_SIZE'] / 1e6:.2f} GB -> {v['FETCH_SIZE'] * 1e3 / (ms * 1e-3) / 1e12:.2f} TB/s")
    if "TCC_HIT_sum" in v and v.get("TCC_MISS_sum", 0) + v["TCC_HIT_sum"] > 0:
        print(f"   L2 hit {100 * v['TCC_HIT_sum'] / (v['TCC_HIT_sum'] + v['TCC_MISS_sum']):.1f}%")
    if "SQ_LDS_BANK_CONFLICT" in v and v.get("SQ_INSTS_LDS"):
        print(f"   LDS bank-conflict cycles / LDS instr {v['SQ_LDS_BANK_CONFLICT'] / v['SQ_INSTS_LDS']:.2f}")
