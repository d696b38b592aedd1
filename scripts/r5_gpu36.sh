#!/bin/bash
# swizzle A/B of the bf16 64-row-chunk wide Gram kernel: time + LDS bank-conflict cycles
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
for z in 0 1 2; do
  H2O3_WG2_SWZ=$z MB_ARMS=bf16 timeout -k 10 200 python -u scripts/wide_gram_mb.py 2>&1 | grep -v amdgpu.ids | sed "s/^/swz=$z /" || exit 1
  H2O3_WG2_SWZ=$z MB_ARMS=bf16 timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES \
    --output-format csv -d $R/gpurun_out/pmc_swz$z -o p -- python3 scripts/wide_gram_mb.py 3000000 > gpurun_out/pmc_swz$z.log 2>&1 || { tail -5 gpurun_out/pmc_swz$z.log; exit 1; }
  python3 - $z <<'PY'
import csv, glob, sys, collections
z = sys.argv[1]
agg = collections.defaultdict(float)
for f in glob.glob(f"gpurun_out/pmc_swz{z}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gram256" in r.get("Kernel_Name", ""):
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
print(f"swz={z} PMC gram256:", {k: f"{v:.3e}" for k, v in agg.items()})
PY
done
