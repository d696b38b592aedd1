#!/bin/bash
# PMC of the wide Gram kernel after the round-5 changes (bf16 tier, 64-row chunks,
# scalar weights) and of the narrow bf16-tier IRLS kernel
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
MB_ARMS=bf16 timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_BUSY_CYCLES \
  --output-format csv -d $R/gpurun_out/pmc_wide3 -o p -- python3 scripts/wide_gram_mb.py 3000000 > gpurun_out/r5_pmc_wide3.log 2>&1 || { tail -20 gpurun_out/r5_pmc_wide3.log; exit 1; }
H2O3_GLM_BF3=2 H2O3_MB_GRAD=1 timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_BUSY_CYCLES \
  --output-format csv -d $R/gpurun_out/pmc_ws3 -o p -- python3 scripts/glm_ws_mb.py 20000000 > gpurun_out/r5_pmc_ws3.log 2>&1 || { tail -20 gpurun_out/r5_pmc_ws3.log; exit 1; }
python3 - <<'PY' > gpurun_out/pmc_r5_summary.txt
import csv, glob, collections
for d in ("gpurun_out/pmc_wide3", "gpurun_out/pmc_ws3"):
    fs = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    agg = collections.defaultdict(float); cnt = collections.Counter()
    for f in fs:
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")[:70]
            agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            cnt[(k, r["Counter_Name"])] += 1
    ks = sorted({k for k, _ in agg}, key=lambda k: -agg.get((k, "SQ_WAVE_CYCLES"), 0))
    print("==", d)
    for k in ks[:4]:
        g = lambda c: agg.get((k, c), float("nan"))
        wc, busy = g("SQ_WAVE_CYCLES"), g("SQ_BUSY_CYCLES")
        print(f"  {k}")
        print("    " + "  ".join(f"{c}={g(c):.3e}" for c in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_LDS_BANK_CONFLICT", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE")))
        print(f"    wait/wave-cycles {g('SQ_WAIT_ANY') / wc:.2f}   MFMA busy / (SQ_BUSY_CYCLES x 4 SIMD... raw ratio) {g('SQ_VALU_MFMA_BUSY_CYCLES') / busy:.2f}")
PY
cat gpurun_out/pmc_r5_summary.txt
find gpurun_out/pmc_wide3 gpurun_out/pmc_ws3 -name "*.csv" -size +20M -delete
