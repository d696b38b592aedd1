set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6g
timeout -k 10 120 python -u -m pytest -x -q --timeout 100 --timeout-method thread -m gpu "tests/test_deeplearning.py" > gpurun_out/r6g/tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/r6g/tests.log; exit 1; }
timeout -k 10 200 python scripts/km_dl_mb.py 20000000 > gpurun_out/r6g/mb.txt 2>&1 || { echo "mb failed"; tail gpurun_out/r6g/mb.txt; exit 1; }
H2O3_DL_GEMM=0 timeout -k 10 200 python scripts/km_dl_mb.py 1000000 > gpurun_out/r6g/mb_torchmm.txt 2>&1 || { echo "mb2 failed"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE SQ_BUSY_CYCLES \
  --output-format csv -d /tmp/pmc_km -o p -- python3 scripts/km_dl_mb.py 20000000 > gpurun_out/r6g/pmc.log 2>&1 || { echo "pmc failed"; tail gpurun_out/r6g/pmc.log; exit 1; }
python3 - <<'PY' > gpurun_out/r6g/pmc_summary.txt
import csv, glob, collections
fs = glob.glob("/tmp/pmc_km/**/*counter_collection.csv", recursive=True)
agg = collections.defaultdict(float); n = collections.Counter()
for f in fs:
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")[:80]
        agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        if r["Counter_Name"] == "SQ_WAVE_CYCLES":
            n[k] += 1
ks = sorted({k for k, _ in agg}, key=lambda k: -agg.get((k, "SQ_WAVE_CYCLES"), 0))
for k in ks[:8]:
    g = lambda c: agg.get((k, c), float("nan"))
    wc = g("SQ_WAVE_CYCLES")
    print(f"{k}  (dispatches {n[k]})")
    print("    " + "  ".join(f"{c}={g(c):.3e}" for c in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_LDS_BANK_CONFLICT", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE")))
    print(f"    wait_any/wave {g('SQ_WAIT_ANY') / wc:.2f}  wait_inst/wave {g('SQ_WAIT_INST_ANY') / wc:.2f}  active/wave {g('SQ_ACTIVE_INST_ANY') / wc:.2f}  mfma_busy/(4*GRBM) {g('SQ_VALU_MFMA_BUSY_CYCLES') / (4 * 256 * g('GRBM_GUI_ACTIVE')):.3f}")
PY
timeout -k 10 300 python bench.py --algo dl --rows 2000000 --hidden 1024,1024 --batch 1024 --steps 200 --warmup 20 \
  > gpurun_out/r6g/dl_h1024.json 2> gpurun_out/r6g/dl_h1024.err || { echo "dl bench failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/profua -o ua --output-format csv -- python bench.py --rows 12500000 --histogram-type UniformAdaptive --nbins 20 --steps 4 --warmup 2 --no-glm \
  > gpurun_out/r6g/ua_prof.log 2>&1 && cp $(find /tmp/profua -name "*kernel_stats.csv" | head -1) gpurun_out/r6g/ua_12m5_kernel_stats.csv || { echo "ua prof failed"; exit 1; }
echo done
