# A/B of the DRF position-ordered response payload (H2O3_DRF_POSV) at the
# BASELINE DRF shape: per-level pair-histogram times of the last tree.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for M in 0 1; do
  OUT=gpurun_out/rocprof_drf_posv$M
  H2O3_DRF_POSV=$M timeout -k 10 600 rocprofv3 --kernel-trace -d $OUT -o run --output-format csv -- python3 -u bench.py \
    --algo drf --rows 50000000 --cols 500 --cat-cols 100 --cat-card 1000 --steps 1 --warmup 1 > $OUT.log 2>&1
  echo "posv=$M $(grep '"metric"' $OUT.log | cut -c1-160)"
  python3 - "$(ls $OUT/*/run_kernel_trace.csv $OUT/run_kernel_trace.csv 2>/dev/null | head -1)" <<'PY'
import csv, sys
tr = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ph = [r for r in tr if "pair_hist" in r["Kernel_Name"]]
half = len(ph) // 2
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in ph[half:]]
print("  last tree pair_hist per call (ms):", [round(x, 2) for x in d], "sum", round(sum(d), 1))
PY
done
