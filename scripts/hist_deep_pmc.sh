# Deep-level vs root histogram: timing per feature-group width, then HBM bytes
# (FETCH_SIZE) and L2 hits per level from one PMC pass each.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_deep
: > gpurun_out/hist_deep.txt
for L in root deep; do
  for W in 36 52 28; do
    LEVEL=$L H2O3_HIST_FGW=$W timeout -k 10 120 python scripts/hist_deep_mb.py >> gpurun_out/hist_deep.txt 2>&1
  done
done
cat gpurun_out/hist_deep.txt
for L in root deep; do
  LEVEL=$L REPS=2 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE TCC_HIT_sum -d gpurun_out/pmc_deep/$L \
    -o run --output-format csv -- python3 scripts/hist_deep_mb.py
done
