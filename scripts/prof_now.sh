# Current per-tree kernel breakdown: headline 100M rows and the 12.5M per-GPU share.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/rocprof_gbm100m
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 > $OUT.log 2>&1
tail -n 1 $OUT.log | cut -c1-200
ROWS=100000000 bash scripts/prof_gbm_rows.sh
ROWS=12500000 bash scripts/prof_gbm_rows.sh
