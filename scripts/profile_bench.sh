set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/rocprof_gbm100m}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python bench.py --rows 100000000 --steps 5 --warmup 1 > $OUT.log 2>&1
tail -n 1 $OUT.log
head -12 $OUT/run_kernel_stats.csv | cut -c1-200
