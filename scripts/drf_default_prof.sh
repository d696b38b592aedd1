# Default DRF (AutoML DRF_1 shape) on 2M x 50: phase timers + rocprof kernel stats.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/drf_default_timing.py > gpurun_out/drf_default.log 2>&1
cat gpurun_out/drf_default.log | cut -c1-3000
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof_drf2m -o run --output-format csv -- python3 scripts/drf_default_timing.py > gpurun_out/rocprof_drf2m.log 2>&1
head -25 gpurun_out/rocprof_drf2m/run_kernel_stats.csv | cut -d, -f1-5 | cut -c1-160
rm -f gpurun_out/rocprof_drf2m/run_kernel_trace.csv
