set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6b
# timed-window-only trace: a standalone script grows warmup trees, then the traced trees
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof12 -o run --output-format csv -- python scripts/devtree_trace.py --rows 12500000 --trees 20 > gpurun_out/r6b/trace_run.log 2>&1 && \
python scripts/prof_summary.py $(find /tmp/prof12 -name "*kernel_trace.csv" | head -1) gpurun_out/r6b/devtree_12m5_summary.txt --after-gap-ms 100 --per 20 && \
cp $(find /tmp/prof12 -name "*kernel_stats.csv" | head -1) gpurun_out/r6b/devtree_12m5_kernel_stats.csv
