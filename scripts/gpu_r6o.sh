set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6o
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6o/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r6o/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/r6o/bench.json 2> gpurun_out/r6o/bench.err || { echo "bench failed"; tail -20 gpurun_out/r6o/bench.err; exit 1; }
cat gpurun_out/r6o/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof100 -o run --output-format csv -- python scripts/devtree_trace.py --rows 100000000 --trees 10 --warmup 3 \
  > gpurun_out/r6o/prof.log 2>&1 && python scripts/prof_summary.py $(find /tmp/prof100 -name "*kernel_trace.csv" | head -1) gpurun_out/r6o/gbm_100m_pertree_summary.txt --after-gap-ms 100 --per 10 \
  && cp $(find /tmp/prof100 -name "*kernel_stats.csv" | head -1) gpurun_out/r6o/gbm_100m_kernel_stats.csv || { echo "prof failed"; exit 1; }
echo done
