set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6p
timeout -k 10 500 python bench.py --algo drf --rows 6250000 --cols 500 --cat-cols 100 --steps 5 --warmup 2 > gpurun_out/r6p/drf_6m25.json 2> gpurun_out/r6p/drf_6m25.err || { echo "drf bench failed"; tail -5 gpurun_out/r6p/drf_6m25.err; exit 1; }
cat gpurun_out/r6p/drf_6m25.json
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d /tmp/profdrf -o run -- python scripts/drf_trace.py --rows 6250000 --trees 5 --warmup 2 \
  > gpurun_out/r6p/prof.log 2>&1 && python scripts/prof_summary.py $(find /tmp/profdrf -name "*kernel_trace.csv" | head -1) gpurun_out/r6p/drf_6m25_pertree_summary.txt --after-gap-ms 100 --per 5 || { echo "prof failed"; exit 1; }
echo done
