set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r7l
cd /tmp && ALGO=coxph timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r7l/prof -o cox -- python3 $GRAFT_REPO_ROOT/scripts/prof_any.py > $GRAFT_REPO_ROOT/gpurun_out/r7l/rocprof.log 2>&1 || { echo "rocprof failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r7l/rocprof.log; exit 1; }
echo ok
