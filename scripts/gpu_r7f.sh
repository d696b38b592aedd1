set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r7f
timeout -k 10 400 python -u scripts/drf_host_prof.py > gpurun_out/r7f/drf_host_prof.txt 2>&1 || { echo "drf prof failed"; tail -20 gpurun_out/r7f/drf_host_prof.txt; exit 1; }
head -3 gpurun_out/r7f/drf_host_prof.txt
