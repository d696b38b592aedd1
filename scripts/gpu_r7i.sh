set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r7i
timeout -k 10 200 python -u scripts/gram_f64_mb.py > gpurun_out/r7i/gram_f64_mb_ld712.txt 2>&1 || { echo "mb failed"; tail -20 gpurun_out/r7i/gram_f64_mb_ld712.txt; exit 1; }
cat gpurun_out/r7i/gram_f64_mb_ld712.txt
LDX=711 timeout -k 10 200 python -u scripts/gram_f64_mb.py > gpurun_out/r7i/gram_f64_mb_ld711.txt 2>&1 || { echo "mb failed"; tail -20 gpurun_out/r7i/gram_f64_mb_ld711.txt; exit 1; }
cat gpurun_out/r7i/gram_f64_mb_ld711.txt
