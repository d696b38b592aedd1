set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u scripts/algo_survey2.py 2>&1 | tee gpurun_out/algo_survey2.log || { tail -5 gpurun_out/algo_survey2.log; exit 1; }
grep "{" gpurun_out/algo_survey2.log || true
