set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r7k
for a in coxph isolationforest extendedisolationforest; do
  ALGO=$a timeout -k 10 300 python -u scripts/prof_any.py > gpurun_out/r7k/prof_$a.txt 2>&1 || { echo "$a prof failed"; tail -20 gpurun_out/r7k/prof_$a.txt; exit 1; }
  grep train_s gpurun_out/r7k/prof_$a.txt
done
