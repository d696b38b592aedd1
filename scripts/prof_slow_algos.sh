set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for a in aggregator rulefit infogram; do
  ALGO=$a timeout -k 10 300 python -u scripts/prof_rulefit.py > gpurun_out/prof_$a.log 2>&1
  grep train_s gpurun_out/prof_$a.log
done
