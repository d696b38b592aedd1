# A/B matrix of GBM knobs on one box (same data, same process image)
set -e
export TMPDIR=/tmp
run() {
  tag=$1; shift
  env "$@" H2O3_PROFILE=1 timeout -k 10 300 python bench.py --rows 100000000 --steps 4 --warmup 1 > gpurun_out/ab_$tag.log 2>&1
  echo "$tag $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$tag.log) $(grep -o "'gbm.gamma': ([0-9.]*\|'tree.hist.L0': ([0-9.]*\|'tree.hist': ([0-9.]*\|'tree.split': ([0-9.]*\|'tree.partition': ([0-9.]*" gpurun_out/ab_$tag.log | tr '\n' ' ')"
}
run fg16_fused H2O3_HIST_FG=16 H2O3_FUSED_LEAF=1
run fg32_fused H2O3_HIST_FG=32 H2O3_FUSED_LEAF=1
run fg32_unfused H2O3_HIST_FG=32 H2O3_FUSED_LEAF=0
run fg16_unfused H2O3_HIST_FG=16 H2O3_FUSED_LEAF=0
