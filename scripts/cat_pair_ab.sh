# cat_pair_kernel: sorted prefix = occupied levels only. GPU tests of the pair
# kernels, then the DRF 10M x 500 (100 cat, card 1000) bench under rocprof.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_tree_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "cat_pair" > gpurun_out/cat_pair_tests.log 2>&1 || { tail -30 gpurun_out/cat_pair_tests.log; exit 1; }
tail -n 1 gpurun_out/cat_pair_tests.log
bash scripts/prof_drf.sh
