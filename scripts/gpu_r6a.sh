set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6a
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_devtree_gpu.py > gpurun_out/r6a/devtree_test.log 2>&1 && \
timeout -k 10 300 python bench.py --rows 12500000 --steps 40 --warmup 5 --no-glm > gpurun_out/r6a/bench12m5.json 2> gpurun_out/r6a/bench12m5.err && \
H2O3_DEV_TREE=0 timeout -k 10 300 python bench.py --rows 12500000 --steps 40 --warmup 5 --no-glm > gpurun_out/r6a/bench12m5_old.json 2> gpurun_out/r6a/bench12m5_old.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-glm > gpurun_out/r6a/bench100m.json 2> gpurun_out/r6a/bench100m.err
