# 2 ranks on one GPU (gloo): tree test + bench rehearsal of the packed-record multi-rank path.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_distributed_gpu.py -m gpu > gpurun_out/pytest_dist2.log 2>&1 || { tail -60 gpurun_out/pytest_dist2.log; exit 1; }
tail -n 3 gpurun_out/pytest_dist2.log
H2O3_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --standalone --nnodes=1 --nproc-per-node 2 \
  bench.py --gpus 2 --rows 4000000 --steps 3 --warmup 1 > gpurun_out/rehearse2.log 2>&1
grep '"metric"' gpurun_out/rehearse2.log | grep -o '"ms_per_step": [0-9.]*\|"train_logloss_after": [0-9.]*\|"glm_ms_per_iter": [0-9.]*'
timeout -k 10 300 python bench.py --rows 4000000 --steps 3 --warmup 1 > gpurun_out/rehearse1.log 2>&1
grep '"metric"' gpurun_out/rehearse1.log | grep -o '"ms_per_step": [0-9.]*\|"train_logloss_after": [0-9.]*'
