# Two ranks on ONE GPU over gloo: exercises the multi-rank GPU code path
# (feature reduce-scatter, candidate merge, sibling kernel on the local slice)
# without RCCL (which refuses two ranks on one device).  Not a perf run.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
H2O3_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --standalone --nnodes=1 --nproc-per-node 2 \
  bench.py --gpus 2 --rows 4000000 --steps 3 --warmup 1 > gpurun_out/rehearse2.log 2>&1
grep '"metric"' gpurun_out/rehearse2.log | cut -c1-300
H2O3_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --standalone --nnodes=1 --nproc-per-node 2 \
  bench.py --gpus 2 --algo glm --rows 4000000 --steps 3 --warmup 1 > gpurun_out/rehearse2_glm.log 2>&1
grep '"metric"' gpurun_out/rehearse2_glm.log | cut -c1-300
# DRF with mtries sampling and forced chunked deep levels (need-mask path) on two ranks
H2O3_HIST_BUDGET=4000000 H2O3_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --standalone --nnodes=1 --nproc-per-node 2 \
  bench.py --gpus 2 --algo drf --rows 1000000 --cols 64 --cat-cols 8 --cat-card 50 --steps 2 --warmup 1 > gpurun_out/rehearse2_drf.log 2>&1
grep '"metric"' gpurun_out/rehearse2_drf.log | cut -c1-300
# same GBM config on one rank: the 2-rank train_logloss_after must match
timeout -k 10 300 python bench.py --rows 4000000 --steps 3 --warmup 1 > gpurun_out/rehearse1.log 2>&1
grep '"metric"' gpurun_out/rehearse1.log | grep -o '"train_logloss_after": [0-9.]*'
grep '"metric"' gpurun_out/rehearse2.log | grep -o '"train_logloss_after": [0-9.]*'
H2O3_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --standalone --nnodes=1 --nproc-per-node 2 \
  bench.py --gpus 2 --algo kmeans --rows 4000000 --steps 3 --warmup 1 > gpurun_out/rehearse2_km.log 2>&1
grep '"metric"' gpurun_out/rehearse2_km.log | cut -c1-200
