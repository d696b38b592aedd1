# 8 ranks on ONE GPU over gloo: exercises the N=8 shapes (F=100 -> Fl=13, padded
# feature slices) of the multi-rank GBM / GLM path without RCCL.  Not a perf run.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
H2O3_DIST_BACKEND=gloo OMP_NUM_THREADS=2 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --master-port 29533 --nproc-per-node 8 \
  bench.py --gpus 8 --rows 4000000 --steps 3 --warmup 1 > gpurun_out/rehearse8.log 2>&1 || { tail -30 gpurun_out/rehearse8.log; exit 1; }
grep '"metric"' gpurun_out/rehearse8.log | cut -c1-260
grep -o '"train_logloss_after": [0-9.]*\|"glm_ms_per_iter": [0-9.]*' gpurun_out/rehearse8.log
