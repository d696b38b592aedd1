#!/bin/bash
# round 5: collective bytes per tree level at W = 8 (8 gloo ranks sharing one
# GPU: the byte counts are those of an 8-GPU run, the times are not)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
export H2O3_DIST_BACKEND=gloo OMP_NUM_THREADS=2 PYTORCH_ALLOC_CONF=expandable_segments:True
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --master-port 29541 --nproc-per-node 8 \
  scripts/coll_bytes.py --algo gbm --rows 100000000 --cols 100 --trees 2 --out gpurun_out/coll_bytes_gbm_w8.json \
  > gpurun_out/r5_coll_gbm.log 2>&1 || { tail -30 gpurun_out/r5_coll_gbm.log; exit 1; }
grep MB_per_tree gpurun_out/r5_coll_gbm.log
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --master-port 29542 --nproc-per-node 8 \
  scripts/coll_bytes.py --algo drf --rows 50000000 --cols 500 --cat-cols 100 --trees 1 --out gpurun_out/coll_bytes_drf_w8.json \
  > gpurun_out/r5_coll_drf.log 2>&1 || { tail -30 gpurun_out/r5_coll_drf.log; exit 1; }
grep MB_per_tree gpurun_out/r5_coll_drf.log
