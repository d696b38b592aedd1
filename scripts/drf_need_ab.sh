#!/bin/bash
# A/B of the DRF need mask on the 10M x 500 (100 cat, card 1000) shape.
set -e
mkdir -p gpurun_out
for need in 0 1; do
  H2O3_HIST_NEED=$need timeout -k 10 300 python -u bench.py --algo drf --rows 10000000 --cols 500 --cat-cols 100 \
    --cat-card 1000 --steps 3 --warmup 1 > gpurun_out/drf_need$need.json 2> gpurun_out/drf_need$need.err
  tail -n 1 gpurun_out/drf_need$need.json
done
