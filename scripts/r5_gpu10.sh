#!/bin/bash
# round 5: wide Gram bf16 / bf16x3 timings + DRF collective bytes with the int32 / byte-based exchange
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/wide_gram_mb.py > gpurun_out/r5_wide_gram_mb3.txt 2>&1 || { tail -20 gpurun_out/r5_wide_gram_mb3.txt; exit 1; }
cat gpurun_out/r5_wide_gram_mb3.txt
bash scripts/r5_coll_drf.sh
