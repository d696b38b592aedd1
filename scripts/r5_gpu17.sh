#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/glm_devsolve_mb.py 1001 > gpurun_out/r5_devsolve.txt 2>&1 || { cat gpurun_out/r5_devsolve.txt; exit 1; }
cat gpurun_out/r5_devsolve.txt
timeout -k 10 200 python -u scripts/glm_devsolve_mb.py 101 > gpurun_out/r5_devsolve101.txt 2>&1 || { cat gpurun_out/r5_devsolve101.txt; exit 1; }
cat gpurun_out/r5_devsolve101.txt
