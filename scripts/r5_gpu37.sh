#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_gpu_full37.log 2>&1
rc=$?
tail -3 gpurun_out/r5_gpu_full37.log
if [ $rc -ne 0 ]; then grep -E "FAILED|^E " gpurun_out/r5_gpu_full37.log | head -20; exit 1; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke37.log 2>&1 || { tail -20 gpurun_out/smoke37.log; exit 1; }
tail -2 gpurun_out/smoke37.log
timeout -k 10 500 python -u bench.py > gpurun_out/bench37.json 2> gpurun_out/bench37.err || { tail -20 gpurun_out/bench37.err; exit 1; }
cut -c1-300 gpurun_out/bench37.json
