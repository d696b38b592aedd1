#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5_gpu_full28.log 2>&1
rc=$?
tail -5 gpurun_out/r5_gpu_full28.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|error" gpurun_out/r5_gpu_full28.log | head -20; exit 1; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke28.log 2>&1 || { tail -20 gpurun_out/smoke28.log; exit 1; }
tail -3 gpurun_out/smoke28.log
