#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r5_eta_mb.txt
: > $o
timeout -k 10 200 python -u scripts/wide_eta_mb.py 768 1024 1536 2048 3072 4096 8192 >> $o 2>&1 || { cat $o; exit 1; }
H2O3_WIDE_RW=2 timeout -k 10 200 python -u scripts/wide_eta_mb.py 768 1024 2048 4096 >> $o 2>&1 || { cat $o; exit 1; }
MB_LDX=1024 timeout -k 10 200 python -u scripts/wide_eta_mb.py 1024 2048 4096 >> $o 2>&1 || { cat $o; exit 1; }
MB_P=1022 MB_LDX=1024 timeout -k 10 200 python -u scripts/wide_eta_mb.py 1024 2048 4096 >> $o 2>&1 || { cat $o; exit 1; }
grep -v amdgpu.ids $o
