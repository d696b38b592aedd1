# GLM fused-pass phase sweep (debug bits: 1 no MFMA, 2 no X loads, 4 no y/w loads, 8 no eta).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for D in 0 1 2 3 8 11 15; do
  PYTHONPATH=. H2O3_GI_DBG=$D timeout -k 10 120 python scripts/glm_ws_mb.py >> gpurun_out/glm_dbg_sweep.txt 2>&1
done
grep "ms/pass" gpurun_out/glm_dbg_sweep.txt
