set -e
export TMPDIR=/tmp
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_linalg_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_lin.log 2>&1 || { tail -30 gpurun_out/pytest_lin.log; exit 1; }
tail -n 1 gpurun_out/pytest_lin.log
for cfg in ${CFGS:-1:0 1:7 1:15 0:0 0:15}; do
  H2O3_GLM_BF3=${cfg%%:*} H2O3_GI_DBG=${cfg##*:} timeout -k 10 120 python scripts/glm_ws_mb.py 2>&1 | grep bf3 >> gpurun_out/glm_ws_mb.txt
done
cat gpurun_out/glm_ws_mb.txt
