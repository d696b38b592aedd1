set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_deeplearning.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dl.log 2>&1 || { tail -30 gpurun_out/pytest_dl.log; exit 1; }
tail -2 gpurun_out/pytest_dl.log
bash scripts/gpu_dl.sh
H2O3_DL_GRAPH=0 timeout -k 10 300 python bench.py --algo dl --rows 10000000 --batch 1024 --steps 200 --warmup 20 > gpurun_out/dl_nograph.log 2>&1
echo "no graph: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dl_nograph.log)"
