set -e
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1
tail -1 gpurun_out/bench_default.log | cut -c1-300
timeout -k 10 400 python bench.py --algo glm --steps 10 --warmup 2 > gpurun_out/bench_glm_default.log 2>&1
tail -1 gpurun_out/bench_glm_default.log | cut -c1-300
bash scripts/profile_bench.sh gpurun_out/rocprof_gbm100m
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof_glm100m -o run --output-format csv -- python3 bench.py --algo glm --steps 5 --warmup 1 > gpurun_out/rocprof_glm100m.log 2>&1
tail -n 1 gpurun_out/rocprof_glm100m.log | cut -c1-200
