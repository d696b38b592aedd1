# DL step throughput (10M x 100, MLP 200-200) at two batch sizes + rocprof stats.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for B in 1024 4096; do
  timeout -k 10 300 python bench.py --algo dl --rows 10000000 --batch $B --steps 400 --warmup 20 > gpurun_out/dl_b$B.log 2>&1
  echo "batch=$B $(grep -o '"value": [0-9.]*' gpurun_out/dl_b$B.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dl_b$B.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dl -o dl --output-format csv -- python bench.py --algo dl --rows 10000000 --batch 1024 --steps 100 --warmup 10 > gpurun_out/dl_prof.log 2>&1
cp gpurun_out/prof_dl/dl_kernel_stats.csv gpurun_out/dl_kernel_stats.csv
head -14 gpurun_out/dl_kernel_stats.csv | cut -c1-160
