set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/fprof
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/fprof -o run -- python3 bench.py --steps 25 --warmup 5 > gpurun_out/fprof_bench.log 2>&1
timeout -k 10 180 python bench.py --dtype bf16 --layers 1 --steps 200 --warmup 20 > gpurun_out/f_bench_bf16_1l.log 2>&1
timeout -k 10 180 python bench.py --global-batch 180 --steps 200 --warmup 20 > gpurun_out/f_bench_b180.log 2>&1
find gpurun_out/fprof -maxdepth 3 | head -20
tail -1 gpurun_out/f_bench_bf16_1l.log; tail -1 gpurun_out/f_bench_b180.log
