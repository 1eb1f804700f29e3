set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python bench.py --layers 1 --dtype bf16 --steps 200 --warmup 20 > gpurun_out/cfg2_bf16_1x32.log 2>&1
tail -1 gpurun_out/cfg2_bf16_1x32.log
timeout -k 10 120 python bench.py --layers 1 --steps 200 --warmup 20 > gpurun_out/cfg2_fp32_1x32.log 2>&1
tail -1 gpurun_out/cfg2_fp32_1x32.log
timeout -k 10 120 python bench.py --dtype bf16 --steps 200 --warmup 20 > gpurun_out/cfg2_bf16_2x32.log 2>&1
tail -1 gpurun_out/cfg2_bf16_2x32.log
