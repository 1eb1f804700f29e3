set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench/lm_bench.py --config charlm --steps 10 --warmup 2 > gpurun_out/r2k_charlm_b128.log 2>&1
tail -1 gpurun_out/r2k_charlm_b128.log
timeout -k 10 300 python bench/lm_bench.py --config bilstm --steps 3 --warmup 1 > gpurun_out/r2k_bilstm_b4096.log 2>&1
tail -1 gpurun_out/r2k_bilstm_b4096.log
