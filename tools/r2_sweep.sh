set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench/gemm_tiles.py > gpurun_out/r2_gemm_tiles.log 2>&1
cat gpurun_out/r2_gemm_tiles.log
for b in 1024 2048; do
timeout -k 10 600 python bench/lm_bench.py --config charlm --batch $b --steps 6 --warmup 2 > gpurun_out/r2_charlm_b$b.log 2>&1
tail -1 gpurun_out/r2_charlm_b$b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('charlm B', d['config']['global_batch'], d['value'], d['ms_per_step'], d['device_peak_mib'])"
done
