set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 python bench/step_profile.py --steps 80 > gpurun_out/r2_stepprof.log 2>&1
cat gpurun_out/r2_stepprof.log | tail -1 | tr ' ' '\n' | awk '{a[NR]=$1} END {for(i=1;i<=NR;i+=10){s=0;n=0;for(j=i;j<i+10&&j<=NR;j++){s+=a[j];n++}; printf "steps %d-%d mean %.3f ms\n", i, i+n-1, s/n}}'
for e in 1 3; do
  timeout -k 10 180 python src/motion/main.py --epochs $e --seed 123456789 --no-validation --synthetic local > gpurun_out/r2_cli_e$e.log 2>&1
  grep "Training Duration\|Throughput" gpurun_out/r2_cli_e$e.log
done
timeout -k 10 900 python bench/lm_bench.py --config bilstm --batch 11264 --steps 3 --warmup 1 > gpurun_out/r2_bilstm_b11264.log 2>&1 || tail -5 gpurun_out/r2_bilstm_b11264.log
tail -1 gpurun_out/r2_bilstm_b11264.log | cut -c1-500
