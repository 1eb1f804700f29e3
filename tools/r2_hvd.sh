# horovod trainer on the fused flat-Adam path: multirank oracle + 1-GPU CLI epochs
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2_hvd_tests.log 2>&1
tail -2 gpurun_out/r2_hvd_tests.log
for b in 480 960 1440; do
  timeout -k 10 120 python src/motion/main.py --epochs 1 --batch-size $b --no-validation --synthetic horovod > gpurun_out/r2_hvd_$b.log 2>&1
  grep -h "Training Duration\|seq/s" gpurun_out/r2_hvd_$b.log | tail -2
done
