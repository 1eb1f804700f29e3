set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2p_tests.log 2>&1 || { tail -30 gpurun_out/r2p_tests.log; exit 1; }
tail -1 gpurun_out/r2p_tests.log
for e in 1 3; do
  timeout -k 10 180 python src/motion/main.py --epochs $e --seed 123456789 --no-validation --synthetic local > gpurun_out/r2p_cli_e$e.log 2>&1
  grep "Warm-up\|Training Duration" gpurun_out/r2p_cli_e$e.log
done
timeout -k 10 180 python src/motion/main.py --epochs 1 --seed 123456789 --no-validation --synthetic --no-warmup local > gpurun_out/r2p_cli_nowarm.log 2>&1
grep "Training Duration" gpurun_out/r2p_cli_nowarm.log
for i in 1 2 3; do timeout -k 10 180 python bench.py --steps 20 --warmup 5 > gpurun_out/r2p_bench_driver$i.log 2>&1; tail -1 gpurun_out/r2p_bench_driver$i.log | cut -c1-190; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_ps.py -x -v --timeout 150 --timeout-method thread > gpurun_out/r2p_ps.log 2>&1 || { tail -60 gpurun_out/r2p_ps.log; exit 1; }
tail -4 gpurun_out/r2p_ps.log
