set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_bilstm%d.csv PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=300 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=100
timeout -k 10 900 python bench/lm_bench.py --config bilstm --batch 4096 --steps 5 --warmup 2 > gpurun_out/r2t_bilstm_tune.log 2>&1
tail -1 gpurun_out/r2t_bilstm_tune.log | cut -c1-250
export PYTORCH_TUNABLEOP_TUNING=0
timeout -k 10 600 python bench/lm_bench.py --config bilstm --batch 4096 --steps 5 --warmup 2 > gpurun_out/r2t_bilstm_tuned.log 2>&1
tail -1 gpurun_out/r2t_bilstm_tuned.log | cut -c1-250
ls -la gpurun_out/ | grep tunable
