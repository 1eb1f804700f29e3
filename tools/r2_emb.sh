set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lstm_large.py -x -q -k "embedding" --timeout 120 --timeout-method thread > gpurun_out/r2_emb_tests.log 2>&1
tail -2 gpurun_out/r2_emb_tests.log
timeout -k 10 200 python -u bench/lm_bench.py --config charlm --steps 5 --warmup 2 > gpurun_out/r2_persist_charlm2.log 2>&1
tail -1 gpurun_out/r2_persist_charlm2.log
