# deferred-dW BPTT: one vs two sequences per workgroup at the headline batch
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-nb}
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
for nb in 1 2; do
  PDRNN_TUNE=dwout_nb=$nb timeout -k 10 180 python bench.py > gpurun_out/${tag}_bench_nb$nb.log 2>&1 || { tail -20 gpurun_out/${tag}_bench_nb$nb.log; exit 1; }
  tail -1 gpurun_out/${tag}_bench_nb$nb.log | python tools/bench_line.py "nb=$nb"
done
PDRNN_LSTM_STAMPS=1 PDRNN_TUNE=dwout_nb=2 timeout -k 10 180 python bench.py --steps 10 --warmup 2 > gpurun_out/${tag}_stamps.log 2>&1 || { tail -20 gpurun_out/${tag}_stamps.log; exit 1; }
grep "stamps\] bwd" gpurun_out/${tag}_stamps.log | tail -2
timeout -k 10 300 python -u -m pytest tests/test_gpu_lstm_persist.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_persist_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_persist_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_persist_tests.log
for v in 0 1; do
  PDRNN_LSTM_PERSIST_VERIFY=$v timeout -k 10 300 python bench/lm_bench.py --config charlm --steps 10 --warmup 3 > gpurun_out/${tag}_charlm_verify$v.log 2>&1 || { tail -20 gpurun_out/${tag}_charlm_verify$v.log; exit 1; }
  echo "verify=$v $(tail -1 gpurun_out/${tag}_charlm_verify$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['persist_verify'], d['persist_fallbacks'])")"
done
