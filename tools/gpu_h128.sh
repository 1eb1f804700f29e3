# fp32 large-H path (one gpurun call): GEMM / large LSTM / GRU / persistent
# tests, then the --hidden 128 fp32 benches and their kernel tables
#   tools/gpu_h128.sh TAG
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-h128}
timeout -k 10 900 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_lstm_large.py tests/test_gpu_gru_large.py tests/test_gpu_lstm_persist.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
for cell in lstm gru; do
  timeout -k 10 300 python bench.py --hidden 128 --cell $cell --steps 20 --warmup 5 > gpurun_out/${tag}_bench_$cell.log 2>&1 || { tail -20 gpurun_out/${tag}_bench_$cell.log; exit 1; }
  tail -1 gpurun_out/${tag}_bench_$cell.log | python tools/bench_line.py "H=128 fp32 $cell"
done
bash tools/gpu_tables.sh ${tag}tb
