# fp32 large-H path (one gpurun call): GEMM / large LSTM / GRU / persistent
# tests, then the --hidden 128 fp32 benches and their kernel tables
#   tools/gpu_h128.sh TAG
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-h128}
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_coverage.py tests/test_gpu_gemm.py tests/test_gpu_lstm_large.py tests/test_gpu_gru_large.py tests/test_gpu_lstm_persist.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
for cell in lstm gru; do
  timeout -k 10 300 python bench.py --hidden 128 --cell $cell --steps 20 --warmup 5 > gpurun_out/${tag}_bench_$cell.log 2>&1 || { tail -20 gpurun_out/${tag}_bench_$cell.log; exit 1; }
  tail -1 gpurun_out/${tag}_bench_$cell.log | python tools/bench_line.py "H=128 fp32 $cell"
done
PDRNN_TUNE=large_overlap=0 timeout -k 10 300 python bench.py --hidden 128 --steps 20 --warmup 5 > gpurun_out/${tag}_bench_lstm_noovl.log 2>&1 || { tail -20 gpurun_out/${tag}_bench_lstm_noovl.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_lstm_noovl.log | python tools/bench_line.py "H=128 fp32 lstm, no cross-layer overlap"
for cell in 0 1; do
  timeout -k 10 120 python bench/persist_bench.py --hidden 128 --dtype fp32 --batch 1440 --seq 128 --cell $cell --tiles 0 1 2 4 > gpurun_out/${tag}_persist_f32_cell$cell.json 2> gpurun_out/${tag}_persist_f32_cell$cell.err || { tail -20 gpurun_out/${tag}_persist_f32_cell$cell.err; exit 1; }
  cat gpurun_out/${tag}_persist_f32_cell$cell.json
done
# A/B: two sequences per K-split forward workgroup at the headline batch
timeout -k 10 180 python bench.py --steps 200 --warmup 20 > gpurun_out/${tag}_b1440_nbf1.log 2>&1 || { tail -20 gpurun_out/${tag}_b1440_nbf1.log; exit 1; }
tail -1 gpurun_out/${tag}_b1440_nbf1.log | python tools/bench_line.py "B=1440 fwd NB=1"
PDRNN_TUNE=nb_fwd=2,split_fwd=2 timeout -k 10 180 python bench.py --steps 200 --warmup 20 > gpurun_out/${tag}_b1440_nbf2.log 2>&1 || { tail -20 gpurun_out/${tag}_b1440_nbf2.log; exit 1; }
tail -1 gpurun_out/${tag}_b1440_nbf2.log | python tools/bench_line.py "B=1440 fwd NB=2"
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread -k "gru" > gpurun_out/${tag}_gru_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_gru_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_gru_tests.log
timeout -k 10 180 python bench.py --cell gru --steps 200 --warmup 20 > gpurun_out/${tag}_gru1440.log 2>&1 || { tail -20 gpurun_out/${tag}_gru1440.log; exit 1; }
tail -1 gpurun_out/${tag}_gru1440.log | python tools/bench_line.py "GRU B=1440"
bash tools/gpu_tables.sh ${tag}tb
