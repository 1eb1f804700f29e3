set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_lstm_large.py tests/test_gpu_lstm_pipeline.py tests/test_gpu_coverage.py tests/test_gpu_gru_large.py -x -q --timeout 200 --timeout-method thread > gpurun_out/h128b_tests.log 2>&1 || { tail -30 gpurun_out/h128b_tests.log; exit 1; }
tail -1 gpurun_out/h128b_tests.log
for cell in lstm gru; do
  timeout -k 10 300 python bench.py --hidden 128 --cell $cell --steps 20 --warmup 10 > gpurun_out/h128b_$cell.log 2>&1
  tail -1 gpurun_out/h128b_$cell.log | python tools/bench_line.py "H=128 fp32 $cell"
done
D=pytorch_distributed_rnn_amd/build_native/probe
for B in 360 512 720 900 1024; do timeout -k 10 120 $D/sw_probe $B 20 2 6 >> gpurun_out/fwd6_probe.log 2>&1; done
grep -h "^mode\|^B=" gpurun_out/fwd6_probe.log
