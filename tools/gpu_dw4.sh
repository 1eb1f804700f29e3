set -e
mkdir -p gpurun_out
P=pytorch_distributed_rnn_amd/build_native/probe/sw_probe
for B in 180 360 512; do timeout -k 10 120 $P $B 20 2 4 >> gpurun_out/dw4_probe.log 2>&1; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_train.py -k "seq_in_wave" > gpurun_out/dw4_tests.log 2>&1
