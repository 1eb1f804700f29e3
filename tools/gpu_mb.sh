set -e
mkdir -p gpurun_out
P=pytorch_distributed_rnn_amd/build_native/probe/sw_probe
timeout -k 10 120 $P 1440 20 3 7 >> gpurun_out/mb11_probe.log 2>&1
timeout -k 10 120 $P 720 20 2 7 >> gpurun_out/mb11_probe.log 2>&1
timeout -k 10 120 $P 180 20 2 7 >> gpurun_out/mb11_probe.log 2>&1
