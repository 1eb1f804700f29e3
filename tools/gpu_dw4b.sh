set -e
mkdir -p gpurun_out
P=pytorch_distributed_rnn_amd/build_native/probe/sw_probe
for B in 600 720 1024 1440; do timeout -k 10 120 $P $B 20 2 3 4 >> gpurun_out/dw4b_probe.log 2>&1; done
