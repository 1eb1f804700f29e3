set -e
mkdir -p gpurun_out
D=pytorch_distributed_rnn_amd/build_native/probe
for B in 97 180 256 360; do timeout -k 10 120 $D/sw_probe $B 20 4 8 >> gpurun_out/bwd5_probe.log 2>&1; done
grep -h "^mode\|^B=\|dW sum" gpurun_out/bwd5_probe.log
