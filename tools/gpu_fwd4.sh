set -e
mkdir -p gpurun_out
D=pytorch_distributed_rnn_amd/build_native/probe
for B in 97 180 360 512 720 1024; do timeout -k 10 120 $D/sw_probe $B 20 2 5 >> gpurun_out/fwd4_probe.log 2>&1; done
grep -h "^mode\|^B=" gpurun_out/fwd4_probe.log
