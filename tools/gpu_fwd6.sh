set -e
mkdir -p gpurun_out
D=pytorch_distributed_rnn_amd/build_native/probe
for B in 360 512 720 900 1024; do timeout -k 10 120 $D/sw_probe $B 20 2 6 >> gpurun_out/fwd6_probe.log 2>&1; done
grep -h "^mode\|^B=" gpurun_out/fwd6_probe.log
