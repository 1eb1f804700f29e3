#!/bin/bash
# Build (here, on the CPU) or run (on the GPU box) the stand-alone
# sequence-in-wave kernel probe (bench/sw_probe.cpp).
#   bench/sw_probe.sh build
#   bench/sw_probe.sh run TAG [B...]
set -e
cd "$(dirname "$0")/.."
K=pytorch_distributed_rnn_amd/csrc/kernels
OUT=pytorch_distributed_rnn_amd/build_native/probe
if [ "$1" = build ]; then
  mkdir -p $OUT
  FL="-O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -Ipytorch_distributed_rnn_amd/csrc/include ${PROBE_FLAGS}"
  # the two kernel files under study always rebuild (PROBE_FLAGS diagnostics);
  # the gate-split family only when its source changed
  # SW_SRC: an alternative lstm_sw.hip (A/B against another revision)
  /opt/rocm/bin/hipcc -c $FL -mllvm -amdgpu-mfma-vgpr-form=1 ${SW_SRC:-$K/lstm_sw.hip} -o $OUT/lstm_sw.o 2>/dev/null &
  for f in lstm_small lstm_small_dw; do
    if [ ! -f $OUT/$f.o ] || [ $K/$f.hip -nt $OUT/$f.o ]; then
      /opt/rocm/bin/hipcc -c -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics \
        -Ipytorch_distributed_rnn_amd/csrc/include $K/$f.hip -o $OUT/$f.o 2>/dev/null &
    fi
  done
  /opt/rocm/bin/hipcc -c $FL bench/sw_probe.cpp -o $OUT/sw_probe.o 2>/dev/null &
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 $OUT/*.o -o $OUT/${PROBE_NAME:-sw_probe}
  echo built $OUT/${PROBE_NAME:-sw_probe}
  exit 0
fi
tag=${2:-sw}
shift 2 || true
mkdir -p gpurun_out
for B in ${@:-180 1440}; do
  timeout -k 10 120 $OUT/sw_probe $B 20 >> gpurun_out/${tag}_probe.log 2>&1 || { cat gpurun_out/${tag}_probe.log; exit 1; }
done
cat gpurun_out/${tag}_probe.log
