# GPU loop (one gpurun call): fused-step tests, the bench at the 1/2/4/8-GPU
# per-rank batches, the forced-collective graph-replayed synced step, and a
# kernel-trace window of the default bench.
#   tools/gpu_check.sh TAG [quick|full]
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-chk}
mode=${2:-quick}
if [ "$mode" = full ]; then
  timeout -k 10 1500 python -u -m pytest tests -m gpu --maxfail=10 -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_gpu_tests.log; exit 1; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
  tail -1 gpurun_out/${tag}_smoke.log
else
  timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_kernels.py tests/test_gpu_comm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_gpu_tests.log; exit 1; }
fi
tail -1 gpurun_out/${tag}_gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 1; }
tail -1 gpurun_out/${tag}_bench.log | cut -c1-400
# config 2 (bf16 motion) and the GRU cell at the headline shape
timeout -k 10 300 python bench.py --dtype bf16 > gpurun_out/${tag}_bench_bf16.log 2>&1 || { tail -20 gpurun_out/${tag}_bench_bf16.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_bf16.log | python tools/bench_line.py "bf16"
timeout -k 10 300 python bench.py --layers 1 --dtype bf16 > gpurun_out/${tag}_bench_bf16_l1.log 2>&1 || { tail -20 gpurun_out/${tag}_bench_bf16_l1.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_bf16_l1.log | python tools/bench_line.py "bf16 1 layer (config 2)"
timeout -k 10 300 python bench.py --layers 1 > gpurun_out/${tag}_bench_fp32_l1.log 2>&1 || { tail -20 gpurun_out/${tag}_bench_fp32_l1.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_fp32_l1.log | python tools/bench_line.py "fp32 1 layer"
timeout -k 10 300 python bench.py --cell gru > gpurun_out/${tag}_bench_gru.log 2>&1 || { tail -20 gpurun_out/${tag}_bench_gru.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_gru.log | python tools/bench_line.py "gru"
for B in 1440 720 360 180; do
  timeout -k 10 180 python bench.py --steps 200 --warmup 20 --global-batch $B > gpurun_out/${tag}_bench$B.log 2>&1 || { tail -20 gpurun_out/${tag}_bench$B.log; exit 1; }
  tail -1 gpurun_out/${tag}_bench$B.log | python tools/bench_line.py "B=$B eager"
done
# one rank's epoch of the 2/4/8-GPU run (per-rank batch B, 6912 / N sequences),
# synced step (forced one-rank RCCL all-reduce + Adam) replayed per epoch
for B in 720 360 180; do
  E=$((B * 24 / 5))
  PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1 timeout -k 10 180 python bench.py --steps 200 --warmup 20 --global-batch $B --epoch-sequences $E --cuda-graph > gpurun_out/${tag}_synced$B.log 2>&1 || { tail -20 gpurun_out/${tag}_synced$B.log; exit 1; }
  tail -1 gpurun_out/${tag}_synced$B.log | python tools/bench_line.py "B=$B synced-graph"
done
# the GRU's synced step, graph-replayed per epoch
PDRNN_FORCE_GRAD_SYNC=1 PDRNN_FORCE_COLLECTIVE=1 timeout -k 10 180 python bench.py --cell gru --steps 200 --warmup 20 --global-batch 180 --epoch-sequences 864 --cuda-graph > gpurun_out/${tag}_synced180_gru.log 2>&1 || { tail -20 gpurun_out/${tag}_synced180_gru.log; exit 1; }
tail -1 gpurun_out/${tag}_synced180_gru.log | python tools/bench_line.py "GRU B=180 synced-graph"
bash tools/gpu_windows.sh ${tag}
