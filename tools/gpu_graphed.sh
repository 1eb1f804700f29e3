# graphed autograd step: tests, then the fp32 H=128 benches (graph / eager) and a timeline
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-gr}
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread -k "graphed or fused_step_matches" > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
for cell in lstm gru; do
  PDRNN_CUDA_GRAPH=1 timeout -k 10 300 python bench.py --hidden 128 --cell $cell --steps 20 --warmup 10 > gpurun_out/${tag}_h128_$cell.log 2>&1 || { tail -20 gpurun_out/${tag}_h128_$cell.log; exit 1; }
  tail -1 gpurun_out/${tag}_h128_$cell.log | python tools/bench_line.py "H=128 fp32 $cell graphed"
  timeout -k 10 300 python bench.py --hidden 128 --cell $cell --steps 20 --warmup 10 > gpurun_out/${tag}_h128_${cell}_eager.log 2>&1 || { tail -20 gpurun_out/${tag}_h128_${cell}_eager.log; exit 1; }
  tail -1 gpurun_out/${tag}_h128_${cell}_eager.log | python tools/bench_line.py "H=128 fp32 $cell eager"
done
BENCH_ARGS="--warmup 10" bash tools/gpu_timeline.sh ${tag}_tl "PDRNN_CUDA_GRAPH=1"
