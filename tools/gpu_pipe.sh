# fp32 --hidden 128 stacked-layer pipeline (CELL=gru for the GRU): tests, then a bench A/B (one gpurun call):
#   bash tools/gpu_pipe.sh TAG "ENV1=... ENV2=..." ...   (the first run is the default)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-pipe}; shift
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_lstm_pipeline.py \
    tests/test_gpu_lstm_persist.py tests/test_gpu_lstm_large.py > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
  tail -1 gpurun_out/${tag}_tests.log
fi
i=0
for cfg in "" "$@"; do
  timeout -k 10 300 env $cfg python bench.py --hidden 128 --cell ${CELL:-lstm} --steps 20 --warmup 5 $BENCH_ARGS > gpurun_out/${tag}_$i.log 2>&1 || { tail -20 gpurun_out/${tag}_$i.log; exit 1; }
  tail -1 gpurun_out/${tag}_$i.log | python tools/bench_line.py "[$cfg]"
  i=$((i + 1))
done
