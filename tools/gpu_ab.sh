# headline-batch A/B of launch-geometry overrides (one gpurun call):
#   tools/gpu_ab.sh TAG "ENV1=..." "ENV2=..." ...   (the first run is the default)
#   BENCH_ARGS="--global-batch 180 --epoch-sequences 864" tools/gpu_ab.sh ...  (other shapes)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-ab}; shift
i=0
for cfg in "" "$@"; do
  timeout -k 10 180 env $cfg python bench.py --steps 200 --warmup 20 $BENCH_ARGS > gpurun_out/${tag}_$i.log 2>&1 || { tail -20 gpurun_out/${tag}_$i.log; exit 1; }
  tail -1 gpurun_out/${tag}_$i.log | python tools/bench_line.py "[$cfg]"
  i=$((i + 1))
done
