# kernel timeline (start / end / queue) of fp32 --hidden 128 training steps:
#   bash tools/gpu_timeline.sh TAG "ENV=..." ...   (one profile per configuration)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-tl}; shift
i=0
for cfg in "" "$@"; do
  for kv in $cfg; do export "$kv"; done
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_${tag}_$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --hidden 128 --steps 10 --warmup 5 $BENCH_ARGS > $GRAFT_REPO_ROOT/gpurun_out/${tag}_$i.log 2>&1)
  for kv in $cfg; do unset "${kv%%=*}"; done
  db=$(find /tmp/prof_${tag}_$i -name '*.db' | head -1)
  python tools/prof_window.py "$db" --anchor xent_rows --skip 8 --first 4 --timeline 1 --out gpurun_out/${tag}_${i}_timeline.md > /dev/null
  echo "[$cfg]"; head -3 gpurun_out/${tag}_${i}_timeline.md
  i=$((i + 1))
done
