# A/B of an env knob: stamps at B=1440 + bench at 1440/720/180 for each setting
#   tools/r3_ab.sh TAG VAR VAL_A VAL_B
set -e
export TMPDIR=/tmp
tag=$1; var=$2; shift 2
mkdir -p gpurun_out
for v in "$@"; do
  env $var=$v PDRNN_LSTM_STAMPS=1 timeout -k 10 120 python bench.py --steps 3 --warmup 2 --global-batch 1440 > gpurun_out/${tag}_${v}_stamps.log 2>&1
  echo "== $var=$v"; grep -A2 "grid=1440" gpurun_out/${tag}_${v}_stamps.log | grep -v XCC | tail -3
  grep "bwd(" gpurun_out/${tag}_${v}_stamps.log | tail -1
  for B in 1440 720 180; do
    env $var=$v timeout -k 10 180 python bench.py --steps 200 --warmup 20 --global-batch $B > gpurun_out/${tag}_${v}_bench$B.log 2>&1
    tail -1 gpurun_out/${tag}_${v}_bench$B.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=$B', d['value'], d['ms_per_step'])"
  done
done
