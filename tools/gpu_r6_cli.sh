#!/bin/bash
# where the CLI's one-epoch Training Duration goes (PDRNN_EPOCH_TIMELINE)
set -e
export TMPDIR=/tmp
out=gpurun_out/cli6
mkdir -p $out
for tr in local distributed horovod; do
  for i in 1 2; do
    if [ $tr = local ]; then
      PDRNN_EPOCH_TIMELINE=1 timeout -k 10 120 python src/motion/main.py --batch-size 1440 --epochs 1 --seed 123456789 --no-validation --synthetic local > $out/${tr}$i.log 2>&1
    else
      PDRNN_EPOCH_TIMELINE=1 timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=2950$i src/motion/main.py --batch-size 1440 --epochs 1 --seed 123456789 --no-validation --synthetic $tr > $out/${tr}$i.log 2>&1
    fi
    echo "== $tr $i"; grep -E "timeline|Training Duration" $out/${tr}$i.log | sed 's/.*\] //' | head -40
  done
done
