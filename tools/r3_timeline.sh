set -e
export TMPDIR=/tmp
for B in 480 1440; do
  PDRNN_EPOCH_TIMELINE=1 timeout -k 10 120 python src/motion/main.py --epochs 1 --seed 123456789 --no-validation --synthetic --batch-size $B local > gpurun_out/r3tl_$B.log 2>&1
  echo "== local $B"; grep "timeline\|Training Duration" gpurun_out/r3tl_$B.log | grep -v "batch[1-9]" | tail -12
done
PDRNN_EPOCH_TIMELINE=1 timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29611 src/motion/main.py --epochs 1 --seed 123456789 --no-validation --synthetic --batch-size 480 distributed > gpurun_out/r3tl_d480.log 2>&1
echo "== distributed 480"; grep "timeline\|Training Duration" gpurun_out/r3tl_d480.log | tail -40
