#!/bin/bash
# Round-6 baseline (one gpurun call): the driver's bench line twice, a 200-step
# bench, and two PMC passes over a short bench run -- bytes (FETCH_SIZE /
# WRITE_SIZE, each in its own pass: TCC limit) beside the SQ counters that
# name each kernel's binding resource.
#   tools/gpu_r6_base.sh TAG
set -e
export TMPDIR=/tmp
tag=${1:-r6b}
out=gpurun_out/$tag
mkdir -p $out
for i in 1 2; do
  timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/drv$i.log 2>&1 || { tail -20 $out/drv$i.log; exit 1; }
  tail -1 $out/drv$i.log | python tools/bench_line.py "driver-style $i"
done
timeout -k 10 240 python bench.py --steps 200 --warmup 20 > $out/b200.log 2>&1 || { tail -20 $out/b200.log; exit 1; }
tail -1 $out/b200.log | python tools/bench_line.py "200 steps"
root=$PWD
cd /tmp
i=0
for set in "FETCH_SIZE SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVES" \
           "WRITE_SIZE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d /tmp/pmc_$i -o run -- python3 $root/bench.py --steps 10 --warmup 2 > $root/$out/pmc$i.log 2>&1
  mkdir -p $root/$out/p$i
  find /tmp/pmc_$i -name '*counter_collection*.csv' -exec cp {} $root/$out/p$i/ \;
done
cd $root
python3 tools/pmc_summary.py $out/summary.md $out/p1 $out/p2 > /dev/null
grep -E "lstm_sw|lstm_small_dw|slab" $out/summary.md | head -60
