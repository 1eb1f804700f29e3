#!/bin/bash
# slab reduction: A columns per workgroup 64 / 32 / 16 (kernel time at B = 1440 and 180)
set -e
export TMPDIR=/tmp
out=gpurun_out/${1:-redcw}
mkdir -p $out
timeout -k 10 400 env PDRNN_TUNE=reduce_cw=16 python -u -m pytest tests/test_gpu_train.py -x -q -k "headline_batch or seq_in_wave_step" --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for cw in 64 32 16; do
  for B in 1440 180; do
    cd /tmp && PDRNN_TUNE=reduce_cw=$cw timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/p_${cw}_$B -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --global-batch $B --epoch-sequences $((B * 24 / 5)) > $GRAFT_REPO_ROOT/$out/p_${cw}_$B.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$out/p_${cw}_$B.log; exit 1; }
    cd $GRAFT_REPO_ROOT
    python -c "import csv; r=[x for x in csv.DictReader(open('$out/p_${cw}_$B/run_kernel_stats.csv')) if 'slab_reduce' in x['Name']][0]; print('cw=$cw B=$B', round(float(r['AverageNs'])/1000, 2), 'us')"
  done
done
