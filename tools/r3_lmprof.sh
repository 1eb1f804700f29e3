# kernel tables of the char-LM and bi-LSTM benches (rocprofv3 --kernel-trace --stats)
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
tag=${1:-r3lp}
mkdir -p $R/gpurun_out/$tag
for cfg in charlm bilstm; do
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/$tag/$cfg -o run -- python3 $R/bench/lm_bench.py --config $cfg --steps 3 --warmup 1 > $R/gpurun_out/$tag/$cfg.log 2>&1
  cd $R
  db=$(find /tmp/$tag/$cfg -name '*.db' | head -1)
  python tools/prof_summary.py "$db" --out gpurun_out/$tag/${cfg}_kernel_stats.md > /dev/null
  tail -1 gpurun_out/$tag/$cfg.log | cut -c1-220
  head -16 gpurun_out/$tag/${cfg}_kernel_stats.md | cut -c1-160
done
