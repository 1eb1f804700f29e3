# kernel table of one LM bench config (rocprofv3 --kernel-trace --stats); the trace is the LAST GPU
# step of the call (rocprofv3 has been seen to SIGSEGV in exit() after writing its database), the
# table is built CPU-only afterwards.   tools/r3_lmprof.sh TAG charlm|bilstm
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
tag=${1:-r3lp}; cfg=${2:-charlm}
mkdir -p $R/gpurun_out/$tag
if [ -z "$NOBENCH" ]; then
  timeout -k 10 300 python bench/lm_bench.py --config $cfg --steps 6 --warmup 2 > gpurun_out/$tag/${cfg}_bench.log 2>&1
  tail -1 gpurun_out/$tag/${cfg}_bench.log | cut -c1-220
fi
cd /tmp
rc=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/$tag/$cfg -o run -- python3 $R/bench/lm_bench.py --config $cfg --steps 3 --warmup 1 > $R/gpurun_out/$tag/${cfg}_prof.log 2>&1 || rc=$?
cd $R
echo "profiler exit status $rc (no further GPU step in this call)"
db=$(find /tmp/$tag/$cfg -name '*.db' | head -1)
[ -n "$db" ] && python tools/prof_summary.py "$db" --out gpurun_out/$tag/${cfg}_kernel_stats.md > /dev/null && head -18 gpurun_out/$tag/${cfg}_kernel_stats.md | cut -c1-150
exit 0
