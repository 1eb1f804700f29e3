# comm-stream overlap evidence with the bucketed reducer forced through RCCL at one rank.
#   tools/r3_overlap.sh bilstm   -- plain vs --ddp throughput, then a kernel trace
#   tools/r3_overlap.sh charlm   -- kernel trace (persistent recurrence + bucket all-reduces)
# rocprofv3 has been seen to SIGSEGV in exit() AFTER writing its database for runs that hold
# an RCCL communicator: the trace step is the LAST GPU step of the call; the stream analysis
# after it is CPU-only (sqlite).
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cfg=${1:-bilstm}
mkdir -p $R/gpurun_out
if [ "$cfg" = bilstm ]; then
  timeout -k 10 300 python bench/lm_bench.py --config bilstm --steps 4 --warmup 1 > gpurun_out/r3ov_bilstm_plain.log 2>&1
  PDRNN_FORCE_COLLECTIVE=1 timeout -k 10 300 python bench/lm_bench.py --config bilstm --steps 4 --warmup 1 --ddp > gpurun_out/r3ov_bilstm_ddp.log 2>&1
  tail -1 gpurun_out/r3ov_bilstm_plain.log | cut -c1-200
  tail -1 gpurun_out/r3ov_bilstm_ddp.log | cut -c1-200
fi
cd /tmp
rc=0
PDRNN_FORCE_COLLECTIVE=1 timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/ov_$cfg -o run -- python3 $R/bench/lm_bench.py --config $cfg --steps 2 --warmup 1 --ddp > $R/gpurun_out/r3ov_${cfg}_prof.log 2>&1 || rc=$?
cd $R
echo "profiler exit status $rc (no further GPU step in this call)"
db=$(find /tmp/ov_$cfg -name '*.db' | head -1)
[ -n "$db" ] && python tools/prof_streams.py "$db" --match "rccl|nccl|Reduce|allreduce" --out gpurun_out/r3ov_${cfg}_streams.md > /dev/null
exit $rc
