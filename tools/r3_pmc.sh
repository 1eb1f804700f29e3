# PMC counters of the fused step's kernels at one batch (4 passes) + in-kernel loop stamps.
#   tools/r3_pmc.sh TAG BATCH
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
tag=${1:-r3p}; B=${2:-1440}
mkdir -p $R/gpurun_out/$tag /tmp/$tag
passes=(
 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
 "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA"
 "FETCH_SIZE"
 "WRITE_SIZE"
)
dirs=""
i=0
for p in "${passes[@]}"; do
  i=$((i+1))
  cd /tmp
  timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d /tmp/$tag/p$i -o run -- python3 $R/bench.py --steps 3 --warmup 2 --global-batch $B > $R/gpurun_out/$tag/p$i.log 2>&1
  cd $R
  dirs="$dirs /tmp/$tag/p$i"
done
python tools/pmc_summary.py gpurun_out/$tag/summary.md $dirs
PDRNN_LSTM_STAMPS=1 timeout -k 10 120 python bench.py --steps 3 --warmup 2 --global-batch $B > gpurun_out/$tag/stamps.log 2>&1
grep stamps gpurun_out/$tag/stamps.log | tail -4
