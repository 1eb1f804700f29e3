# PMC counters of the persistent large-H recurrence kernels (char-LM layer shape, bench/persist_bench.py)
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmcp /tmp/pmcp
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
  timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d /tmp/pmcp/p$i -o run -- python3 $R/bench/persist_bench.py --reps 1 --seq 128 > $R/gpurun_out/pmcp/p$i.log 2>&1
  cd $R
  dirs="$dirs /tmp/pmcp/p$i"
done
python tools/pmc_summary.py gpurun_out/pmcp/summary.md --match "persist|lstm_large" $dirs
echo pmc-done
