# PMC counters of the one-launch step (B=180) and the headline step (B=1440)
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc2 /tmp/pmc2
passes=(
 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
 "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA"
 "FETCH_SIZE"
 "WRITE_SIZE"
)
dirs=""
for B in 180 1440; do
  i=0
  for p in "${passes[@]}"; do
    i=$((i+1))
    cd /tmp
    timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d /tmp/pmc2/b${B}_p$i -o run -- python3 $R/bench.py --steps 3 --warmup 2 --global-batch $B > $R/gpurun_out/pmc2/b${B}_p$i.log 2>&1
    cd $R
    dirs="$dirs /tmp/pmc2/b${B}_p$i"
  done
done
python tools/pmc_summary.py gpurun_out/pmc2/summary.md $dirs
echo pmc-done
