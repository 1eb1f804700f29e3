# PMC counters + timing ablations of the small-H motion kernels (B=180 and 1440).
# Raw profiler output stays in /tmp on the box; only summaries land in gpurun_out/.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc /tmp/pmc
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
    timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d /tmp/pmc/b${B}_p$i -o run -- python3 $R/bench.py --steps 3 --warmup 2 --global-batch $B > $R/gpurun_out/pmc/b${B}_p$i.log 2>&1
    cd $R
    dirs="$dirs /tmp/pmc/b${B}_p$i"
  done
done
python tools/pmc_summary.py gpurun_out/pmc/summary.md $dirs
echo pmc-done
for bits in 0 32 64 128 1 2 4 8 16; do
  PDRNN_HIP_EXTRA_FLAGS="-DPDRNN_ABLATE=$bits" timeout -k 10 300 python -m pytorch_distributed_rnn_amd._build > /dev/null
  echo "ablate=$bits" >> gpurun_out/pmc/ablate.log
  timeout -k 10 120 python bench/stamps.py 180,1440 >> gpurun_out/pmc/ablate.log 2>&1
done
grep -c stamps gpurun_out/pmc/ablate.log
du -sh gpurun_out
