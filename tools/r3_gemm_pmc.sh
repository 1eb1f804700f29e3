# PMC passes over bench/gemm_pmc_driver.py (in-tree NTxNT / KMxKM GEMM vs hipBLASLt)
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
tag=${1:-r3gp}
mkdir -p $R/gpurun_out/$tag /tmp/$tag
passes=(
 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_F16"
 "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES"
 "FETCH_SIZE"
 "TCC_HIT_sum TCC_MISS_sum"
)
dirs=""
i=0
for p in "${passes[@]}"; do
  i=$((i+1))
  cd /tmp
  timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d /tmp/$tag/p$i -o run -- python3 $R/bench/gemm_pmc_driver.py > $R/gpurun_out/$tag/p$i.log 2>&1
  cd $R
  dirs="$dirs /tmp/$tag/p$i"
done
python tools/pmc_summary.py gpurun_out/$tag/summary.md $dirs --match "gemm|Cijk"
cat gpurun_out/$tag/summary.md
