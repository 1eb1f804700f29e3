#!/bin/bash
# PMC passes (rocprofv3, counters only: no trace domains) over the stand-alone
# sequence-in-wave probe.  tools/gpu_sw_pmc.sh TAG B MODE
set -e
tag=${1:-pmc}; B=${2:-1440}; M=${3:-2}
export TMPDIR=/tmp
mkdir -p gpurun_out/$tag
P=$PWD/pytorch_distributed_rnn_amd/build_native/probe/sw_probe
cd /tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_WR" \
           "SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d /tmp/pmc_$i -o run -- $P $B 3 $M > $GRAFT_REPO_ROOT/gpurun_out/$tag/pass$i.log 2>&1 || [ $i = 3 ]
  mkdir -p $GRAFT_REPO_ROOT/gpurun_out/$tag/p$i
  find /tmp/pmc_$i -name '*counter_collection*.csv' -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/$tag/p$i/ \;
done
cd $GRAFT_REPO_ROOT
python3 tools/pmc_summary.py gpurun_out/$tag/summary.md gpurun_out/$tag/p1 gpurun_out/$tag/p2 gpurun_out/$tag/p3 > /dev/null 2>&1 || true
cat gpurun_out/$tag/summary.md | head -60
