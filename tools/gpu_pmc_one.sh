#!/bin/bash
# One rocprofv3 counter pass (no trace domains) over a command, CSV summary.
#   tools/gpu_pmc_one.sh TAG "COUNTERS" -- cmd args...
set -e
tag=$1; ctr=$2; shift 3
export TMPDIR=/tmp
mkdir -p gpurun_out/$tag
root=$PWD
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d /tmp/pmc_$tag -o run -- "$@" > $root/gpurun_out/$tag/pass.log 2>&1
cd $root
find /tmp/pmc_$tag -name '*counter_collection*.csv' -exec cp {} gpurun_out/$tag/ \;
python3 tools/pmc_summary.py gpurun_out/$tag/summary.md gpurun_out/$tag > /dev/null
cat gpurun_out/$tag/summary.md
