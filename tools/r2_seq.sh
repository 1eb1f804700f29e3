set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/prof_seq -o run -- python3 bench.py --steps 50 --warmup 10 > gpurun_out/seq_prof.log 2>&1
db=$(find /tmp/prof_seq -name '*.db' | head -1)
python tools/prof_seq.py "$db" lstm_small_bwd_gs_kernel 30 2 > gpurun_out/seq_steps.txt
python tools/prof_seq.py "$db" lstm_small_bwd_gs_kernel 61 3 >> gpurun_out/seq_steps.txt
cat gpurun_out/seq_steps.txt | head -80
