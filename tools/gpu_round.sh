# everything one GPU round trip can check (stops at the first failure):
# large-H tests + LM benches, large-H kernel tables, motion tests + benches
# (eager per-GPU batches, synced epoch graphs) + kernel window
#   tools/gpu_round.sh TAG
set -e
tag=${1:-rd}
bash tools/gpu_lm.sh ${tag}lm
bash tools/gpu_check.sh ${tag} quick
bash tools/gpu_tables.sh ${tag}tb
