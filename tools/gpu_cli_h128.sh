# end-to-end CLI training at --hidden-units 128 fp32 (LSTM and GRU), with the
# stacked-layer pipeline on and off: loss / accuracy logs (one gpurun call)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-cli}
for cell in lstm gru; do
  for pipe in 1 0; do
    PDRNN_TUNE=large_pipe=$pipe timeout -k 10 300 python -m pytorch_distributed_rnn_amd.cli --synthetic --hidden-units 128 \
      --cell $cell --epochs 40 --seed 1 --checkpoint-directory /tmp/ckpt_${tag}_${cell}_$pipe local \
      > gpurun_out/${tag}_${cell}_pipe$pipe.log 2>&1 || { tail -20 gpurun_out/${tag}_${cell}_pipe$pipe.log; exit 1; }
    echo "== $cell pipe=$pipe"; grep -E "Evaluation Epoch|Training Duration|Test Evaluation" gpurun_out/${tag}_${cell}_pipe$pipe.log | tail -3
  done
done
