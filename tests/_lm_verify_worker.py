"""Worker of tests/test_gpu_multirank.py::test_two_rank_deferred_persist_verification:
one rank of a 2-rank char-LM job on a shared GPU (gloo), 3 training steps.
With PDRNN_TEST_INJECT_RANK=r, rank r flags its first persistent launch as
timed out; every rank must then skip its Adam update on the device and
re-run the skipped steps (train/lm.py settle).  Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_rnn_amd import _ext  # noqa: E402
from pytorch_distributed_rnn_amd.data.charlm import CharCorpus  # noqa: E402
from pytorch_distributed_rnn_amd.models.charlm import CharLM  # noqa: E402
from pytorch_distributed_rnn_amd.parallel import env  # noqa: E402
from pytorch_distributed_rnn_amd.train.lm import LMTrainer  # noqa: E402


def main():
    torch.manual_seed(0)
    corpus = CharCorpus.synthetic(200_000, seed=3)
    model = CharLM(256, 64, 1024, 1, compute_dtype=torch.bfloat16)
    tr = LMTrainer(model, corpus, global_batch=32, seq_len=32, device=torch.device("cuda", 0),
                   distributed=True, backend="gloo", log_interval=0)
    mod = _ext.require()
    segs = list(CharCorpus.segments(tr.streams, 32, 3))
    tr.inner.reset_hidden_state()
    inject = int(os.environ.get("PDRNN_TEST_INJECT_RANK", "-1"))
    if inject == tr.rank:
        mod.persist_inject_timeouts(1)
    losses = [tr.train_step(inp, tgt) for inp, tgt in segs]
    tr.settle()
    torch.cuda.synchronize()
    flat = torch.cat([p.detach().double().reshape(-1) for p in tr.inner.parameters()])
    rec = json.dumps({"rank": tr.rank, "verify": mod.persist_verify_mode(), "fallbacks": mod.persist_fallbacks(),
                      "disabled": bool(mod.persist_disabled()), "checksum": float(flat.sum()),
                      "abs": float(flat.abs().sum()), "losses": [float(x) for x in losses]})
    # one file per rank: the ranks' stdout lines interleave under torch.distributed.run
    with open(f"verify_rank{tr.rank}.json", "w") as f:
        f.write(rec + "\n")
    env.shutdown()


if __name__ == "__main__":
    main()
