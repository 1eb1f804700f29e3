"""Print the key fields of one bench.py JSON line from stdin: tools/bench_line.py LABEL"""
import json
import sys

d = json.loads(sys.stdin.read().strip().splitlines()[-1])
extra = {k: d[k] for k in ("step_seq_per_s", "epoch_time_s", "epochs") if k in d}
print(sys.argv[1] if len(sys.argv) > 1 else "", "value", d["value"], "ms/step", d["ms_per_step"], extra)
