#!/usr/bin/env python
"""Scaling report -- the counterpart of the reference's analysis notebooks
(reference: evaluation/Experiments.ipynb:49-216, Experiments_network.ipynb).

Parses rank 0's ``"0: Memory Usage: M, Training Duration: D"`` line (the same
regex as the notebook) from

* this framework's runner output (JSON Lines, bench/runner.py), and/or
* the reference's published result files (``{"results": [{command, stdout,
  stderr, config}]}``, e.g. /root/reference/evaluation/results_*.json --
  read with the json module only),

and prints markdown tables: epoch time / sequences-per-second / memory per
(trainer, nodes|GPUs, batch), the local baseline, and the speed-up of ours
over the reference for matching configurations.  ``--dedup`` drops the
duplicated ``results_ranks.json`` entries the notebook double-counts
(SURVEY.md §6).  ``--csv`` writes the table for any plotting tool.

Network-fault sweeps (reference: evaluation/Experiments_network.ipynb:37-137,
fabfile.py:125-191): records with a ``rule_type`` / ``rule_value`` (the
reference's netem files) or a ``fault_delay_ms`` / ``fault_loss_pct`` config
(bench/runner.py --fault) are tabulated as epoch time per (trainer, nodes,
rule); like the notebook, loss-sweep epochs above 200 s are clipped to 100
(Experiments_network.ipynb:100).

``--plot DIR`` draws the notebooks' figures with matplotlib (imported only
then): epoch time vs nodes/GPUs (Experiments.ipynb:107), memory vs
nodes/GPUs (:142) and the delay / loss sweeps (Experiments_network.ipynb:59-61,
85), one PNG + SVG each.

    python bench/report.py --ours results/matrix.jsonl \\
        --reference /root/reference/evaluation/results_202007141530.json \\
                    /root/reference/evaluation/results_202007141730.json
    python bench/report.py --network --ours results/fault_sweep_gloo.jsonl \\
        --reference /root/reference/evaluation/results_network_202007211500.json \\
                    /root/reference/evaluation/results_network_202007211630.json --plot profiles/plots
"""
from __future__ import annotations

import argparse
import csv
import json
import re
import statistics
from collections import defaultdict
from pathlib import Path
from typing import Dict, Iterable, List, Optional, Tuple

PERF = re.compile(r"(\d+): Memory Usage: ([\d.]+), Training Duration: ([\d.]+)")
NB_NET = re.compile(r"0: Memory Usage: (\d+\.\d+), Training Duration: (\d+\.\d+)")  # Experiments_network.ipynb:37
THRU = re.compile(r"(\d+): Throughput: sequences=(\d+) sequences_per_sec=[\d.]+ world_size=(\d+)")
EPOCH_SEQUENCES = 6912


def _records(path: Path) -> Iterable[Dict]:
    text = Path(path).read_text()
    try:
        obj = json.loads(text)
        if isinstance(obj, dict) and "results" in obj:
            yield from obj["results"]
            return
    except ValueError:
        pass
    for line in text.splitlines():
        line = line.strip()
        if line:
            yield json.loads(line)


def parse_run(rec: Dict) -> Optional[Tuple[str, int, int, float, float, int]]:
    """-> (trainer, nodes/gpus, batch, duration_s, memory_mib, epoch_sequences)
    from rank 0's lines (epoch size from the Throughput line when present,
    else the reference's 6912-sequence training set)."""
    cfg = rec.get("config") or {}
    trainer = cfg.get("trainer") or rec.get("trainer")
    n = cfg.get("gpus") or cfg.get("hosts") or 1
    params = cfg.get("parameters") or {}
    batch = params.get("--batch-size")
    if batch is None:
        m = re.search(r"--batch-size (\d+)", rec.get("command", ""))
        batch = int(m.group(1)) if m else None
    if cfg.get("slots", 1) not in (1, n) and "gpus" not in cfg:
        return None  # reference: only slots == 1 (Experiments.ipynb:77)
    text = (rec.get("stderr") or "") + "\n" + (rec.get("stdout") or "")
    seqs = EPOCH_SEQUENCES
    for m in THRU.finditer(text):
        if m.group(1) == "0":
            seqs = int(m.group(2)) * int(m.group(3))
    for m in PERF.finditer(text):
        if m.group(1) == "0":
            return trainer, int(n), int(batch), float(m.group(3)), float(m.group(2)), seqs
    return None


def aggregate(paths: List[Path], dedup: bool = False) -> Dict[Tuple[str, int, int], Dict[str, float]]:
    seen = set()
    acc: Dict[Tuple[str, int, int], List[Tuple[float, float, int]]] = defaultdict(list)
    for p in paths:
        for rec in _records(p):
            if dedup:
                k = (rec.get("command"), (rec.get("stderr") or "")[-200:])
                if k in seen:
                    continue
                seen.add(k)
            r = parse_run(rec)
            if r:
                acc[r[:3]].append(r[3:])
    out = {}
    for k, v in acc.items():
        d = statistics.mean(x[0] for x in v)
        out[k] = {"duration_s": d, "seq_per_s": statistics.mean(x[2] for x in v) / d,
                  "memory_mib": statistics.mean(x[1] for x in v), "runs": len(v)}
    return out


def parse_network(rec: Dict) -> Optional[Tuple[str, int, str, float, float]]:
    """-> (trainer, nodes/gpus, rule_type, rule_value, duration_s) of one
    fault-sweep run: the reference's netem record or a runner --fault run."""
    cfg = rec.get("config") or {}
    if "rule_type" in rec:
        trainer, rtype, value = rec.get("trainer"), rec["rule_type"], float(rec["rule_value"])
        m = re.search(r"-np (\d+)", rec.get("command", ""))
        n = int(m.group(1)) if m else 12
    elif "fault_delay_ms" in cfg:
        trainer, n = cfg.get("trainer"), int(cfg.get("gpus") or 1)
        if cfg.get("fault_loss_pct"):
            rtype, value = "loss", float(cfg["fault_loss_pct"])
        else:
            rtype, value = "delay", float(cfg.get("fault_delay_ms") or 0)
    else:
        return None
    if "rule_type" in rec:
        # the notebook's parse, kept verbatim: the FIRST match of the
        # unanchored regex in stderr -- with 12 ranks that can be rank 10's
        # line ("10: Memory Usage ..." contains "0: Memory Usage"), which is
        # how the published figures were computed
        m = NB_NET.search(rec.get("stderr") or "")
        return (trainer, n, rtype, value, float(m.group(2))) if m else None
    text = (rec.get("stderr") or "") + "\n" + (rec.get("stdout") or "")
    for m in PERF.finditer(text):
        if m.group(1) == "0":
            return trainer, n, rtype, value, float(m.group(3))
    return None


def aggregate_network(paths: List[Path]) -> Dict[Tuple[str, int, str, float], Dict[str, float]]:
    acc: Dict[Tuple[str, int, str, float], List[float]] = defaultdict(list)
    for p in paths:
        for rec in _records(p):
            r = parse_network(rec)
            if r:
                d = r[4]
                if r[2] == "loss" and d > 200:
                    d = 100.0  # the notebook's per-run outlier clip (Experiments_network.ipynb:100)
                acc[r[:4]].append(d)
    out = {}
    for k, v in acc.items():
        out[k] = {"duration_s": statistics.mean(v), "runs": len(v)}
    # a delay of 0 is also the loss sweep's 0 point (and vice versa)
    for (tr, n, rt, v), val in list(out.items()):
        if v == 0:
            other = "loss" if rt == "delay" else "delay"
            out.setdefault((tr, n, other, 0.0), dict(val))
    return out


def network_table(rows: Dict, title: str) -> str:
    lines = [f"### {title}", ""]
    for rtype, unit in (("delay", "ms"), ("loss", "%")):
        keys = sorted({(tr, n) for tr, n, rt, _ in rows if rt == rtype})
        vals = sorted({v for _, _, rt, v in rows if rt == rtype})
        if not keys:
            continue
        lines += [f"{rtype} sweep: epoch time (s) at each {rtype} ({unit})", "",
                  "| trainer | nodes/GPUs | " + " | ".join(f"{v:g}" for v in vals) + " |",
                  "|---|---|" + "---|" * len(vals)]
        for tr, n in keys:
            cells = [f"{rows[(tr, n, rtype, v)]['duration_s']:.2f}" if (tr, n, rtype, v) in rows else "–"
                     for v in vals]
            lines.append(f"| {tr} | {n} | " + " | ".join(cells) + " |")
        lines.append("")
    return "\n".join(lines)


def plot(ours: Dict, ref: Dict, net_ours: Dict, net_ref: Dict, out_dir: Path, label: str) -> List[Path]:
    """The notebooks' figures (matplotlib, Agg backend)."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    out_dir.mkdir(parents=True, exist_ok=True)
    written = []

    def save(fig, name):
        for ext in ("png", "svg"):
            p = out_dir / f"{name}.{ext}"
            fig.savefig(p, bbox_inches="tight", dpi=110)
            written.append(p)
        plt.close(fig)

    for metric, ylabel, name in (("duration_s", "epoch time (s)", "time_vs_nodes"),
                                 ("seq_per_s", "sequences / s (whole job)", "throughput_vs_nodes"),
                                 ("memory_mib", "peak RSS rank 0 (MiB)", "memory_vs_nodes")):
        srcs = [(s, r) for s, r in ((f"reference (Pi cluster)", ref), (label, ours)) if r]
        if not srcs:
            continue
        fig, axes = plt.subplots(1, len(srcs), figsize=(6 * len(srcs), 4), squeeze=False)
        for ax, (src, rows) in zip(axes[0], srcs):
            for tr in sorted({k[0] for k in rows}):
                for b in sorted({k[2] for k in rows if k[0] == tr}):
                    pts = sorted((k[1], v[metric]) for k, v in rows.items() if k[0] == tr and k[2] == b)
                    if tr == "local" or len(pts) == 1:
                        ax.axhline(pts[0][1], ls="--", lw=1, label=f"{tr} bs {b}")
                    else:
                        ax.plot([p[0] for p in pts], [p[1] for p in pts], marker="o", label=f"{tr} bs {b}")
            ax.set_xlabel("nodes / GPUs")
            ax.set_ylabel(ylabel)
            ax.set_title(src)
            ax.legend(fontsize=7)
            ax.grid(alpha=0.3)
        save(fig, name)
    for rtype, unit in (("delay", "ms"), ("loss", "%")):
        srcs = [(s, r) for s, r in (("reference (12 Pis, netem)", net_ref), (label, net_ours))
                if any(k[2] == rtype for k in r)]
        if not srcs:
            continue
        fig, axes = plt.subplots(1, len(srcs), figsize=(6 * len(srcs), 4), squeeze=False)
        for ax, (src, rows) in zip(axes[0], srcs):
            for tr, n in sorted({(k[0], k[1]) for k in rows if k[2] == rtype}):
                pts = sorted((k[3], v["duration_s"]) for k, v in rows.items() if k[:3] == (tr, n, rtype))
                ax.plot([p[0] for p in pts], [p[1] for p in pts], marker="o", label=f"{tr} x{n}")
            ax.set_xlabel(f"{rtype} ({unit})")
            ax.set_ylabel("epoch time (s)")
            ax.set_title(src)
            ax.legend(fontsize=7)
            ax.grid(alpha=0.3)
        save(fig, f"{rtype}_sweep")
    return written


def table(rows: Dict, title: str) -> str:
    lines = [f"### {title}", "", "| trainer | nodes/GPUs | batch | epoch time (s) | seq/s | memory (MiB) | runs |",
             "|---|---|---|---|---|---|---|"]
    for (tr, n, b), v in sorted(rows.items(), key=lambda kv: (kv[0][0], kv[0][2], kv[0][1])):
        lines.append(f"| {tr} | {n} | {b} | {v['duration_s']:.4f} | {v['seq_per_s']:.1f} | {v['memory_mib']:.1f} | "
                     f"{v['runs']} |")
    return "\n".join(lines)


def compare(ours: Dict, ref: Dict) -> str:
    lines = ["### ours vs reference (matching trainer / count / batch)", "",
             "| trainer | n | batch | ref seq/s | ours seq/s | speed-up |", "|---|---|---|---|---|---|"]
    for k in sorted(set(ours) & set(ref)):
        lines.append(f"| {k[0]} | {k[1]} | {k[2]} | {ref[k]['seq_per_s']:.1f} | {ours[k]['seq_per_s']:.1f} | "
                     f"{ours[k]['seq_per_s'] / ref[k]['seq_per_s']:.0f}x |")
    return "\n".join(lines)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--ours", type=Path, nargs="*", default=[])
    ap.add_argument("--reference", type=Path, nargs="*", default=[])
    ap.add_argument("--dedup", action="store_true")
    ap.add_argument("--csv", type=Path, default=None)
    ap.add_argument("--label", default="this framework (MI355X)")
    ap.add_argument("--network", action="store_true", help="fault-sweep tables (netem / runner --fault records)")
    ap.add_argument("--plot", type=Path, default=None, help="write the notebooks' figures (PNG + SVG) here")
    a = ap.parse_args(argv)
    if a.network:
        net_ours = aggregate_network(a.ours) if a.ours else {}
        net_ref = aggregate_network(a.reference) if a.reference else {}
        parts = []
        if net_ref:
            parts.append(network_table(net_ref, "reference network sweep (12 Raspberry Pis, tc netem)"))
        if net_ours:
            parts.append(network_table(net_ours, a.label))
        print("\n\n".join(parts))
        if a.plot:
            for p in plot({}, {}, net_ours, net_ref, a.plot, a.label):
                print(f"wrote {p}")
        return
    ours = aggregate(a.ours) if a.ours else {}
    ref = aggregate(a.reference, dedup=a.dedup) if a.reference else {}
    parts = []
    if ref:
        parts.append(table(ref, "reference (Raspberry Pi cluster, published result files)"))
    if ours:
        parts.append(table(ours, a.label))
    if ours and ref:
        parts.append(compare(ours, ref))
    print("\n\n".join(parts))
    if a.plot:
        for p in plot(ours, ref, {}, {}, a.plot, a.label):
            print(f"wrote {p}")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["source", "trainer", "n", "batch", "duration_s", "seq_per_s", "memory_mib", "runs"])
            for src, rows in (("reference", ref), ("ours", ours)):
                for (tr, n, b), v in sorted(rows.items()):
                    w.writerow([src, tr, n, b, v["duration_s"], v["seq_per_s"], v["memory_mib"], v["runs"]])


if __name__ == "__main__":
    main()
