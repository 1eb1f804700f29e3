#!/usr/bin/env python
"""Per-kernel register / LDS / occupancy table from hipcc's resource remarks.

    python tools/kernel_resources.py pytorch_distributed_rnn_amd/csrc/kernels/lstm_small.hip [filter]
"""
import re
import subprocess
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "pytorch_distributed_rnn_amd", "csrc", "include")


def main():
    src = sys.argv[1]
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    cmd = ["/opt/rocm/bin/hipcc", "-c", "-O3", "-std=c++17", "--offload-arch=gfx950", "-munsafe-fp-atomics",
           f"-I{INC}", src, "-o", "/tmp/_res.o", "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"name": subprocess.run(["c++filt", m.group(1)], capture_output=True,
                                          text=True).stdout.strip()}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z /\[\]]+?): (\d+)", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = m.group(2)
    print(f"{'kernel':90s} vgpr agpr vspill sspill lds occ")
    for r in rows:
        n = re.sub(r"pdrnn::\(anonymous namespace\)::", "", r["name"])
        n = re.sub(r"\(Pdrnn\w+\)", "", n)
        if flt and flt not in n:
            continue
        print(f"{n[:90]:90s} {r.get('VGPRs','?'):>4} {r.get('AGPRs','?'):>4} {r.get('VGPRs Spill','?'):>6} "
              f"{r.get('SGPRs Spill','?'):>6} {r.get('LDS Size [bytes/block]','?'):>4} "
              f"{r.get('Occupancy [waves/SIMD]','?'):>3}")


if __name__ == "__main__":
    main()
