"""Compute-layout copies ("shadows") of fp32 master weights, rebuilt together.

The HIP kernels read the recurrent weights in layouts of their own:
- gate-interleaved rows, for the forward step and the input projection;
- transposed, for the BPTT step GEMM;
- the stored layout cast to 16 bit, for the dX GEMM;
- the GRU's zero-padded stacks;
- the folded projection bias.

Each shadow is cached on a parameter and keyed on the masters' version counters,
so it is rebuilt only after an optimizer step; FusedAdam's native step bumps the
counters explicitly. Each layout used to be rebuilt with its own torch copy or
add, about ten dispatches a step on the char-LM and the fp32 hidden-128 motion
model (the glue traced by tools/charlm_glue_trace.py). Here every shadow is a
:class:`Shadow` entry in a per-device registry. The first stale lookup after a
step rebuilds *every* stale shadow of that device in one
``shadow_pack`` launch (csrc/kernels/shadow_pack.hip: 3-D strided gathers
through LDS tiles, converting to bf16 / fp16 / fp32). Without the native
extension, or on the CPU, the same jobs run as torch copies.

A shadow is described by a *builder*: a function of the live master tensors
that returns jobs ``(dst_view, src_view, src2_view_or_None)`` of equal shape
(up to 3-D), meaning ``dst = src (+ src2)``. Builders capture only the output
buffers, never the masters, so the registry and the caches keep no parameter
alive.

Reference parity: the reference casts nothing. Its torch.nn.LSTM reads the fp32
parameters directly (/root/reference/src/motion/model.py:9), so this is
MI355X-side machinery with no counterpart there.
"""
import weakref
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
from torch import Tensor

from .. import _ext

Job = Tuple[Tensor, Tensor, Optional[Tensor]]

__all__ = ["Shadow", "get", "refresh", "job", "pack", "cast", "stats"]

_REG: Dict[Tuple[str, int], "weakref.WeakSet[Shadow]"] = {}
_STATS = {"refreshes": 0, "jobs": 0, "launches": 0}


class Shadow:
    """One cached layout: the masters (weakly held), the builder, the output."""

    __slots__ = ("masters", "sig", "build", "out", "ver", "dead", "__weakref__")

    def __init__(self, masters: Sequence[Optional[Tensor]], build: Callable[..., List[Job]], out):
        self.masters = [weakref.ref(m) if m is not None else None for m in masters]
        self.sig = _sig(masters)
        self.build = build
        self.out = out
        self.ver = None
        self.dead = False

    def live(self) -> Optional[List[Optional[Tensor]]]:
        ms = []
        for r in self.masters:
            if r is None:
                ms.append(None)
                continue
            m = r()
            if m is None:
                return None
            ms.append(m)
        return ms


def _sig(ms: Sequence[Optional[Tensor]]):
    return tuple((tuple(m.shape), m.dtype, m.device) if m is not None else None for m in ms)


def _version(ms: Sequence[Optional[Tensor]]):
    return tuple((m._version, m.data_ptr()) if m is not None else None for m in ms)


def _dev_key(device: torch.device) -> Tuple[str, int]:
    return (device.type, device.index if device.index is not None else -1)


def get(anchor: Tensor, key, masters: Sequence[Optional[Tensor]], alloc: Callable[[], object],
        build: Callable[..., List[Job]]):
    """The shadow ``key`` cached on ``anchor``, refreshed if any master moved.

    ``alloc()`` makes the output buffers once. ``build(*masters)`` returns the
    jobs that fill them. A stale lookup refreshes every stale shadow on the
    device in one launch."""
    cache = getattr(anchor, "_pdrnn_shadow", None)
    if cache is None:
        cache = {}
        anchor._pdrnn_shadow = cache
    ent = cache.get(key)
    if ent is None or ent.dead or ent.sig != _sig(masters):
        with torch.no_grad():
            ent = Shadow(masters, build, alloc())
        cache[key] = ent
        _REG.setdefault(_dev_key(anchor.device), weakref.WeakSet()).add(ent)
    if ent.ver != _version(masters):
        refresh(anchor.device)
    return ent.out


def refresh(device: torch.device) -> int:
    """Rebuild every stale shadow registered on ``device``; returns the jobs run."""
    reg = _REG.get(_dev_key(device))
    if not reg:
        return 0
    jobs: List[Job] = []
    for ent in list(reg):
        if ent.dead:
            continue
        ms = ent.live()
        if ms is None or ent.sig != _sig(ms):
            ent.dead = True  # a master was freed or re-shaped: rebuilt on its next lookup
            reg.discard(ent)
            continue
        ver = _version(ms)
        if ent.ver == ver:
            continue
        with torch.no_grad():
            jobs.extend(ent.build(*[m.detach() if m is not None else None for m in ms]))
        ent.ver = ver
    if not jobs:
        return 0
    _STATS["refreshes"] += 1
    _STATS["jobs"] += len(jobs)
    _STATS["launches"] += pack(jobs, device)
    return len(jobs)


def pack(jobs: List[Job], device: Optional[torch.device] = None) -> int:
    """Run pack jobs: one ``shadow_pack`` launch per 16 on the GPU, torch
    copies otherwise.  Returns the launches (0 on the torch path)."""
    if not jobs:
        return 0
    device = device if device is not None else jobs[0][0].device
    mod = _ext.native(device) if device.type == "cuda" else None
    with torch.no_grad():
        if mod is not None and hasattr(mod, "shadow_pack"):
            return int(mod.shadow_pack(jobs))
        for d, s, s2 in jobs:
            d.copy_(s if s2 is None else s + s2)
    return 0


def cast(w: Tensor, dtype: torch.dtype) -> Tensor:
    """``w`` in ``dtype`` (the detached master itself when it already is), as a
    cached shadow: a head's 16-bit weight is converted once per optimizer step,
    inside the shared pack launch, instead of on every forward."""
    if w.dtype == dtype:
        return w.detach()
    if w.dtype != torch.float32 or dtype not in (torch.bfloat16, torch.float16, torch.float32) or w.dim() > 3:
        return w.detach().to(dtype)
    box = []

    def alloc():
        box.append(torch.empty(w.shape, device=w.device, dtype=dtype))
        return box[0]

    def build(src):
        return [job(box[0], src)]

    return get(w, ("p", dtype), [w], alloc, build)


def job(dst: Tensor, src: Tensor, src2: Optional[Tensor] = None) -> Job:
    """A pack job ``dst = src (+ src2)`` on equal-shape views (up to 3-D),
    reordered so the kernel's 64 x 64 tile covers the source's and the
    destination's unit-stride dimensions (dst last, src next), with the
    largest remaining extent in the tile when they coincide."""
    if dst.shape != src.shape or dst.dim() > 3:
        raise ValueError(f"shadow job: shapes {tuple(dst.shape)} vs {tuple(src.shape)}")
    while dst.dim() < 3:
        dst, src = dst.unsqueeze(0), src.unsqueeze(0)
        src2 = src2.unsqueeze(0) if src2 is not None else None

    def inner(t: Tensor) -> int:
        cands = [k for k in range(3) if t.shape[k] > 1] or [2]
        return min(cands, key=lambda k: (abs(t.stride(k)), -k))

    di, si = inner(dst), inner(src)
    if di != si:
        order = [k for k in range(3) if k not in (di, si)] + [si, di]
    else:
        rest = sorted((k for k in range(3) if k != di), key=lambda k: dst.shape[k])
        order = rest + [di]
    return (dst.permute(order), src.permute(order), src2.permute(order) if src2 is not None else None)


def stats() -> Dict[str, int]:
    """Refreshes, jobs and pack launches so far (tests, glue accounting)."""
    return dict(_STATS)
