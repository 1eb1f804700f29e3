"""Fused whole-step training path for the motion classifier on MI355X.

One optimizer step of the reference's training loop (reference:
src/motion/trainer/base.py:103-130 -- zero_grad, forward, CrossEntropyLoss,
backward, Adam.step) becomes, on the native path:

1. ``lstm_small_fwd`` with the classifier head and softmax cross-entropy
   fused into its epilogue (per-sequence loss / correct / dW_fc / dh_T),
2. ``lstm_small_bwd`` (BPTT for every layer in one launch),
3. one deterministic slab reduction writing ALL parameter gradients directly
   into the model's flat gradient buffer (= the DDP all-reduce bucket) plus
   the batch statistics,
4. gradient synchronisation (native RCCL all-reduce of the flat buffer, or
   nothing for a single process),
5. the fused flat Adam kernel.

No autograd graph is built and no per-op kernels run, so the host cost per
step is a handful of launches; the math is identical to the autograd path
(tested against it).  The loss is the local mean over this rank's batch and
gradients are averaged over ranks -- the same semantics as the reference's
DDP step.
"""
from __future__ import annotations

import os
from typing import Callable, Optional

import torch
from torch import Tensor, nn

from .. import _ext
from ..utils.flat import contiguous_span
from ..utils.tracing import trace_range


def _inner(model: nn.Module) -> nn.Module:
    return getattr(model, "module", model)


def supported(model: nn.Module, optimizer, device: torch.device) -> bool:
    from ..models.motion import MotionModel
    from ..ops.adam import FusedAdam
    m = _inner(model)
    if device.type != "cuda" or not isinstance(m, MotionModel) or m.cell not in ("lstm", "gru"):
        return False
    if m.cell == "gru" and getattr(m, "compute_dtype", torch.float32) != torch.float32:
        return False  # the GRU step runs the fp32 kernels only
    if not isinstance(optimizer, FusedAdam):
        return False
    mod = _ext.native(device)
    if mod is None or not hasattr(mod, "lstm_head_train_step"):
        return False
    lstm = m.lstm
    if lstm.bidirectional or lstm.proj_size or not lstm.bias or lstm.dropout:
        return False
    if not mod.lstm_small_supported(lstm.hidden_size, lstm.input_size, lstm.num_layers):
        return False
    if mod.lstm_small_max_split(lstm.hidden_size, lstm.num_layers, False) != 1 or \
            mod.lstm_small_max_split(lstm.hidden_size, lstm.num_layers, True) != 1:
        return False
    if m.cell == "gru":
        H, NL = lstm.hidden_size, lstm.num_layers
        if NL * 4 * H > 512 or NL * H * (8 if H >= 64 else 4) > 512:
            return False
    params = list(m.parameters())
    if any(p.dtype != torch.float32 for p in params):
        return False
    if getattr(m, "compute_dtype", torch.float32) not in (torch.float32, torch.bfloat16):
        return False
    return contiguous_span([p.data for p in params]) is not None


class MotionTrainStep:
    """Callable running one fused training step; returns [loss, n, correct].

    Single process (no gradient sync): the optimizer step is fused into the
    one-pass gradient reduction (``slab_reduce_adam`` kernel), so one step is
    four launches: forward+head+CE, BPTT, the matrix-core weight gradients
    (deferred dW) and the reduction + Adam -- three up to two sequences per CU
    (B <= 512 on 256 CUs), where the BPTT workgroups form the weight gradients
    themselves (kernels/lstm_sw.hip, backward mode 4).

    With gradient sync (multi-GPU) the step is forward+BPTT+reductions, the
    inline RCCL all-reduce and the flat Adam.  ``cuda_graph=True`` (or
    ``PDRNN_CUDA_GRAPH=1``) captures that whole sequence once into a HIP graph
    and replays it: RCCL's eager enqueue leaves ~13 us idle gaps on each side
    of its kernel (measured at the 8-GPU per-rank batch); inside a graph the
    collective is an ordinary kernel node.  The replayed step reads this
    batch's indices from a static buffer and the Adam step count from device
    memory (incremented in the graph), so one capture serves every later
    step; it is re-captured when the batch shape, data tables or optimizer
    hyper-parameters change."""

    RING = 16384

    def __init__(self, model: nn.Module, optimizer, grad_sync: Optional[Callable[[], None]] = None,
                 cuda_graph: Optional[bool] = None, comm=None):
        self.model = model
        self.m = _inner(model)
        self.optimizer = optimizer
        self.grad_sync = grad_sync
        # the communicator grad_sync runs on: a graph replay (whose captured
        # collectives carry no completion event) is registered with ITS
        # watchdog as one unit.  Default: the DDP wrapper's communicator.
        self.comm = comm if comm is not None else getattr(model, "comm", None)
        self.mod = _ext.native(next(self.m.parameters()).device)
        lstm = self.m.lstm
        self.H, self.NL = lstm.hidden_size, lstm.num_layers
        # GRU: the kernels run nn.GRU's parameters packed as [r | z | n_x | n_h]
        # 4-block stacks (ops/gru_fused.py); the reduction writes gradients
        # back in nn.GRU order through a column map
        self.gru = getattr(self.m, "cell", "lstm") == "gru"
        self.weights = []
        for l in range(self.NL):
            self.weights += [getattr(lstm, f"weight_ih_l{l}"), getattr(lstm, f"weight_hh_l{l}"),
                             getattr(lstm, f"bias_ih_l{l}"), getattr(lstm, f"bias_hh_l{l}")]
        flat = getattr(self.m, "_pdrnn_flat", None)
        if not flat or len(flat) != 1:
            raise RuntimeError("fused step needs the model's flat parameter storage")
        self.flat = next(iter(flat.values()))
        # batch statistics land in a ring of rows (returned as views, no copy
        # kernel per step); a row is reused after RING steps
        self.ring = torch.zeros(self.RING, 3, dtype=torch.float32, device=self.flat.grad.device)
        self._slot = 0
        # bf16 model: the kernels round the fp32 master W_ih / W_hh to bf16 as
        # they load them (round_bf16; no cast pass, graph-capturable);
        # gradients land on the fp32 masters
        self.bf16 = getattr(self.m, "compute_dtype", torch.float32) == torch.bfloat16
        self.colmap = None
        if self.gru:
            from ..ops.gru_fused import _unpack_index
            in_dims = tuple(int(self.weights[4 * l].shape[1]) for l in range(self.NL))
            self.colmap = _unpack_index(self.H, in_dims, self.flat.grad.device).to(torch.int32)
        base = self.flat.data.data_ptr()
        self._offs = [((w.data_ptr() - base) // 4, w.shape) for w in self.weights]
        if cuda_graph is None:
            # default: graph replay for the synced multi-GPU step (RCCL's eager
            # enqueue leaves ~13 us idle on each side of the all-reduce; at the
            # 8-GPU per-rank batch that is ~10 % of a step --
            # profiles/r1_v5_graph_step.md).  A single process replays its
            # epochs from a graph only on request (PDRNN_CUDA_GRAPH=1 /
            # cuda_graph=True): at B = 1440 the replay ran 1.5 % slower than
            # the eager launches (0.3364 vs 0.3313 ms/step,
            # profiles/r6/epoch_graph_world1.md)
            env = os.environ.get("PDRNN_CUDA_GRAPH")
            if env is not None:
                cuda_graph = env == "1"
            elif grad_sync is None:
                cuda_graph = False
            else:
                import torch.distributed as dist
                # RCCL only: a gloo collective copies through the host and
                # cannot be captured
                cuda_graph = dist.is_available() and dist.is_initialized() \
                    and dist.get_world_size() > 1 and dist.get_backend() == "nccl"
        self.cuda_graph = bool(cuda_graph)
        self._graph = None       # last replayed synced step (torch.cuda.CUDAGraph = hipGraph)
        self._graphs = {}        # configuration key -> captured step
        self._gru_buf = None     # GRU: persistent [r|z|n_x|n_h] packing buffer (graph-capturable)

    def _operands(self, features: Tensor):
        """(weights as the kernels read them, features, cell code): the bf16
        model's fp32 masters (rounded in-kernel) with bf16 inputs, the GRU's
        4-block packing written into a persistent buffer (one captured cat
        kernel: no allocation, so the packed step graph-replays), else the
        parameters themselves."""
        if self.bf16:
            if features.dtype != torch.bfloat16:
                features = features.to(torch.bfloat16)
            return self.weights, features, 0
        if self.gru:
            from ..ops.gru_fused import _pack, packed_numel
            if self._gru_buf is None:
                self._gru_buf = torch.empty(packed_numel(self.weights, self.NL, self.H), dtype=self.flat.data.dtype,
                                            device=self.flat.data.device)
            return _pack(self.weights, self.NL, self.H, self.flat.data, out=self._gru_buf), features, 1
        return self.weights, features, 0

    def run_steps(self, features: Tensor, labels: Tensor, idx_list) -> Optional[list]:
        """Consecutive training steps (an epoch's batches, the short last one
        included) as ONE HIP-graph replay of the synced step -- forward/BPTT,
        inline RCCL all-reduce and Adam for every batch, the device step
        count advancing from one captured step to the next (adam_flat's
        arrival ticket) -- so neither a per-step graph boundary nor a per-step
        host copy sits between the steps: the batch indices of all steps reach
        the graph's static buffer in one copy before the replay.  Returns each
        step's statistics row, or None when this configuration runs per step
        (no graph replay, host-gathered batches, the first two calls of a
        configuration).  Without gradient sync (one process) each captured
        step is the fused step with Adam folded into its reduction, the
        device step count advanced by that kernel's last workgroup."""
        if not self.cuda_graph:
            return None
        if not idx_list or any(i is None for i in idx_list):
            return None
        adam = self._flat_adam_peek()
        if adam is None:
            return None
        (p, m, v), (lr, b1, b2, eps, wd, step, dec) = adam
        sizes = tuple(int(i.numel()) for i in idx_list)
        key, cfgs = self._epoch_key(features, labels, sizes, idx_list[0].dtype, adam)
        graphs = self.__dict__.setdefault("_graphs", {})
        ent = graphs.get(key)
        if ent is None:
            ent = {"graph": None, "eager": 0}
            if len(graphs) >= self._GRAPHS_MAX:
                graphs.pop(next(iter(graphs)))
            graphs[key] = ent
        n = len(sizes)
        slots = [(self._slot + k) % self.RING for k in range(n)]
        if ent["graph"] is None:
            ent["eager"] += 1
            if ent["eager"] <= 2:
                return None  # RCCL's lazy setup and first-use allocations outside the capture
            self.flat.attach_grads()
            try:
                self._capture_epoch(ent, features, labels, idx_list, cfgs, adam, slots[0])
            except Exception as exc:  # capture unsupported here: stay eager for good
                import warnings
                warnings.warn(f"HIP graph capture of the synced epoch failed ({exc!r}); running per step")
                torch.cuda.synchronize(self.flat.grad.device)
                graphs.clear()
                self.cuda_graph = False
                return None
        self.flat.attach_grads()
        # host-side optimizer state advances by n steps (the graph advances the device count)
        for _ in range(n):
            self._flat_adam()
        c0 = step - 1.0  # optimizer step count before this call's first step
        if ent["step_host"] != c0:
            ent["step"].fill_(c0)
        # one copy of every step's indices: a single slice when the batches are
        # consecutive views of one index tensor (DeviceBatchLoader's split)
        total = sum(sizes)
        b0 = idx_list[0]._base
        esz = idx_list[0].element_size()
        if b0 is not None and b0.is_contiguous() and all(i._base is b0 for i in idx_list) and \
                all(idx_list[k].data_ptr() == idx_list[0].data_ptr() + esz * sum(sizes[:k]) for k in range(n)):
            first = (idx_list[0].data_ptr() - b0.data_ptr()) // esz
            ent["idx_all"].copy_(b0.view(-1).narrow(0, first, total), non_blocking=True)
        else:
            torch.cat(list(idx_list), out=ent["idx_all"])
        with trace_range("pdrnn.graph_epoch"):
            ent["graph"].replay()
        if self.comm is not None and hasattr(self.comm, "track_current"):
            self.comm.track_current()  # the communicator's watchdog bounds the replay
        ent["step_host"] = c0 + n
        self._slot = (self._slot + n) % self.RING
        rows = [(int(c0) + k + ent["slot_off"]) % self.RING for k in range(n)]
        if rows != slots:
            # the host's ring slots are out of step with the captured mapping:
            # move the rows as one gather (the two ranges may overlap, so a
            # row-by-row copy could overwrite a row before it is read)
            dev = self.ring.device
            src = torch.tensor(rows, dtype=torch.long).to(dev, non_blocking=True)
            dst = torch.tensor(slots, dtype=torch.long).to(dev, non_blocking=True)
            self.ring.index_copy_(0, dst, self.ring.index_select(0, src))
        return [self.ring[slot] for slot in slots]

    def _epoch_key(self, features: Tensor, labels: Tensor, sizes, idx_dtype, adam):
        from ..ops.lstm import fused_bwd_nb, small_launch_config
        (p, m, v), (lr, b1, b2, eps, wd, step, dec) = adam
        cfgs = []
        for b in sizes:
            nb_fwd, sp_fwd, _, _ = small_launch_config(b, self.H, self.NL)
            if self.gru:
                from ..ops.lstm import gru_fwd_nb
                nb_fwd, sp_fwd = gru_fwd_nb(b, self.H, features.device), 1
            cfgs.append(((nb_fwd, sp_fwd), fused_bwd_nb(b, self.H, self.NL)))
        key = ("epoch", features.data_ptr(), tuple(features.shape), features.dtype, labels.data_ptr(),
               labels.numel(), tuple(sizes), idx_dtype, tuple(cfgs), lr, b1, b2, eps, wd, dec,
               p.data_ptr(), m.data_ptr(), v.data_ptr(), self.flat.grad.data_ptr())
        return key, cfgs

    def prepare_epoch(self, features: Tensor, labels: Tensor, sizes) -> bool:
        """Capture the epoch graph of ``run_steps`` for these batch sizes ahead
        of time (Trainer.prepare, before the timed epochs): one eager gradient
        all-reduce first -- RCCL's lazy connection setup cannot happen inside a
        capture -- then the capture itself, which runs nothing.  Parameters
        and optimizer state are untouched; the flat gradient (rewritten by
        every step) is left zeroed.  True when the graph is ready."""
        if not self.cuda_graph or not sizes:
            return False
        adam = self._flat_adam_peek()
        if adam is None:
            return False
        dev = self.flat.grad.device
        idx_list = list(torch.split(torch.zeros(sum(sizes), dtype=torch.long, device=dev), list(sizes)))
        key, cfgs = self._epoch_key(features, labels, tuple(sizes), torch.long, adam)
        graphs = self.__dict__.setdefault("_graphs", {})
        if key in graphs and graphs[key]["graph"] is not None:
            return True
        self.flat.attach_grads()
        if self.grad_sync is not None:
            self.grad_sync()
        self.flat.grad.zero_()
        ent = {"graph": None, "eager": 0}
        try:
            self._capture_epoch(ent, features, labels, idx_list, cfgs, adam, self._slot)
        except Exception as exc:
            import warnings
            warnings.warn(f"HIP graph capture of the synced epoch failed ({exc!r}); running per step")
            torch.cuda.synchronize(dev)
            return False
        if len(graphs) >= self._GRAPHS_MAX:
            graphs.pop(next(iter(graphs)))
        graphs[key] = ent
        return True

    def _capture_epoch(self, ent: dict, features: Tensor, labels: Tensor, idx_list, cfgs, adam, slot: int):
        (p, m, v), (lr, b1, b2, eps, wd, step, dec) = adam
        dev = self.flat.grad.device
        hw, hb = self.m.fc.weight, self.m.fc.bias
        sizes = [int(i.numel()) for i in idx_list]
        ent["idx_all"] = torch.cat(list(idx_list)).clone()
        offs = [sum(sizes[:k]) for k in range(len(sizes))]
        views = [ent["idx_all"][o:o + b] for o, b in zip(offs, sizes)]
        # the statistics of captured step k go to ring row (device step count
        # before that step's Adam) + slot_off = the host slot of step k
        ent["slot_off"] = (slot - (int(step) - 1)) % self.RING
        ent["step"] = torch.zeros(1, dtype=torch.float32, device=dev)
        ent["ticket"] = torch.zeros(1, dtype=torch.int32, device=dev)
        ent["step_host"] = None
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            for view, ((nb, sp), nb_bwd) in zip(views, cfgs):
                ws, feats, cell = self._operands(features)  # GRU: re-packed from the updated parameters
                if self.grad_sync is None:
                    # one process: Adam folded into the reduction, which
                    # advances the device step count (the hyper-parameters'
                    # step slot is unused)
                    self.mod.lstm_head_train_step(feats, view, labels, ws, hw, hb, self.flat.grad, self.ring,
                                                  self.H, self.NL, sp, 0, nb, nb_bwd, [p, m, v],
                                                  [lr, b1, b2, eps, wd, 1.0, dec], cell, self.colmap,
                                                  ent["step"], ent["slot_off"], round_bf16=self.bf16,
                                                  adam_ticket=ent["ticket"])
                    continue
                self.mod.lstm_head_train_step(feats, view, labels, ws, hw, hb, self.flat.grad, self.ring,
                                              self.H, self.NL, sp, 0, nb, nb_bwd, None, None, cell, self.colmap,
                                              ent["step"], ent["slot_off"], round_bf16=self.bf16)
                self.grad_sync()
                self.mod.adam_flat(p, self.flat.grad, m, v, None, lr, b1, b2, eps, wd, step + 1.0, 1.0, bool(dec),
                                   False, None, ent["step"], ent["ticket"])
        ent["graph"] = g

    def _flat_adam(self):
        """(state, hyper-parameters) when the optimizer is a plain single-group
        FusedAdam over exactly the model's flat buffer: the step then runs as
        one native launch on the cached flat state (inside the reduction tail
        for a single process, or right after the gradient all-reduce) instead
        of going through ``optimizer.step()``.  Advances the step count."""
        from ..ops.adam import FusedAdam
        from ..parallel.horovod import _DistributedOptimizerMixin
        opt = self.optimizer
        # a Horovod-wrapped FusedAdam qualifies too: its step() only adds the
        # hook-driven synchronize, which the fused step replaces (no autograd
        # hooks fire; the flat gradient is reduced by ``grad_sync``)
        cls = type(opt)
        if cls is not FusedAdam and cls.__bases__ != (_DistributedOptimizerMixin, FusedAdam):
            return None
        if len(opt.param_groups) != 1:
            return None
        g = opt.param_groups[0]
        if g.get("amsgrad") or g.get("maximize") or opt._pdrnn_grad_scale != 1.0:
            return None
        fs = opt._group_flat(0, g)
        if fs is None or fs["flat_p"].data_ptr() != self.flat.data.data_ptr() or \
                fs["flat_p"].numel() != self.flat.data.numel():
            return None
        fs["step"] += 1.0
        b1, b2 = g["betas"]
        hp = [float(g["lr"]), b1, b2, g["eps"], g["weight_decay"], float(fs["step"]),
              1.0 if g.get("decoupled_weight_decay", False) else 0.0]
        return [fs["flat_p"], fs["exp_avg"], fs["exp_avg_sq"]], hp

    def __call__(self, features: Tensor, labels: Tensor, idx: Optional[Tensor]) -> Tensor:
        from ..ops.lstm import fused_bwd_nb, gru_fwd_nb, small_launch_config
        self.flat.attach_grads()
        batch = idx.numel() if idx is not None else features.shape[0]
        nb_fwd, sp_fwd, _, _ = small_launch_config(batch, self.H, self.NL)
        nb_bwd = fused_bwd_nb(batch, self.H, self.NL)
        if self.gru:  # (gate-split family geometry; the sequence-in-wave kernels, H = 32, ignore it)
            nb_fwd, sp_fwd = gru_fwd_nb(batch, self.H, features.device), 1
        hw, hb = self.m.fc.weight, self.m.fc.bias  # the classifier head stays fp32
        slot = self._slot
        stats = self.ring[slot]
        self._slot = (self._slot + 1) % self.RING
        adam = self._flat_adam()
        if self.grad_sync is not None and adam is not None and self.cuda_graph:
            if self._graph_step(features, labels, idx, (nb_fwd, sp_fwd), nb_bwd, adam, stats, slot):
                return stats
        ws, features, cell = self._operands(features)
        if adam is not None and self.grad_sync is None:
            with trace_range("pdrnn.fwd_bwd_adam"):
                self.mod.lstm_head_train_step(features, idx, labels, ws, hw, hb, self.flat.grad, stats, self.H,
                                              self.NL, sp_fwd, 0, nb_fwd, nb_bwd, adam[0], adam[1], cell, self.colmap,
                                              round_bf16=self.bf16)
            return stats
        with trace_range("pdrnn.fwd_bwd"):
            self.mod.lstm_head_train_step(
                features, idx, labels, ws, hw, hb, self.flat.grad, stats, self.H, self.NL, sp_fwd, 0, nb_fwd, nb_bwd,
                None, None, cell, self.colmap, round_bf16=self.bf16)
        if self.grad_sync is not None:
            with trace_range("pdrnn.grad_allreduce"):
                self.grad_sync()
        with trace_range("pdrnn.optimizer"):
            if adam is not None:
                (p, m, v), (lr, b1, b2, eps, wd, step, dec) = adam
                self.mod.adam_flat(p, self.flat.grad, m, v, None, lr, b1, b2, eps, wd, step, 1.0, bool(dec), False,
                                   None, None)
            else:
                self.optimizer.step()
        return stats

    def warmup(self, features: Tensor, labels: Tensor, idx: Optional[Tensor]) -> None:
        """Forward + BPTT + gradient reduction of one batch with the result
        discarded: loads the kernels' code objects and sizes the allocator's
        workspace for this batch shape.  Parameters and optimizer state are not
        touched; the flat gradient (fully rewritten by every step) is zeroed."""
        from ..ops.lstm import fused_bwd_nb, gru_fwd_nb, small_launch_config
        self.flat.attach_grads()
        batch = idx.numel() if idx is not None else features.shape[0]
        nb_fwd, sp_fwd, _, _ = small_launch_config(batch, self.H, self.NL)
        nb_bwd = fused_bwd_nb(batch, self.H, self.NL)
        if self.gru:  # (gate-split family geometry; the sequence-in-wave kernels, H = 32, ignore it)
            nb_fwd, sp_fwd = gru_fwd_nb(batch, self.H, features.device), 1
        ws, features, cell = self._operands(features)
        stats = torch.zeros(3, dtype=torch.float32, device=self.flat.grad.device)
        # the single-process step folds Adam into its reduction: warm THAT
        # kernel variant too (its first launch pays the code-object load), on
        # scratch copies of the parameters and moments -- nothing real moves
        adam_bufs = adam_hp = None
        if self.grad_sync is None:
            st = self._flat_adam_peek()
            if st is not None:
                (p, m, v), adam_hp = st
                adam_bufs = [p.clone(), m.clone(), v.clone()]
        self.mod.lstm_head_train_step(features, idx, labels, ws, self.m.fc.weight, self.m.fc.bias, self.flat.grad,
                                      stats, self.H, self.NL, sp_fwd, 0, nb_fwd, nb_bwd, adam_bufs, adam_hp,
                                      cell, self.colmap, round_bf16=self.bf16)
        self.flat.grad.zero_()

    def _flat_adam_peek(self):
        """_flat_adam's operands without advancing the step count."""
        opt = self.optimizer
        g = opt.param_groups[0] if len(opt.param_groups) == 1 else None
        fs = opt._group_flat(0, g) if g is not None and hasattr(opt, "_group_flat") else None
        if fs is None:
            return None
        res = self._flat_adam()
        if res is not None:
            fs["step"] -= 1.0  # undo the advance
        return res

    # ------------------------------------------------------------ HIP graph
    # captured steps are kept per configuration (full and short last batch of
    # an epoch alternate: no re-capture every epoch)
    _GRAPHS_MAX = 4

    def _graph_step(self, features: Tensor, labels: Tensor, idx: Optional[Tensor], nb_fwd,
                    nb_bwd: int, adam, stats: Tensor, slot: int) -> bool:
        """Run the synced step as a graph replay.  False: run it eagerly --
        the first two steps of a configuration, so that RCCL's lazy connection
        setup and the kernels' first-use allocations happen outside the
        capture (the GRU's packing writes a persistent buffer: captured too)."""
        if idx is None:
            return False  # host-gathered batches change pointers every step
        (p, m, v), (lr, b1, b2, eps, wd, step, dec) = adam
        key = (features.data_ptr(), tuple(features.shape), features.dtype, labels.data_ptr(), labels.numel(),
               (idx.numel(), idx.dtype), nb_fwd, nb_bwd, lr, b1, b2, eps, wd, dec,
               p.data_ptr(), m.data_ptr(), v.data_ptr(), self.flat.grad.data_ptr())
        graphs = self.__dict__.setdefault("_graphs", {})
        ent = graphs.get(key)
        if ent is None:
            ent = {"graph": None, "eager": 0}
            if len(graphs) >= self._GRAPHS_MAX:
                graphs.pop(next(iter(graphs)))
            graphs[key] = ent
        if ent["graph"] is None:
            ent["eager"] += 1
            if ent["eager"] <= 2:
                return False
            try:
                self._capture(ent, features, labels, idx, nb_fwd, nb_bwd, adam, slot)
            except Exception as exc:  # capture unsupported here: stay eager for good
                import warnings
                warnings.warn(f"HIP graph capture of the synced step failed ({exc!r}); running eagerly")
                torch.cuda.synchronize(self.flat.grad.device)
                graphs.clear()
                self.cuda_graph = False
                return False
        self._graph = ent["graph"]
        # the graph's Adam launch uses (device step count + 1) and stores it back
        if ent["step_host"] != step - 1.0:
            ent["step"].fill_(step - 1.0)
        ent["idx"].copy_(idx, non_blocking=True)
        with trace_range("pdrnn.graph_step"):
            ent["graph"].replay()
        if self.comm is not None and hasattr(self.comm, "track_current"):
            self.comm.track_current()  # the communicator's watchdog bounds the replay
        ent["step_host"] = step
        # the graph wrote the statistics into ring row (step - 1 + slot_off):
        # the row assigned to this step whenever the host's ring slot and step
        # count advanced together since the capture (the usual case); else
        # one copy moves them
        row = (int(step) - 1 + ent["slot_off"]) % self.RING
        if row != slot:
            stats.copy_(self.ring[row], non_blocking=True)
        return True

    def _capture(self, ent: dict, features: Tensor, labels: Tensor, idx: Tensor, nb_fwd, nb_bwd: int, adam,
                 slot: int):
        (p, m, v), (lr, b1, b2, eps, wd, step, dec) = adam
        dev = self.flat.grad.device
        hw, hb = self.m.fc.weight, self.m.fc.bias
        ent["idx"] = idx.clone()
        # statistics go straight into the epoch ring: row = device step count
        # (before this step's Adam advances it) + slot_off
        ent["slot_off"] = (slot - (int(step) - 1)) % self.RING
        ent["step"] = torch.zeros(1, dtype=torch.float32, device=dev)
        ent["ticket"] = torch.zeros(1, dtype=torch.int32, device=dev)
        ent["step_host"] = None
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            nb, sp = nb_fwd  # (sequences per forward workgroup, forward lanes per unit)
            ws, feats, cell = self._operands(features)  # GRU: the re-pack is part of the graph
            self.mod.lstm_head_train_step(feats, ent["idx"], labels, ws, hw, hb, self.flat.grad, self.ring,
                                          self.H, self.NL, sp, 0, nb, nb_bwd, None, None, cell, self.colmap,
                                          ent["step"], ent["slot_off"], round_bf16=self.bf16)
            self.grad_sync()
            self.mod.adam_flat(p, self.flat.grad, m, v, None, lr, b1, b2, eps, wd, step, 1.0, bool(dec), False,
                               None, ent["step"], ent["ticket"])
        ent["graph"] = g
