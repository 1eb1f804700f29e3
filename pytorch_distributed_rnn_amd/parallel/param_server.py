"""Parameter-server training over torch RPC (TensorPipe) + distributed autograd.

Capability parity with the reference PS mode (reference:
src/motion/param_server/__init__.py:11-73, master.py:9-59, worker.py:17-112,
util.py:11-25): rank 0 hosts the ONLY model instance (created lazily, once,
under a lock, by the first worker's RPC); ranks 1..W-1 are trainers whose model
is a proxy (``RemoteModel``) that runs forward AND backward on the server
through ``rpc_sync`` inside a ``dist_autograd.context``; each trainer steps its
own ``DistributedOptimizer(Adam)`` over the server's parameter RRefs, applying
its gradients immediately (asynchronous, Hogwild-style -- no averaging).

MI355X-native differences:

* the server keeps the model (and the fused HIP LSTM kernels) on its GPU.
  Two payload paths (``--ps-payload``):

  - ``collective`` (default when every rank owns a GPU): RPC is only the
    control plane.  The batch, the logits and the logits' gradient travel by
    send/recv on a 2-rank process group {server, trainer} -- RCCL, GPU to
    GPU over xGMI, one communicator per trainer so the server's RPC threads
    never interleave two trainers on one communicator (gloo on CPU or
    shared-GPU runs).  The server back-propagates with ``autograd.grad``
    (per-trainer gradients, never summed into a shared ``.grad``) and steps
    that trainer's own Adam, the state the reference's DistributedOptimizer
    keeps per trainer on the parameters' owner;
  - ``rpc`` (the reference's path): payloads inside the RPC messages plus
    distributed autograd.  They are host-staged: TensorPipe in torch-ROCm 2.10
    has no device channel -- a CUDA tensor in an RPC fails with "Attempting
    to send a Tensor with unexpected device type cuda:0"
    (profiles/r2_ps_device_payload_tried.md);
* fixes of reference quirks, each behind a flag: trainers
  shard the data over the W-1 trainers (``--ps-legacy-sharding`` restores the
  reference's ``num_replicas=W`` sharding that never trains on shard 0);
  trainer 1 asks the server to write the checkpoint at the end (the reference
  never saves in PS mode); log lines go through ``logging`` at ``--log``
  level (the reference's PS path silently drops them).
"""
from __future__ import annotations

import logging
import os
import threading
from datetime import timedelta
from pathlib import Path
from typing import Optional

import torch
import torch.nn.functional as F
from torch import nn

from .. import _ext

PS_NAME = "parameter_server"
RPC_TIMEOUT_S = float(os.environ.get("PDRNN_RPC_TIMEOUT", 60))

_server_model = None
_server_lock = threading.Lock()
# trainer rank -> 2-rank payload group {0, rank} (collective payload mode)
_PAYLOAD_GROUPS = {}
_PAYLOAD_BACKEND = None


def _local_gpu_ok(rank: int, world_size: int) -> bool:
    """Can this rank own a GPU of its host?  From LOCAL_RANK / LOCAL_WORLD_SIZE
    when a launcher set them (multi-host jobs: the per-host count matters, not
    the global world size), else every rank of the job on this host."""
    if not torch.cuda.is_available():
        return False
    n = torch.cuda.device_count()
    lws = os.environ.get("LOCAL_WORLD_SIZE")
    if lws is not None:
        return n >= int(lws)
    lr = os.environ.get("LOCAL_RANK")
    if lr is not None:
        return n > int(lr)
    return n >= world_size


def _local_device_index(rank: int) -> int:
    return int(os.environ.get("LOCAL_RANK", rank))


def payload_mode(requested: str, world_size: int, rank: int = 0) -> str:
    """Local guess only (no agreement): ``auto`` -> collective iff this rank
    could own a GPU.  The job-wide decision is :func:`agree_payload`."""
    if requested != "auto":
        return requested
    return "collective" if _local_gpu_ok(rank, world_size) else "rpc"


_AGREE_STORE = None


def agree_payload(requested: str, rank: int, world_size: int, address: str, port: str,
                  timeout_s: Optional[float] = None):
    """Job-wide payload mode and backend: every rank publishes whether it can
    own a GPU on a TCPStore (rank 0 hosts it, port + 2) and all ranks apply
    the same rule to the same answers, so hosts with different GPU counts
    cannot disagree (a split decision would leave some ranks in the payload
    group rendezvous until it times out).  Returns (mode, backend): mode
    ``collective`` iff requested so, or ``auto`` and every rank owns a GPU;
    backend ``nccl`` (RCCL) iff every rank owns a GPU, else ``gloo``."""
    global _AGREE_STORE
    if requested == "rpc":
        return "rpc", None
    from torch.distributed import TCPStore
    import time
    t = timedelta(seconds=timeout_s if timeout_s is not None else max(RPC_TIMEOUT_S, 60.0))
    store = TCPStore(address, int(port) + 2, world_size, rank == 0, t)
    store.set(f"pdrnn_ps_gpu/{rank}", "1" if _local_gpu_ok(rank, world_size) else "0")
    keys = [f"pdrnn_ps_gpu/{r}" for r in range(world_size)]
    store.wait(keys, t)
    all_gpu = all(store.get(k) == b"1" for k in keys)
    # the store lives in rank 0: it may only go away once everyone has read
    store.add("pdrnn_ps_gpu_read", 1)
    if rank == 0:
        deadline = time.monotonic() + t.total_seconds()
        while store.add("pdrnn_ps_gpu_read", 0) < world_size:
            if time.monotonic() > deadline:
                raise TimeoutError("payload-mode agreement: not every rank read the decision")
            time.sleep(0.005)
    _AGREE_STORE = store if rank == 0 else None
    mode = requested if requested != "auto" else ("collective" if all_gpu else "rpc")
    return mode, ("nccl" if all_gpu else "gloo")


def init_payload_groups(rank: int, world_size: int, address: str, port: str,
                        backend: Optional[str] = None) -> None:
    """Process group for the tensor payloads, next to the RPC agent (port + 1).

    Backend: RCCL when every rank owns a GPU (device payloads, GPU<->GPU over
    xGMI), gloo otherwise (host payloads) -- as agreed by :func:`agree_payload`
    (every rank must pass the same one).  Every rank creates every pair
    group {0, r} in the same order (``new_group`` is collective); one
    communicator per trainer lets the server serve trainers from concurrent
    RPC threads without interleaving their send/recv on one communicator."""
    import torch.distributed as dist
    global _PAYLOAD_BACKEND
    if backend is None:
        backend = "nccl" if _local_gpu_ok(rank, world_size) else "gloo"
    _PAYLOAD_BACKEND = backend
    if backend == "nccl":
        torch.cuda.set_device(_local_device_index(rank) % torch.cuda.device_count())
    dist.init_process_group(_PAYLOAD_BACKEND, init_method=f"tcp://{address}:{int(port) + 1}", rank=rank,
                            world_size=world_size, timeout=timedelta(seconds=max(RPC_TIMEOUT_S, 60.0)))
    for r in range(1, world_size):
        _PAYLOAD_GROUPS[r] = dist.new_group([0, r])


def shutdown_payload_groups() -> None:
    import torch.distributed as dist
    _PAYLOAD_GROUPS.clear()
    if dist.is_initialized():
        dist.destroy_process_group()


def _payload_device(compute_device: torch.device) -> torch.device:
    return compute_device if _PAYLOAD_BACKEND == "nccl" else torch.device("cpu")


def _to_payload(t: torch.Tensor) -> torch.Tensor:
    return t.contiguous() if _PAYLOAD_BACKEND == "nccl" else t.cpu().contiguous()


def _on_device(device: torch.device):
    """RPC handler threads start on the default device: pin the server's."""
    import contextlib
    return torch.cuda.device(device) if device.type == "cuda" else contextlib.nullcontext()


# --------------------------------------------------------------------------- helpers
def call_method(method, rref, *args, **kwargs):
    """Run ``method(rref.local_value(), ...)`` on the owner of ``rref``."""
    return method(rref.local_value(), *args, **kwargs)


def remote_method(method, rref, *args, **kwargs):
    import torch.distributed.rpc as rpc
    return rpc.rpc_sync(rref.owner(), call_method, args=[method, rref] + list(args), kwargs=kwargs)


# --------------------------------------------------------------------------- server
class ServerModel:
    """The single model instance living on the parameter server."""

    def __init__(self, input_dim: int, hidden_dim: int, layer_dim: int, output_dim: int,
                 cell: str = "lstm"):
        from ..models.motion import MotionModel
        self.device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
            else torch.device("cpu")
        self.model = MotionModel(input_dim, hidden_dim, layer_dim, output_dim, cell=cell).to(self.device)
        if self.device.type == "cuda":
            from ..utils.flat import flatten_module
            flatten_module(self.model)  # one flat span: a trainer's Adam step is one adam_flat launch
        self.native_adam_steps = 0
        self.lock = threading.Lock()
        self.step_lock = threading.Lock()
        self._pending = {}  # trainer rank -> logits of its in-flight step (collective payloads)
        self._optims = {}   # trainer rank -> that trainer's Adam over the server's parameters

    def begin_step(self) -> bool:
        """Serialise one trainer's forward/backward/step transaction.

        Without it, trainer A's optimizer step rewrites parameters in place
        while trainer B's backward still needs the values its forward saw
        (autograd version-counter error, or silently stale gradients).  The
        update order between trainers stays asynchronous and un-averaged."""
        return self.step_lock.acquire(timeout=RPC_TIMEOUT_S)

    def end_step(self) -> None:
        if self.step_lock.locked():
            self.step_lock.release()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.model(x.to(self.device)).cpu()

    def get_dist_gradients(self, cid: int):
        import torch.distributed.autograd as dist_autograd
        grads = dist_autograd.get_gradients(cid)
        return {i: v.detach().cpu() for i, (_, v) in enumerate(grads.items())}

    def get_param_rrefs(self):
        import torch.distributed.rpc as rpc
        return [rpc.RRef(p) for p in self.model.parameters()]

    # ---------------------------------------------------- collective payloads
    # RPC carries only the control message; the batch, the logits and the
    # logits' gradient move over a 2-rank process group {server, trainer}
    # (RCCL send/recv GPU<->GPU on a node with one GPU per rank, gloo on the
    # CPU).  Forward and backward still run on the server, each trainer keeps
    # its own Adam state there (as the reference's DistributedOptimizer does:
    # one local optimizer per trainer on the parameters' owner), and the
    # gradients never leave the server.
    def forward_p2p(self, rank: int, shape, dtype: str) -> None:
        import torch.distributed as dist
        g = _PAYLOAD_GROUPS[rank]
        with _on_device(self.device):
            x = torch.empty(tuple(shape), dtype=getattr(torch, dtype), device=_payload_device(self.device))
            dist.recv(x, src=rank, group=g)
            out = self.model(x.to(self.device, non_blocking=True))
            self._pending[rank] = out
            dist.send(_to_payload(out.detach()), dst=rank, group=g)

    def backward_p2p(self, rank: int, lr: float) -> None:
        import torch.distributed as dist
        g = _PAYLOAD_GROUPS[rank]
        with _on_device(self.device):
            out = self._pending.pop(rank)
            dout = torch.empty(out.shape, dtype=out.dtype, device=_payload_device(self.device))
            dist.recv(dout, src=rank, group=g)
            params = [p for p in self.model.parameters() if p.requires_grad]
            # per-trainer gradients, never accumulated into the shared .grad
            # (a hogwild peer's backward may be running at the same time)
            grads = torch.autograd.grad(out, params, dout.to(self.device, non_blocking=True))
            with self.lock:  # one optimizer update at a time (torch's _LocalOptimizer.global_lock)
                opt = self._optims.get(rank)
                if opt is None:
                    # per-trainer flat moments over the server's flat parameter span:
                    # one adam_flat_kernel launch per step (torch.optim.Adam on the CPU)
                    from ..ops.adam import FusedAdam
                    opt = self._optims[rank] = FusedAdam(params, lr=lr)
                for p, gr in zip(params, grads):
                    p.grad = gr
                before = getattr(opt, "native_steps", 0)
                opt.step()
                for p in params:
                    p.grad = None
                # counted only when FusedAdam really ran the flat native kernel
                # (not its per-group reference fallback)
                if getattr(opt, "native_steps", 0) > before:
                    self.native_adam_steps += 1

    def save(self, path: str, epoch: int, loss: float) -> str:
        from ..train.checkpoint import save_checkpoint
        with self.lock:
            save_checkpoint(Path(path), epoch, self.model, None, loss)
        return path

    def state_dict(self):
        return {k: v.detach().cpu() for k, v in self.model.state_dict().items()}


def get_parameter_network(input_dim, hidden_dim, layer_dim, output_dim, cell="lstm"):
    """Singleton accessor, called remotely by every trainer (first call builds)."""
    global _server_model
    with _server_lock:
        if _server_model is None:
            _server_model = ServerModel(input_dim, hidden_dim, layer_dim, output_dim, cell)
        return _server_model


def _rpc_options(address: str, port: str):
    import torch.distributed.rpc as rpc
    return rpc.TensorPipeRpcBackendOptions(init_method=f"tcp://{address}:{port}",
                                           rpc_timeout=RPC_TIMEOUT_S)


def run_parameter_server(rank: int, world_size: int, address: str = "127.0.0.1",
                         port: str = "29500", payload: str = "rpc") -> None:
    import torch.distributed.rpc as rpc
    if torch.cuda.is_available():
        torch.cuda.set_device(0)
    logging.info("PS master initializing RPC")
    rpc.init_rpc(name=PS_NAME, rank=rank, world_size=world_size,
                 rpc_backend_options=_rpc_options(address, port))
    payload, backend = agree_payload(payload, rank, world_size, address, port)
    if payload == "collective":
        init_payload_groups(rank, world_size, address, port, backend)
        logging.info(f"Payload groups initialized ({_PAYLOAD_BACKEND})")
    logging.info("RPC initialized! Running parameter server...")
    rpc.shutdown(graceful=True)  # returns when every trainer has finished
    if _server_model is not None:
        logging.info(f"Server optimizer steps on the native flat Adam: {_server_model.native_adam_steps}")
    if payload == "collective":
        shutdown_payload_groups()
    logging.info("RPC shutdown on parameter server.")


# --------------------------------------------------------------------------- trainer side
class RemoteModel(nn.Module):
    """Trainer-side proxy: forward runs on the parameter server."""

    def __init__(self, input_dim, hidden_dim, layer_dim, output_dim, cell="lstm", payload: str = "rpc",
                 rank: Optional[int] = None):
        super().__init__()
        import torch.distributed.rpc as rpc
        self.param_server_rref = rpc.remote(PS_NAME, get_parameter_network,
                                            args=(input_dim, hidden_dim, layer_dim, output_dim, cell))
        self.payload = payload
        self.rank = rank
        self.output_dim = output_dim
        # collective payloads live on this trainer's GPU when the group is RCCL
        self.payload_device = torch.device("cuda", torch.cuda.current_device()) \
            if payload == "collective" and _PAYLOAD_BACKEND == "nccl" else torch.device("cpu")

    def get_global_param_rrefs(self):
        return remote_method(ServerModel.get_param_rrefs, self.param_server_rref)

    def forward(self, x, idx=None):
        if idx is not None:
            x = x.index_select(0, idx)
        if self.payload == "collective":
            return self._forward_p2p(x)
        return remote_method(ServerModel.forward, self.param_server_rref, x)

    def _forward_p2p(self, x):
        """Control message over RPC, batch and logits over the payload group.
        Returns the logits as a leaf: their gradient goes back with
        :meth:`backward_p2p`."""
        import torch.distributed as dist
        import torch.distributed.rpc as rpc
        g = _PAYLOAD_GROUPS[self.rank]
        x = x.to(self.payload_device).contiguous()
        fut = rpc.rpc_async(self.param_server_rref.owner(), call_method,
                            args=[ServerModel.forward_p2p, self.param_server_rref, self.rank, tuple(x.shape),
                                  str(x.dtype).rsplit(".", 1)[-1]], timeout=RPC_TIMEOUT_S)
        dist.send(x, dst=0, group=g)
        out = torch.empty(x.shape[0], self.output_dim, dtype=torch.float32, device=self.payload_device)
        dist.recv(out, src=0, group=g)
        fut.wait()
        return out.requires_grad_()

    def backward_p2p(self, dlogits: torch.Tensor, lr: float) -> None:
        """Send the logits' gradient; the server back-propagates it and steps
        this trainer's Adam on its parameters."""
        import torch.distributed as dist
        import torch.distributed.rpc as rpc
        fut = rpc.rpc_async(self.param_server_rref.owner(), call_method,
                            args=[ServerModel.backward_p2p, self.param_server_rref, self.rank, lr],
                            timeout=RPC_TIMEOUT_S)
        dist.send(dlogits.contiguous(), dst=0, group=_PAYLOAD_GROUPS[self.rank])
        fut.wait()


def _make_worker_trainer_cls():
    from ..data.loader import ShardedSampler
    from ..train.formatter import TrainingMessageFormatter
    from ..train.trainer import Trainer

    class ParameterWorkerTrainer(Trainer):
        def __init__(self, rank, world_size, model, training_set, batch_size, learning_rate,
                     validation_set=None, test_set=None, checkpoint_dir=None,
                     legacy_sharding: bool = False, hogwild: bool = False):
            self.rank = rank
            self.hogwild = hogwild
            self._world = world_size
            if legacy_sharding:
                sampler = ShardedSampler(len(training_set), num_replicas=world_size, rank=rank)
            else:
                sampler = ShardedSampler(len(training_set), num_replicas=world_size - 1, rank=rank - 1)
            eval_ok = rank == 0
            super().__init__(model=model, training_set=training_set, batch_size=batch_size,
                             learning_rate=learning_rate,
                             validation_set=validation_set if eval_ok else None,
                             test_set=test_set if eval_ok else None, checkpoint_dir=checkpoint_dir,
                             sampler=sampler, device=torch.device("cpu"), flatten=False, warmup=False)

        def world_size(self):
            return self._world

        def _get_formatter(self, epochs):
            return TrainingMessageFormatter(epochs, self.rank)

        def _get_optimizer(self, model, lr):
            self._lr = lr
            if model.payload == "collective":
                return None  # this trainer's Adam lives on the server (ServerModel.backward_p2p)
            from torch.distributed.optim import DistributedOptimizer
            return DistributedOptimizer(torch.optim.Adam, model.get_global_param_rrefs(), lr=lr)

        def _train_step(self, formatter):
            import torch.distributed.autograd as dist_autograd
            self.model.train()
            total_loss, total_correct = 0.0, 0
            batches = len(self.train_loader)
            rref = self.model.param_server_rref
            for batch_idx, (data, target) in enumerate(self.train_loader):
                if not self.hogwild:
                    remote_method(ServerModel.begin_step, rref)
                try:
                    loss_v, correct = self._one_step(data, target)
                finally:
                    if not self.hogwild:
                        remote_method(ServerModel.end_step, rref)
                total_loss += loss_v
                total_correct += correct
                self.sequences_seen += len(data)
                logging.info(formatter.train_progress_message(
                    batch_idx=batch_idx, batches=batches, training_examples=len(data),
                    correct=correct, loss=loss_v))
            n = len(self.train_loader.dataset)
            return total_loss / n, total_correct / n

        def _one_step(self, data, target):
            if self.model.payload == "collective":
                from ..ops.xent import cross_entropy_with_stats
                output = self.model(data)
                target = target.to(output.device).long().reshape(-1)
                # fused softmax-CE + argmax counts (one xent launch when the
                # logits arrive on this trainer's GPU over RCCL)
                loss, stats = cross_entropy_with_stats(output, target)
                loss.backward()
                self.model.backward_p2p(output.grad, self._lr)
                loss_v, _, correct = stats.tolist()
                return loss_v, int(correct)
            import torch.distributed.autograd as dist_autograd
            with dist_autograd.context() as cid:
                output = self.model(data)
                target = target.long().reshape(-1)
                loss = F.cross_entropy(output, target)
                loss_v = loss.item()
                correct = int((output.argmax(dim=1) == target).sum())
                dist_autograd.backward(cid, [loss])
                grads = remote_method(ServerModel.get_dist_gradients, self.model.param_server_rref, cid)
                assert grads, "distributed autograd produced no gradients on the server"
                self.optimizer.step(cid)
            return loss_v, correct

        def _save_checkpoint(self, epoch, loss, best=False):
            return None

    return ParameterWorkerTrainer


def run_worker(rank, world_size, epochs, batch_size, learning_rate, input_dim, hidden_dim, layer_dim,
               output_dim, train_set, validation_set, test_set, address="127.0.0.1", port="29500",
               legacy_sharding=False, checkpoint_dir: Optional[Path] = None, cell="lstm",
               hogwild: bool = False, payload: str = "rpc"):
    import torch.distributed.rpc as rpc
    logging.info(f"Worker rank {rank} initializing RPC")
    rpc.init_rpc(name=f"trainer_{rank}", rank=rank, world_size=world_size,
                 rpc_backend_options=_rpc_options(address, port))
    payload, backend = agree_payload(payload, rank, world_size, address, port)
    if payload == "collective":
        init_payload_groups(rank, world_size, address, port, backend)
    logging.info(f"Worker {rank} done initializing RPC")
    model = RemoteModel(input_dim, hidden_dim, layer_dim, output_dim, cell, payload=payload, rank=rank)
    cls = _make_worker_trainer_cls()
    trainer = cls(rank, world_size, model, train_set, batch_size, learning_rate, validation_set,
                  test_set, legacy_sharding=legacy_sharding, hogwild=hogwild)
    result = trainer.train(epochs)
    if checkpoint_dir is not None and rank == 1:
        path = Path(checkpoint_dir) / "best-model.pt"
        remote_method(ServerModel.save, model.param_server_rref, str(path), epochs - 1, float("nan"))
        logging.info(f"Worker {rank} asked the parameter server to save {path}")
    rpc.shutdown()
    if payload == "collective":
        shutdown_payload_groups()
    return trainer, result


# --------------------------------------------------------------------------- CLI
def add_sub_command(parent_parser):
    p = parent_parser.add_parser("parameter-server")
    p.add_argument("--world-size", type=int, required=True,
                   help="Total number of processes: the server plus every trainer.")
    p.add_argument("--rank", type=int, required=True, help="Global rank; 0 is the server.")
    p.add_argument("--master-address", type=str, default="localhost",
                   help="Address of the server (rank 0).")
    p.add_argument("--master-port", type=str, default="29500", help="Port of the server.")
    p.add_argument("--ps-legacy-sharding", action="store_true",
                   help="shard over all W ranks like the reference (shard 0 never trained)")
    p.add_argument("--ps-hogwild", action="store_true",
                   help="let trainers' forward/backward/step interleave on the server (reference "
                        "behaviour; races on in-place parameter updates)")
    p.add_argument("--ps-payload", choices=("auto", "rpc", "collective"), default="auto",
                   help="tensor payloads (batch, logits, logits' gradient): 'rpc' = inside the RPC "
                        "messages + distributed autograd (reference); 'collective' = RPC for control, "
                        "send/recv on a {server, trainer} process group (RCCL GPU<->GPU when every "
                        "rank owns a GPU, else gloo); 'auto' = collective iff every rank owns a GPU")
    p.set_defaults(func=execute)


def execute(args):
    logging.getLogger().setLevel(args.log)
    os.environ["MASTER_ADDR"] = args.master_address
    os.environ["MASTER_PORT"] = args.master_port
    address = "127.0.0.1" if args.master_address == "localhost" else args.master_address
    payload = getattr(args, "ps_payload", "auto")  # agreed across ranks in run_* (agree_payload)
    if args.rank == 0:
        run_parameter_server(0, args.world_size, address, args.master_port, payload=payload)
        return None
    torch.set_num_threads(args.num_threads)
    from ..cli import _load_datasets
    from ..data.motion import MotionDataset
    training_set, validation_set, test_set = _load_datasets(args)
    return run_worker(args.rank, args.world_size, args.epochs, args.batch_size, args.learning_rate,
                      training_set.num_features, args.hidden_units, args.stacked_layer,
                      len(MotionDataset.LABELS), training_set, validation_set, test_set,
                      address=address, port=args.master_port,
                      legacy_sharding=args.ps_legacy_sharding,
                      checkpoint_dir=args.checkpoint_directory if not args.no_validation else None,
                      cell=getattr(args, "cell", "lstm"), hogwild=args.ps_hogwild, payload=payload)
