"""Data-parallel training over the GPUs of one node (one process per GPU).

Global batch L = G*l: rank k owns examples [b*L + k*l, b*L + (k+1)*l) of global batch b
and the matching columns of the per-epoch (s, N) negative arrays, which every rank draws
identically from the shared seed (learning/OieInduction.py:183-184).  The forward kernel
writes rank k's per-example records into rows [k*l, (k+1)*l) of the exchange buffer; one
in-place all-gather (RCCL over xGMI; gloo on CPU) gives every rank all L records; every
rank then runs the identical deterministic update, so the replicas stay bit-identical.

This is the same gradient as a dense all-reduce of dW (d,m), dA (n,r), dAb (n), dC (r,m)
summed over ranks -- at 0.52 MB per rank per step instead of >200 MB for the dense
gradients at the headline shape.

Partitioned update (dp_update="partitioned", include/rae.h RAE_DPUPD_PARTITIONED): rank k
updates only the A / Ab / W rows it owns (row % G == k) and, before each forward, every owner
sends each peer the rows that peer's examples read (Exchange.rows, an all-to-all); replicas
differ in rows nobody read recently until Exchange.sync_rows gathers them.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env_world():
    """(world_size, rank, local_rank) from torchrun's environment (1, 0, 0 without it)."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rk = int(os.environ.get("RANK", "0"))
    lr = int(os.environ.get("LOCAL_RANK", str(rk)))
    return ws, rk, lr


def init(backend: str | None = None):
    ws, rk, lr = env_world()
    if ws > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # RAE_DIST_BACKEND=gloo: host-staged collectives (ranks sharing one GPU, tests only)
        backend = backend or os.environ.get("RAE_DIST_BACKEND") or None
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(lr)
            kw["device_id"] = torch.device("cuda", lr)
        dist.init_process_group(backend=backend, rank=rk, world_size=ws, **kw)
    return ws, rk, lr


class Exchange:
    """The collectives of one data-parallel plan (one process per GPU).

    exchange(buf)            in-place all-gather of the per-example records: rank k's slice is
                             rows [k*l, (k+1)*l) of the global batch.
    exchange.rows(send, recv)
                             all-to-all of equal peer blocks (partitioned update: owners send
                             the rows each peer's next forward reads, include/rae.h rae_dp_*).
    exchange.max_int(v)      max over ranks (the row-list capacities every rank must agree on).
    exchange.sync_rows(ts)   gather, for every tensor, row x from its owner x % G (replicas of
                             the partitioned update made identical: labelling, checkpoints).

    RCCL ("nccl" backend) moves the device buffers in place, stream-ordered, so the records and
    rows collectives can sit inside a captured HIP graph.  The gloo backend (CPU tests; several
    ranks sharing one GPU) has no device path: buffers are staged through host memory, which
    synchronises the stream, so that mode runs eagerly (graph_chunk=1)."""

    def __init__(self, world_size: int, rank: int, group=None):
        self.world_size = world_size
        self.rank = rank
        self.group = group

    def _staged(self, t):
        return t.is_cuda and dist.get_backend(self.group) != "nccl"

    def __call__(self, buf: torch.Tensor):
        n = buf.numel() // self.world_size
        rk = self.rank
        if self._staged(buf):
            host = buf.cpu()
            dist.all_gather_into_tensor(host, host[rk * n:(rk + 1) * n].clone(), group=self.group)
            buf.copy_(host)
        elif not buf.is_cuda:
            dist.all_gather_into_tensor(buf, buf[rk * n:(rk + 1) * n].clone(), group=self.group)
        else:
            dist.all_gather_into_tensor(buf, buf[rk * n:(rk + 1) * n], group=self.group)

    def rows(self, send: torch.Tensor, recv: torch.Tensor):
        if self._staged(send):
            hs = send.cpu()
            hr = torch.empty_like(hs)
            dist.all_to_all_single(hr, hs, group=self.group)
            recv.copy_(hr)
        else:
            dist.all_to_all_single(recv, send, group=self.group)

    def all_gather_object(self, obj):
        """Every rank's `obj` (a picklable Python object), in rank order -- set-up only (the
        peer-to-peer exchange's IPC handles)."""
        out = [None] * self.world_size
        dist.all_gather_object(out, obj, group=self.group)
        return out

    def barrier(self):
        """Host barrier of the ranks (the peer-to-peer exchange's run starts: no rank queues a
        step whose wait kernel would spin while a peer is still in host code)."""
        dist.barrier(group=self.group)

    def max_int(self, v: int) -> int:
        dev = torch.device("cuda", torch.cuda.current_device()) if \
            dist.get_backend(self.group) == "nccl" else torch.device("cpu")
        t = torch.tensor([int(v)], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return int(t.item())

    def sync_rows(self, tensors):
        """Row x of every tensor (dim 0) is current on rank x % G: gather every row from its
        owner, so all replicas hold identical tensors (bitwise copies, no arithmetic)."""
        G, rk = self.world_size, self.rank
        for t in tensors:
            if t is None:
                continue
            n = t.shape[0]
            per = -(-n // G)
            mine = t[rk::G]
            buf = torch.zeros((per,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
            buf[:mine.shape[0]] = mine
            staged = self._staged(t)
            src = buf.cpu() if staged else buf
            out = torch.empty((G * per,) + tuple(t.shape[1:]), dtype=t.dtype, device=src.device)
            dist.all_gather_into_tensor(out, src, group=self.group)
            out = out.to(t.device)
            for k in range(G):
                cnt = len(range(k, n, G))
                t[k::G] = out[k * per:k * per + cnt]


def make_exchange(world_size: int, rank: int, group=None):
    """The Exchange of a world_size > 1 data-parallel run (None for one rank)."""
    if world_size == 1:
        return None
    return Exchange(world_size, rank, group)


def warm_up(exchange, buf):
    """Run one collective eagerly so the communicator exists before graph capture."""
    if exchange is not None:
        exchange(buf)
        if buf.is_cuda:
            torch.cuda.synchronize(buf.device)


def max_over_ranks(x: float) -> float:
    if not dist.is_initialized():
        return x
    dev = torch.device("cuda", torch.cuda.current_device()) if \
        dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier():
    if dist.is_initialized():
        dist.barrier()
