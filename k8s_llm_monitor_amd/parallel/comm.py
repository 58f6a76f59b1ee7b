"""Tensor-parallel collectives.

Every function is a no-op at tp_size 1 and is safe inside a hipGraph capture (RCCL collectives
are capturable on the current stream).  Message sizes at Llama-3-70B TP=8 decode are
[B, 8192] bf16 (1 MiB at B=64): latency-bound on xGMI, so the engine issues exactly two per
layer and never splits them into buckets.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from .state import get_state


def _rccl(st, x: torch.Tensor) -> bool:
    """Device tensor on an RCCL group (gloo groups - CPU runs, or several ranks sharing one GPU in
    tests - lack the *_into_tensor collectives)."""
    return x.is_cuda and dist.get_backend(st.tp_group) == "nccl"


def tp_all_reduce(x: torch.Tensor, ps=None) -> torch.Tensor:
    """In-place sum over the TP group (C-1 / C-2 / C-3): the one-shot IPC all-reduce for messages
    that fit its staging buffer (decode), RCCL for the rest (prefill)."""
    st = ps or get_state()
    if st.tp_size == 1:
        return x
    car = st.custom_ar
    if car is not None and car.fits(x):
        return car.all_reduce_(x)
    dist.all_reduce(x, op=dist.ReduceOp.SUM, group=st.tp_group)
    return x


class _Done:
    """A completed collective (TP 1, or one that ran synchronously)."""

    def wait(self) -> None:
        pass


_DONE = _Done()


class _StreamWork:
    """An all-reduce queued on the comm stream: ``wait()`` makes the current stream wait for it."""

    __slots__ = ("ev",)

    def __init__(self, ev):
        self.ev = ev

    def wait(self) -> None:
        torch.cuda.current_stream().wait_event(self.ev)


_COMM_STREAMS: dict = {}


def comm_stream(device: torch.device):
    """The process's high-priority stream for IPC collectives issued asynchronously (one per
    device, so those collectives keep program order among themselves on every rank)."""
    s = _COMM_STREAMS.get(device)
    if s is None:
        s = _COMM_STREAMS[device] = torch.cuda.Stream(device=device, priority=-1)
    return s


def tp_all_reduce_async(x: torch.Tensor, ps=None):
    """In-place sum over the TP group, returned as a handle whose ``wait()`` must precede any use
    of ``x``; compute queued on the current stream between the call and ``wait()`` overlaps the
    collective, and ``wait()`` blocks the current stream, never the host.

    RCCL runs the collective on the process group's own stream.  A message that fits the IPC
    staging buffer goes to the one-launch custom all-reduce on ``comm_stream``: the comm stream
    first waits for the work already queued on the current stream (the producer of ``x``), so
    every rank issues its IPC collectives in program order - the same total order the synchronous
    calls have - and the caller must wait() every handle before its next synchronous collective."""
    st = ps or get_state()
    if st.tp_size == 1:
        return _DONE
    car = st.custom_ar
    if car is not None and car.fits(x):
        cs = comm_stream(x.device)
        cs.wait_stream(torch.cuda.current_stream(x.device))
        with torch.cuda.stream(cs):
            car.all_reduce_(x)
        x.record_stream(cs)  # the caching allocator must not hand x out again before the reduce ran
        ev = torch.cuda.Event()
        ev.record(cs)
        return _StreamWork(ev)
    return dist.all_reduce(x, op=dist.ReduceOp.SUM, group=st.tp_group, async_op=True)


def tp_all_gather_last(x: torch.Tensor, ps=None) -> torch.Tensor:
    """Concatenate the last dim across the TP group, rank order (C-4: vocab-parallel logits)."""
    st = ps or get_state()
    if st.tp_size == 1:
        return x
    x = x.contiguous()
    car = st.custom_ar
    if car is not None and car.fits_gather(x):  # one-shot IPC gather (decode logits)
        out = car.all_gather(x)
    else:
        out = torch.empty((st.tp_size,) + tuple(x.shape), dtype=x.dtype, device=x.device)
        if _rccl(st, x):
            dist.all_gather_into_tensor(out, x, group=st.tp_group)
        else:  # gloo has no all_gather_into_tensor
            dist.all_gather(list(out.unbind(0)), x, group=st.tp_group)
    return out.movedim(0, -2).reshape(*x.shape[:-1], st.tp_size * x.shape[-1])


def tp_all_to_all(out: torch.Tensor, inp: torch.Tensor, out_splits: list, in_splits: list, ps=None) -> torch.Tensor:
    """Uneven all-to-all of rows over the TP group (C-5: MoE expert dispatch / combine)."""
    st = ps or get_state()
    if st.tp_size == 1:
        out.copy_(inp)
        return out
    dist.all_to_all_single(out, inp.contiguous(), out_splits, in_splits, group=st.tp_group)
    return out


def tp_all_gather_rows(x: torch.Tensor, ps=None) -> torch.Tensor:
    """Concatenate equal-shaped [n, ...] row blocks of every TP rank in rank order."""
    st = ps or get_state()
    if st.tp_size == 1:
        return x
    x = x.contiguous()
    car = st.custom_ar
    if car is not None and car.fits_gather(x):  # one-shot IPC gather (EP decode slices)
        return car.all_gather(x).reshape((st.tp_size * x.shape[0],) + tuple(x.shape[1:]))
    out = torch.empty((st.tp_size * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    if _rccl(st, x):
        dist.all_gather_into_tensor(out, x, group=st.tp_group)
    else:
        dist.all_gather(list(out.chunk(st.tp_size)), x, group=st.tp_group)
    return out


def tp_broadcast_object(obj, src_tp_rank: int = 0, ps=None):
    """Broadcast a picklable control message (the step schedule, C-6) from the TP leader over the
    CPU gloo group."""
    st = ps or get_state()
    if st.tp_size == 1:
        return obj
    lst = [obj]
    src = st.rank - st.tp_rank + src_tp_rank
    dist.broadcast_object_list(lst, src=src, group=st.cpu_group)
    return lst[0]


def shard_range(n: int, parts: int, idx: int) -> tuple[int, int]:
    """Contiguous shard [lo, hi) of n items; n must divide evenly (TP shapes always do)."""
    if n % parts != 0:
        raise ValueError(f"{n} is not divisible by tp_size {parts}")
    s = n // parts
    return idx * s, (idx + 1) * s


def kv_head_range(n_kv_heads: int, head_dim: int, parts: int, idx: int) -> tuple[int, int]:
    """Rows [lo, hi) of the K (or V) projection held by TP rank ``idx``.

    ``n_kv_heads % parts == 0``: contiguous shards of n_kv_heads / parts heads.  Fewer KV heads
    than ranks (e.g. 8 KV heads at TP 16, or the 2-KV-head test models at TP 4): each KV head is
    replicated on ``parts / n_kv_heads`` consecutive ranks - rank r holds head r // (parts /
    n_kv_heads), which is exactly the KV head of its query heads (the query heads of one GQA group
    are contiguous and split over those same ranks), so attention stays rank-local."""
    if n_kv_heads % parts == 0:
        return shard_range(n_kv_heads * head_dim, parts, idx)
    if parts % n_kv_heads != 0:
        raise ValueError(f"{n_kv_heads} KV heads cannot be sharded or replicated over tp_size {parts}")
    h = idx // (parts // n_kv_heads)
    return h * head_dim, (h + 1) * head_dim


def all_reduce_max_scalar(v: float, group: Optional[object] = None) -> float:
    """Max of a host float over the whole world (bench timing: max over ranks)."""
    if not (dist.is_available() and dist.is_initialized()):
        return v
    st = get_state()
    dev = st.device if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def all_reduce_sum_scalar(v: float, group: Optional[object] = None) -> float:
    if not (dist.is_available() and dist.is_initialized()):
        return v
    st = get_state()
    dev = st.device if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return float(t.item())
