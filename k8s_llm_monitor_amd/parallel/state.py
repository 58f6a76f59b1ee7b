"""Process-group state: one process per GPU, ``torch.distributed`` over RCCL (backend ``"nccl"``
is RCCL on ROCm) for device tensors and gloo for CPU tensors / control messages.

Layout of the world:

* ``tp``  - tensor-parallel group: Megatron column/row-parallel linears, vocab-parallel embedding
            and LM head; two all-reduces per layer.  On an 8-GPU MI355X node every pair of GPUs
            has its own xGMI link, so TP=8 is a full mesh; RCCL rings are per-link bound, which is
            why decode-sized all-reduces (<= 1 MiB) stay latency-bound and bucket sizes are chosen
            per call site, not globally.
* ``dp``  - independent engine replicas (``world // tp``).  No collectives on the hot path; the
            control plane routes requests round-robin.
* ``ep``  - expert parallel for Mixtral shares the TP group: attention activations are already
            replicated across it and each rank owns n_experts / tp experts.  Prefill dispatches
            (token, expert) rows to the owning rank by all-to-all and combines them by the reverse
            all-to-all (models/llama.py ``_moe_a2a``, the default, ``K8SLLM_MOE_COMM``); decode
            runs every local expert on the replicated rows and sums by all-reduce, or by the
            static-capacity all-to-all (``K8SLLM_MOE_DECODE=a2a``).

The reference has no GPU communication at all (SURVEY.md §2.11 "There is no NCCL, MPI, Gloo").
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class ParallelState:
    world_size: int = 1
    rank: int = 0
    local_rank: int = 0
    tp_size: int = 1
    tp_rank: int = 0
    dp_size: int = 1
    dp_rank: int = 0
    tp_group: Optional[object] = None  # device collectives (RCCL on GPU, gloo on CPU)
    cpu_group: Optional[object] = None  # gloo group spanning the TP group, for control broadcast
    bus_group: Optional[object] = None  # gloo group of the step bus: no serving timeout (idle waits)
    device: torch.device = torch.device("cpu")
    custom_ar: Optional[object] = None  # one-shot IPC all-reduce for small TP messages (custom_ar.py)

    @property
    def is_tp(self) -> bool:
        return self.tp_size > 1

    @property
    def tp_leader(self) -> bool:
        return self.tp_rank == 0


_STATE = ParallelState()


def get_state() -> ParallelState:
    return _STATE


def set_state(s: ParallelState) -> None:
    global _STATE
    _STATE = s


def env_world() -> tuple[int, int, int]:
    """(world_size, rank, local_rank) from torchrun-style env vars (1, 0, 0 when absent)."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    lr = int(os.environ.get("LOCAL_RANK", str(rank)))
    return ws, rank, lr


def init_parallel(tp_size: int = 1, device: Optional[str] = None, backend: Optional[str] = None,
                  timeout_s: float = 600.0) -> ParallelState:
    """Initialise torch.distributed (if WORLD_SIZE > 1) and carve the TP / DP groups.

    ``device`` defaults to ``cuda:<local_rank>`` when a GPU is visible, else CPU (gloo).
    Rehearsal overrides (several ranks sharing one GPU, e.g. the DP bench under torchrun on a
    1-GPU box): ``K8SLLM_DEVICE`` pins every rank's device, ``K8SLLM_DIST_BACKEND`` picks the
    process-group backend (gloo: RCCL refuses two ranks on one device).
    """
    import datetime

    ws, rank, lr = env_world()
    device = device or os.environ.get("K8SLLM_DEVICE") or None
    backend = backend or os.environ.get("K8SLLM_DIST_BACKEND") or None
    if device is None:
        device = f"cuda:{lr}" if torch.cuda.is_available() else "cpu"
    dev = torch.device(device)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    if tp_size < 1 or ws % tp_size != 0:
        raise ValueError(f"tp_size={tp_size} must divide world_size={ws}")
    st = ParallelState(world_size=ws, rank=rank, local_rank=lr, tp_size=tp_size, tp_rank=rank % tp_size,
                       dp_size=ws // tp_size, dp_rank=rank // tp_size, device=dev)
    if ws > 1:
        if not dist.is_initialized():
            be = backend or ("nccl" if dev.type == "cuda" else "gloo")
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29511")
            kw = {}
            if be == "nccl":
                kw["device_id"] = dev
            if os.environ.get("K8SLLM_EXTERNAL_STORE") == "1":
                # the launcher (bench.py spawn_ranks) hosts the store on a port it holds bound
                kw["store"] = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), ws + 1,
                                            is_master=False, timeout=datetime.timedelta(seconds=timeout_s))
            dist.init_process_group(be, rank=rank, world_size=ws,
                                    timeout=datetime.timedelta(seconds=timeout_s), **kw)
        be = dist.get_backend()
        # every rank must create every group, in the same order.  The TP groups start with the
        # start-up bound ``timeout_s``: their first collectives (custom all-reduce self-test and
        # handle exchange, step-bus set-up, identity exchange, warm-up and graph-capture
        # all-reduces) wait for the slowest rank's weight load.  serving_timeouts() lowers them to
        # K8SLLM_TP_TIMEOUT_S once the engine is warm (LLMEngine.warmup).  The step bus has a group
        # of its own that is never bounded: a worker waits in it for as long as the server is idle.
        up = datetime.timedelta(seconds=timeout_s)
        idle = datetime.timedelta(days=7)
        for g in range(ws // tp_size):
            ranks = list(range(g * tp_size, (g + 1) * tp_size))
            grp = dist.new_group(ranks, timeout=up) if tp_size > 1 else None
            cpu = (dist.new_group(ranks, backend="gloo", timeout=up) if (tp_size > 1 and be != "gloo")
                   else grp)
            bus = dist.new_group(ranks, backend="gloo", timeout=idle) if tp_size > 1 else None
            if rank in ranks:
                st.tp_group, st.cpu_group, st.bus_group = grp, cpu, bus
        from .custom_ar import maybe_create

        st.custom_ar = maybe_create(st)  # GPU, TP 2..8, self-test vs RCCL passed (K8SLLM_CUSTOM_AR=0: off)
    set_state(st)
    return st


def serving_timeouts(st: Optional[ParallelState] = None) -> None:
    """Lower the TP groups' collective timeout from the start-up bound to the serving bound
    (K8SLLM_TP_TIMEOUT_S, default 60 s): how long a rank can block on a dead peer before the
    process-group watchdog aborts it (the engine's PeerMonitor / step watchdog mark /health 503
    within seconds, parallel/health.py).  The step-bus group keeps no bound."""
    import datetime

    st = st or get_state()
    if st.tp_size == 1 or not (dist.is_available() and dist.is_initialized()):
        return
    to = datetime.timedelta(seconds=float(os.environ.get("K8SLLM_TP_TIMEOUT_S", "60")))
    from torch.distributed.distributed_c10d import _set_pg_timeout

    for g in {id(x): x for x in (st.tp_group, st.cpu_group) if x is not None}.values():
        _set_pg_timeout(to, g)


def barrier_all() -> None:
    if dist.is_available() and dist.is_initialized():
        st = get_state()
        if st.device.type == "cuda" and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[st.device.index])
        else:
            dist.barrier()


def destroy() -> None:
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
    set_state(ParallelState())
