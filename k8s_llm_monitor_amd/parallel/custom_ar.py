"""One-shot IPC all-reduce for latency-bound tensor-parallel decode messages (custom_ar.hip).

Every TP rank registers a double-buffered staging buffer and a signal block, exchanges their IPC
handles over the CPU gloo group, and maps every peer's (``hipIpcOpenMemHandle``, xGMI peer
access).  ``all_reduce_(x)`` is then ONE kernel launch, hipGraph-capturable, that stages x, flags
every peer and sums all ranks' slices in rank order - one xGMI hop reading all peers at once,
instead of a ring's 2(W-1) latency-bound hops over one link.  Messages larger than the staging
buffer (prefill activations) keep RCCL (``parallel/comm.tp_all_reduce`` picks per call).

The same protocol provides a one-shot all-gather (the vocab-parallel logits, C-4), so a TP decode
step captured in a hipGraph contains no RCCL call at all.

On by default at TP 2..8 on the GPU (``K8SLLM_CUSTOM_AR=0`` keeps RCCL for everything), but only
after a startup self-test on the actual devices is exact (``self_test``: integer-valued bf16
all-reduces (one- and two-shot), all-gathers, all-to-alls and fused decode tails against CPU-group
references, exact in any summation order, as RCCL's are);
a rank that sees a mismatch or a raised error flag turns it off on every rank of the group.
Validated on one MI355X with two processes sharing the GPU (tests/test_custom_ar.py,
tests/test_tp_gpu.py); no multi-GPU xGMI run exists yet, which is what the self-test guards.
A call whose peer never arrives sets the error flag instead of hanging; the engine enqueues a copy
of the flag after every step (``error_async``) and fails the step if it was set.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist

DEFAULT_MAX_BYTES = 16 << 20  # >= 64 rows x 64128 bf16 (TP=2 logits shard) and 64 x 8192 activations
DEFAULT_SPIN_LIMIT = 4_000_000  # polls before a missing peer is declared failed (seconds, not forever)


class CustomAllReduce:
    def __init__(self, rank: int, world: int, cpu_group=None, max_bytes: int = DEFAULT_MAX_BYTES,
                 spin_limit: int = DEFAULT_SPIN_LIMIT):
        from ..ops import native

        if world < 2 or world > 8:
            raise ValueError("custom all-reduce supports 2..8 ranks")
        self.rank, self.world = rank, world
        self.n_a2a_launches = 0
        self.max_elems = (max_bytes // 2) // 8 * 8
        self.spin_limit = int(spin_limit)
        self._n = native()
        self.state, handles = self._n.car_create(rank, world, self.max_elems)
        gathered: list = [None] * world
        dist.all_gather_object(gathered, handles, group=cpu_group)
        self._n.car_open(self.state, b"".join(gathered))
        if cpu_group is not None or dist.is_initialized():
            dist.barrier(group=cpu_group)  # every rank mapped every peer before the first call

    def fits(self, x: torch.Tensor) -> bool:
        return (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and x.numel() % 8 == 0
                and 0 < x.numel() <= self.max_elems)

    def fits_gather(self, x: torch.Tensor) -> bool:
        return self.fits(x)

    def all_gather(self, x: torch.Tensor) -> torch.Tensor:
        """[world, *x.shape]: every rank's x in rank order (x must satisfy ``fits_gather``)."""
        out = torch.empty((self.world,) + tuple(x.shape), dtype=x.dtype, device=x.device)
        self._n.car_all_gather(self.state, x, out, self.spin_limit)
        return out

    def error_async(self, host_flag: torch.Tensor) -> None:
        """Enqueue a copy of the error flag into ``host_flag`` (pinned int32) on the current stream."""
        self._n.car_error_async(self.state, host_flag)

    def all_reduce_(self, x: torch.Tensor, algo: int = -1) -> torch.Tensor:
        """In-place sum over the group (x must satisfy ``fits``).  ``algo``: 0 one-shot, 1 two-shot
        (reduce-scatter + all-gather in one launch), -1 auto (two-shot from 512 KiB at TP > 2)."""
        self._n.car_all_reduce(self.state, x, x, self.spin_limit, algo)
        return x

    def all_reduce(self, x: torch.Tensor, algo: int = -1) -> torch.Tensor:
        out = torch.empty_like(x)
        self._n.car_all_reduce(self.state, x, out, self.spin_limit, algo)
        return out

    def fits_a2a(self, x: torch.Tensor) -> bool:
        """x [world, ...] bf16 with a per-destination block of a multiple of 8 elements."""
        return (self.fits(x) and x.shape[0] == self.world and (x.numel() // self.world) % 8 == 0)

    def all_to_all(self, x: torch.Tensor) -> torch.Tensor:
        """out[p] = rank p's x[this rank] for x [world, ...] (fixed equal blocks; graph-capturable)."""
        out = torch.empty_like(x)
        self._n.car_all_to_all(self.state, x, out, self.spin_limit)
        self.n_a2a_launches += 1  # host-side launches (graph captures included, replays not)
        return out

    def fits_tail(self, M: int, d: int) -> bool:
        return 0 < M <= 256 and d % 32 == 0 and d <= 8192 and M * d <= self.max_elems

    def fused_tail(self, slabs: torch.Tensor, nslabs: int, residual: torch.Tensor, norm_w: torch.Tensor, eps: float,
                   out: torch.Tensor, packed: bool, algo: int = -1) -> torch.Tensor:
        """The TP row-parallel tail of a decode layer in ONE launch: this rank's split-K slabs
        [nslabs, M, d] summed, all-reduced over the group, ``residual += `` the result, RMSNorm * w
        written to ``out`` (row-major, or fragment-packed for the next skinny GEMM).  ``algo``: 0
        one-shot, 1 two-shot (each rank reduces 1/world of the columns, then gathers the rest:
        2 (W - 1) / W rows over the links instead of W - 1), -1 auto (two-shot from 512 KiB at
        TP > 2, e.g. Llama-3-70B TP=8 decode: 64 x 8192); both give bit-identical results."""
        self._n.car_fused_tail(self.state, slabs, nslabs, residual, norm_w, out, eps, packed, self.spin_limit, algo)
        return out

    def error(self) -> bool:
        """True if a call gave up waiting for a peer (its output was invalid)."""
        return self._n.car_error(self.state) != 0

    def close(self) -> None:
        if self.state:
            self._n.car_destroy(self.state)
            self.state = 0


def enabled() -> bool:
    return os.environ.get("K8SLLM_CUSTOM_AR", "1") != "0"


def self_test(car: CustomAllReduce, ps, sizes=None) -> bool:
    """Collective over the TP group: every custom collective the engine routes through IPC, run on
    the real devices against exact references built over the CPU group, on integer-valued bf16
    data (every sum stays an integer of magnitude < 256, exact in any summation order - what RCCL
    returns too).  Covered: the all-reduce one-shot AND two-shot, the all-gather (vocab-parallel
    logits), the all-to-all (EP decode dispatch / combine) and the fused decode tail (slab sum +
    all-reduce + residual add + RMSNorm, one-shot and two-shot, row-major and fragment-packed: the
    Llama-3-70B TP=8 decode hot path) - residual bit-exact, the RMSNorm output within bf16
    rounding of the fp32 reference and one-shot == two-shot bit for bit.  A cross-device
    visibility or ordering fault in any of them therefore turns the custom path off on every rank
    (RCCL carries everything) instead of producing wrong tokens.  True on every rank only if every
    rank passed."""
    from .. import ops

    dev = ps.device
    world, rank, grp = car.world, ps.tp_rank, ps.cpu_group
    sizes = sizes or (8, 4096, 64 * 4096, car.max_elems)
    ok = True

    def gather_cpu(t: torch.Tensor) -> list:
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t.contiguous(), group=grp)
        return parts

    try:
        for n in sizes:
            n = max(8, min(int(n), car.max_elems)) // 8 * 8
            g = torch.Generator().manual_seed(7919 + n)
            xc = (torch.randint(-8, 9, (n,), generator=g) + rank).to(torch.bfloat16)
            x = xc.to(dev)
            ref = xc.float()
            dist.all_reduce(ref, group=grp)
            ref = ref.to(torch.bfloat16)
            ys = [car.all_reduce(x, algo=a) for a in (0, 1)]  # one-shot, two-shot
            m = min(n, car.max_elems // world // 8 * 8)
            gat = car.all_gather(x[:m].contiguous())
            torch.cuda.synchronize(dev)
            ok = (ok and all(torch.equal(y.cpu(), ref) for y in ys)
                  and torch.equal(gat.cpu(), torch.stack(gather_cpu(xc[:m]))) and not car.error())
        # all-to-all: out[p] = rank p's x[this rank]
        for blk in (8, 64 * 128):
            if world * blk > car.max_elems:
                continue
            g = torch.Generator().manual_seed(31 * blk + rank)
            xc = torch.randint(-100, 101, (world, blk), generator=g).to(torch.bfloat16)
            got = car.all_to_all(xc.to(dev))
            parts = gather_cpu(xc)
            torch.cuda.synchronize(dev)
            ok = ok and torch.equal(got.cpu(), torch.stack([parts[p][rank] for p in range(world)])) and not car.error()
        # the fused decode tail
        for M, d, ns, packed in ((8, 1024, 2, False), (17, 8 * 512, 2, True)):
            if not car.fits_tail(M, d):
                continue
            g = torch.Generator().manual_seed(1000 * M + d + rank)
            slabs = torch.randint(-3, 4, (ns, M, d), generator=g).float()
            res = torch.randint(-8, 9, (M, d), generator=g).to(torch.bfloat16)
            w = (1 + torch.randint(-4, 5, (d,), generator=g).float() / 16).to(torch.bfloat16)
            part = slabs.sum(0).to(torch.bfloat16).reshape(-1)
            y = torch.zeros_like(part, dtype=torch.float32)
            for p in gather_cpu(part):  # rank order, fp32, one rounding
                y += p.float()
            r2 = (res.float() + y.reshape(M, d)).to(torch.bfloat16)
            rf = r2.float()
            ref_out = rf * torch.rsqrt(rf.pow(2).mean(-1, keepdim=True) + 1e-5) * w.float()
            outs = []
            for algo in ((0, 1) if d % (8 * world) == 0 else (0,)):
                rg = res.to(dev)
                out = (ops.packed_empty(M, d, torch.bfloat16, dev) if packed
                       else torch.empty(M, d, dtype=torch.bfloat16, device=dev))
                car.fused_tail(slabs.to(dev).contiguous(), ns, rg, w.to(dev), 1e-5, out, packed, algo=algo)
                torch.cuda.synchronize(dev)
                got = out.cpu()
                if packed:
                    got = ops.unpack_skinny(got.view(-1, d // 32, 64, 8))[:M]
                err = (got.float() - ref_out).abs().max().item()
                ok = (ok and torch.equal(rg.cpu(), r2) and err <= 2e-2 * ref_out.abs().max().item()
                      and not car.error())
                outs.append(got)
            ok = ok and all(torch.equal(o, outs[0]) for o in outs)
    except Exception:  # noqa: BLE001 - any failure disables the custom path
        ok = False
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=grp)
    return bool(flag.item())


def maybe_create(ps) -> Optional[CustomAllReduce]:
    """Collective over the TP group: a CustomAllReduce on the GPU at TP 2..8 (unless disabled),
    kept only if its startup self-test against RCCL passes on every rank."""
    if not (enabled() and ps.tp_size > 1 and ps.tp_size <= 8 and ps.device.type == "cuda"):
        return None
    car = CustomAllReduce(ps.tp_rank, ps.tp_size, cpu_group=ps.cpu_group)
    if not self_test(car, ps):
        import logging

        logging.getLogger("parallel").warning("custom all-reduce failed its startup self-test: RCCL carries "
                                              "every TP collective")
        car.close()
        return None
    return car
