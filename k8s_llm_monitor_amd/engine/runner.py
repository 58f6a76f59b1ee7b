"""Model runner: owns the paged KV cache, turns a StepPlan into device tensors, runs the model
and samples.

Decode steps are replayed from hipGraphs (``torch.cuda.CUDAGraph`` is hipGraph on ROCm) captured
once per batch-size bucket.  A bucket's graph reads static device buffers (token ids, positions,
slot mapping, block tables, sequence lengths, sampling parameters, RNG state) that the host
refreshes with a handful of async copies before each replay; the only host<->device sync per
step is reading back the sampled token ids.  Prefill runs eagerly (variable shapes).

KV-cache layouts are the ones the HIP kernels are written for (``ops/csrc/rope_cache.hip``):
K ``[NB, Hkv, D/8, 16, 8]`` and V ``[NB, Hkv, D, 16]`` per layer, one allocation for all layers
sized from ``kv_cache_gb`` (MI355X: 288 GB HBM per GPU - an 8B model leaves >250 GB for KV).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from .. import ops
from ..models.llama import AttnMeta, CausalLM
from .sequence import Sequence

BLOCK_SIZE = 16
DEFAULT_BUCKETS = (1, 2, 4, 8, 16, 24, 32, 40, 48, 56, 64, 80, 96, 112, 128, 160, 192, 224, 256)


@dataclass
class RunnerConfig:
    max_num_seqs: int = 64
    max_model_len: int = 8192
    kv_cache_gb: float = 16.0  # <= 0: max_num_seqs x max_model_len worth of blocks
    num_blocks: Optional[int] = None  # overrides kv_cache_gb
    use_graphs: bool = True
    seed: int = 0


class ModelRunner:
    def __init__(self, model: CausalLM, cfg: RunnerConfig):
        self.model = model
        self.cfg = cfg
        self.device = model.device
        c = model.cfg
        self.max_len = min(cfg.max_model_len, c.max_position)
        self.max_blocks_per_seq = (self.max_len + BLOCK_SIZE - 1) // BLOCK_SIZE
        L, hkv, D = c.n_layers, model.hkv, model.D
        per_block = 2 * L * hkv * D * BLOCK_SIZE * 2  # bytes (K + V, bf16)
        if cfg.num_blocks:
            nb = cfg.num_blocks
        elif cfg.kv_cache_gb <= 0:  # auto: every admitted sequence can reach max_len (+ one spare block)
            nb = cfg.max_num_seqs * self.max_blocks_per_seq + 1
        else:
            nb = max(self.max_blocks_per_seq + 1, int(cfg.kv_cache_gb * (1 << 30) // per_block))
        self.num_blocks = nb
        self.k_cache = torch.zeros(L, nb, hkv, D // 8, BLOCK_SIZE, 8, dtype=model.dtype, device=self.device)
        self.v_cache = torch.zeros(L, nb, hkv, D, BLOCK_SIZE, dtype=model.dtype, device=self.device)
        self.kv = [(self.k_cache[i], self.v_cache[i]) for i in range(L)]
        self.is_gpu = self.device.type == "cuda"
        B = cfg.max_num_seqs
        self.B = B
        dev = self.device
        # static decode inputs (graph inputs): views of ONE device buffer laid out like the pinned
        # host staging (_Staging), so a step's inputs go over in a single host-to-device copy
        self.d_all = torch.zeros(_Staging.size(B, self.max_blocks_per_seq), dtype=torch.int32, device=dev)
        (self.d_ids, self.d_src, self.d_pos, self.d_slots, self.d_lens, self.d_topk, self.d_temp, self.d_topp,
         self.d_bt) = _Staging.views(self.d_all, B, self.max_blocks_per_seq)
        self.d_src.fill_(-1)
        self.d_slots.fill_(-1)
        self.d_topp.fill_(1.0)
        self.rng = torch.tensor([cfg.seed, 0], dtype=torch.int64, device=dev)
        self.d_out = torch.zeros(B, dtype=torch.int32, device=dev)
        self.decode_ws = ops.decode_workspace(B, model.hq, D, self.max_blocks_per_seq * BLOCK_SIZE, dev, model.hkv) \
            if self.is_gpu else None
        # pinned host staging, double-buffered: with pipelined decode the host fills step N+1's
        # inputs while step N's host-to-device copies may still be queued
        self.stage = [_Staging(B, self.max_blocks_per_seq, self.is_gpu, idx=i) for i in range(2)]
        # the staging copy as the first node of each decode graph (one graph per staging buffer and
        # bucket): a replay then starts with its own inputs instead of a separate copy in front of it
        # (removes a ~100 us launch gap per decode step between the copy and the graph's first
        # kernel; profiles/r03/README.md)
        self.graph_h2d = True
        self._stage_i = 0
        self.h_out = [torch.zeros(B, dtype=torch.int32, pin_memory=self.is_gpu) for _ in range(2)]
        self._out_i = 0
        self._pf_bufs = [None, None]  # pinned prefill-input staging (_pf_stage)
        self._pf_i = 0
        self._pf_out = [None, None]  # pinned sampled tokens of in-flight prefill steps
        self._pf_oi = 0
        self.buckets = [b for b in DEFAULT_BUCKETS if b < B] + [B]
        self.graphs: dict[int, list] = {}  # bucket -> [graph] (or one graph per staging buffer)
        self.graph_pool = None
        self.n_steps = {"prefill": 0, "decode": 0}
        self.on_launched = None  # hook after every step's launch (TP: enqueue the custom-AR error readback)
        # TP > 1 prefill as two micro-batches whose all-reduces overlap the other's compute
        # (K8SLLM_TP_OVERLAP=0: one batch, serial all-reduces)
        self.overlap = model.overlap_ok()
        self._last_ev = None  # end event of the last launched step (_chain_event)

    # --------------------------------------------------------------------- helpers
    @staticmethod
    def _micro_split(cu: np.ndarray, nd: int, min_rows: int = 4096) -> int:
        """First sequence of the second prefill micro-batch: the split nearest half the rows (0:
        no split - a mixed step, a single sequence, or fewer than ``min_rows`` rows, where the
        all-reduces are small and halving the GEMMs' M costs more than the overlap hides)."""
        S = len(cu) - 1
        if nd or S < 2 or cu[S] < min_rows:
            return 0
        k = int(np.argmin(np.abs(cu[1:S] - cu[S] / 2))) + 1
        if min(cu[k], cu[S] - cu[k]) < min_rows // 4:
            return 0  # too lopsided: the short half would leave the tile GEMM (TILE_MIN_M rows)
        return k

    def bucket_for(self, n: int) -> int:
        for b in self.buckets:
            if b >= n:
                return b
        raise ValueError(f"batch {n} exceeds max_num_seqs {self.B}")

    def _sample(self, logits: torch.Tensor, temp, topk, topp, out=None) -> torch.Tensor:
        # fresh numbers next step: the counter advances inside the sampling kernel (also in a graph)
        return ops.sample(logits, temp, topk, topp, self.rng, out=out, advance=True)

    # --------------------------------------------------------------------- prefill
    def prefill(self, seqs: list[Sequence], decode: Optional[list] = None) -> list[int]:
        """One prefill (or mixed) step, synchronous: see :meth:`prefill_launch`."""
        return self.decode_collect(self.prefill_launch(seqs, decode))

    def _pf_stage(self, n: int) -> torch.Tensor:
        """Pinned int32 staging for one prefill step's inputs, alternating between two buffers
        (the previous step's copy may still be queued behind the step before it); grown on demand."""
        i = self._pf_i
        self._pf_i ^= 1
        buf = self._pf_bufs[i]
        if buf is None or buf.numel() < n:
            buf = torch.empty(max(n, 1 << 16) * 5 // 4, dtype=torch.int32, pin_memory=self.is_gpu)
            self._pf_bufs[i] = buf
        return buf

    def prefill_launch(self, seqs: list[Sequence], decode: Optional[list] = None) -> "DecodeHandle":
        """Enqueue each sequence's scheduled prefill chunk - tokens [num_computed, num_computed +
        chunk) of its prompt (+ any tokens generated before a preemption) - without waiting for it;
        the first num_computed tokens already have their KV in the cache (prefix-cache hits,
        earlier chunks) and are attended through the paged flash prefill.  ``decode`` (a mixed
        step): running sequences that also get their next token in this forward - their rows come
        first and attend through paged_decode.  The handle yields the sampled token of every decode
        row, then of every chunk (the first output token of the sequences whose prompt this step
        completes).  Every input goes over in ONE host-to-device copy from pinned memory, so a step
        can be enqueued while the previous one still runs (pipelined prefill)."""
        dev = self.device
        decode = decode or []
        nd = len(decode)
        starts = [s.num_computed for s in seqs]
        lens = [s.chunk or (s.num_tokens - c) for s, c in zip(seqs, starts)]
        T = nd + sum(lens)
        rows = list(decode) + list(seqs)
        R = len(rows)
        cu = np.zeros(len(seqs) + 1, dtype=np.int32)
        cu[1:] = np.cumsum(lens)
        qs, st = ops.prefill_qblocks(cu.tolist(), ctx_starts=starts)
        nq = len(qs)
        paged = any(starts)
        W = max(len(s.block_table) for s in seqs) if paged else 0
        Wd = max(len(q.block_table) for q in decode) if nd else 0
        # TP > 1: two micro-batches of whole sequences, so one's row-parallel all-reduces overlap
        # the other's compute (models/llama.py _prefill_overlap); their own cu_seqlens / q-block
        # schedules / logits rows ride in the same staging copy
        kA = self._micro_split(cu, nd) if self.overlap else 0
        mb = None
        if kA:
            cuA, cuB = cu[: kA + 1], cu[kA:] - cu[kA]
            mb = (ops.prefill_qblocks(cuA.tolist(), ctx_starts=starts[:kA]),
                  ops.prefill_qblocks(cuB.tolist(), ctx_starts=starts[kA:]))
        # layout of the staging buffer (int32 words; the float sampling parameters bit-cast)
        sizes = dict(ids=T, pos=T, slots=T, cu=len(seqs) + 1, qs=nq, st=nq, lidx=R, temp=R, topk=R, topp=R,
                     cst=len(seqs) if paged else 0, bt=len(seqs) * W, dbt=nd * Wd, dlen=nd,
                     mcu=len(seqs) + 2 if kA else 0, mqs=nq if kA else 0, mst=nq if kA else 0,
                     mlidx=len(seqs) if kA else 0)
        off, o = {}, 0
        for k, n in sizes.items():
            off[k] = o
            o += n
        buf = self._pf_stage(o)
        h = buf.numpy()
        v = {k: h[off[k]:off[k] + n] for k, n in sizes.items()}
        ids, pos, slots = v["ids"], v["pos"], v["slots"]
        for i, q in enumerate(decode):  # the token being fed is the last generated one
            p = q.num_tokens - 1
            ids[i] = q.last_token
            pos[i] = p
            slots[i] = q.block_table[p // BLOCK_SIZE] * BLOCK_SIZE + p % BLOCK_SIZE
        o = nd
        for s, c, n in zip(seqs, starts, lens):
            ch = getattr(s, "chunk_ids", None)  # TP worker views carry just the chunk
            ids[o:o + n] = ch if ch is not None else s.all_ids[c:c + n]
            p = np.arange(c, c + n, dtype=np.int32)
            pos[o:o + n] = p
            bt = np.asarray(s.block_table, dtype=np.int32)
            slots[o:o + n] = bt[p // BLOCK_SIZE] * BLOCK_SIZE + p % BLOCK_SIZE
            o += n
        v["cu"][:] = cu
        v["qs"][:] = qs
        v["st"][:] = st
        v["lidx"][:nd] = np.arange(nd, dtype=np.int32)
        v["lidx"][nd:] = nd + cu[1:] - 1
        v["temp"].view(np.float32)[:] = [s.params.temperature for s in rows]
        v["topk"][:] = [s.params.top_k for s in rows]
        v["topp"].view(np.float32)[:] = [s.params.top_p for s in rows]
        if paged:
            v["cst"][:] = starts
            bt2 = v["bt"].reshape(len(seqs), W)
            bt2[:] = 0
            for i, s in enumerate(seqs):
                bt2[i, : len(s.block_table)] = s.block_table
        if nd:
            dbt = v["dbt"].reshape(nd, Wd)
            dbt[:] = 0
            for i, q in enumerate(decode):
                dbt[i, : len(q.block_table)] = q.block_table
            v["dlen"][:] = [q.num_tokens for q in decode]
        if kA:
            v["mcu"][: kA + 1] = cuA
            v["mcu"][kA + 1:] = cuB
            nqA = len(mb[0][0])
            v["mqs"][:nqA], v["mst"][:nqA] = mb[0]
            v["mqs"][nqA:], v["mst"][nqA:] = mb[1]
            v["mlidx"][:kA] = cuA[1:] - 1
            v["mlidx"][kA:] = cuB[1:] - 1
        d = buf[: sum(sizes.values())].to(dev, non_blocking=True)
        dv = {k: d[off[k]:off[k] + n] for k, n in sizes.items()}
        meta = AttnMeta(is_prefill=True, positions=dv["pos"], slot_mapping=dv["slots"], cu_seqlens=dv["cu"],
                        qb_seq=dv["qs"], qb_start=dv["st"], logits_idx=dv["lidx"].long())
        if paged:
            meta.ctx_start = dv["cst"]
            meta.block_tables = dv["bt"].view(len(seqs), W)
        if kA:
            TA, S_ = int(cu[kA]), len(seqs)
            parts = []
            for (r0, r1), (s0, s1), (q0, q1) in ((((0, TA), (0, kA), (0, nqA))),
                                                 ((TA, T), (kA, S_), (nqA, nq))):
                m = AttnMeta(is_prefill=True, positions=dv["pos"][r0:r1], slot_mapping=dv["slots"][r0:r1],
                             cu_seqlens=dv["mcu"][s0 + (s0 > 0): s1 + 1 + (s0 > 0)], qb_seq=dv["mqs"][q0:q1],
                             qb_start=dv["mst"][q0:q1], logits_idx=dv["mlidx"][s0:s1].long())
                if paged:
                    m.ctx_start = dv["cst"][s0:s1]
                    m.block_tables = dv["bt"].view(S_, W)[s0:s1]
                parts.append(m)
            meta.micro = (parts[0], parts[1], TA)
            self.n_steps["overlapped"] = self.n_steps.get("overlapped", 0) + 1
        if nd:
            meta.num_decode = nd
            meta.dec_block_tables = dv["dbt"].view(nd, Wd)
            meta.dec_seq_lens = dv["dlen"]
            meta.decode_ws = self.decode_ws
            self.n_steps["mixed"] = self.n_steps.get("mixed", 0) + 1
        # tokens attended from the paged cache instead of recomputed (prefix hits + earlier chunks)
        self.n_steps["prefill_context_tokens"] = self.n_steps.get("prefill_context_tokens", 0) + sum(starts)
        self.n_steps["prefill_tokens"] = self.n_steps.get("prefill_tokens", 0) + T
        logits = self.model.forward(dv["ids"], meta, self.kv)
        tok = self._sample(logits, dv["temp"].view(torch.float32), dv["topk"], dv["topp"].view(torch.float32))
        self.n_steps["prefill"] += 1
        if self.on_launched is not None:  # TP: the custom-AR error flag, read back with the tokens
            self.on_launched()
        if not self.is_gpu:
            return DecodeHandle(R, None, tok[:R].tolist())
        j = self._pf_oi
        self._pf_oi ^= 1  # two in flight at most: step N+1 is launched before step N is read back
        if self._pf_out[j] is None or self._pf_out[j].numel() < R:
            self._pf_out[j] = torch.empty(max(R, 2 * self.B), dtype=torch.int32, pin_memory=True)
        out = self._pf_out[j]
        out[:R].copy_(tok[:R], non_blocking=True)
        ev, _ = self._chain_event()
        return DecodeHandle(R, ev, out)

    # --------------------------------------------------------------------- decode
    def _decode_body(self, b: int) -> None:
        # pipelined decode: a row whose input is the token sampled by the previous step (still in
        # flight when this step was enqueued) takes it from d_out on the device (d_src = its row
        # there); other rows take the host-provided id - resolved by the model's first kernel
        meta = AttnMeta(is_prefill=False, positions=self.d_pos[:b], slot_mapping=self.d_slots[:b],
                        block_tables=self.d_bt[:b], seq_lens=self.d_lens[:b], decode_ws=self.decode_ws,
                        dec_src=self.d_src[:b], dec_prev=self.d_out)
        logits = self.model.forward(self.d_ids[:b], meta, self.kv)
        self._sample(logits, self.d_temp[:b], self.d_topk[:b], self.d_topp[:b], out=self.d_out[:b])

    def capture_graphs(self, buckets: Optional[list[int]] = None) -> None:
        if not (self.is_gpu and self.cfg.use_graphs):
            return
        torch.cuda.synchronize()
        # replays must not disturb real sequences: capture with empty rows (len 0, no cache write)
        self.d_lens.zero_()
        self.d_slots.fill_(-1)
        rng_state = self.rng.clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                self._decode_body(self.B)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.graph_pool = torch.cuda.graph_pool_handle()
        for b in sorted(buckets or self.buckets, reverse=True):
            n_el = _Staging.prefix(self.B, self.max_blocks_per_seq, b)
            gs = []
            for st in (self.stage if self.graph_h2d else [None]):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=self.graph_pool):
                    if st is not None:
                        self.d_all[:n_el].copy_(st.h_all[:n_el], non_blocking=True)
                    self._decode_body(b)
                gs.append(g)
            self.graphs[b] = gs
        torch.cuda.synchronize()
        self.rng.copy_(rng_state)

    def decode(self, seqs: list, src_rows: Optional[list] = None, publish=None) -> list[int]:
        """One decode step, synchronous: the sampled token per sequence."""
        return self.decode_collect(self.decode_launch(seqs, src_rows, publish))

    def decode_launch(self, seqs: list, src_rows: Optional[list] = None, publish=None) -> "DecodeHandle":
        """Enqueue one decode step without waiting for it.  ``src_rows[i] >= 0``: sequence i's input
        token is the one the previous (possibly still running) step sampled in that row; else its
        ``last_token``.  Positions come from ``num_tokens``, so a sequence carrying a not yet
        resolved token from the in-flight step is already one position further.  ``publish``
        (TP leader): called with the raw step message (parallel/step_bus.py) after staging and
        before the launch, so the workers replay the same step."""
        n = len(seqs)
        b = self.bucket_for(n) if self.graphs else n
        st = self.stage[self._stage_i]
        self._stage_i ^= 1
        ids, pos_a, slots, lens, src = st.n_ids, st.n_pos, st.n_slots, st.n_lens, st.n_src
        temp, topk, topp, bt_a = st.n_temp, st.n_topk, st.n_topp, st.n_bt
        bt_a[:b] = 0
        for i, s in enumerate(seqs):
            pos = s.num_tokens - 1  # position of the token being fed (the last generated one)
            bt = s.block_table
            r = src_rows[i] if src_rows is not None else -1
            src[i] = r
            ids[i] = s.last_token if r < 0 else 0
            pos_a[i] = pos
            slots[i] = bt[pos // BLOCK_SIZE] * BLOCK_SIZE + pos % BLOCK_SIZE
            lens[i] = pos + 1
            bt_a[i, : len(bt)] = bt
            p = s.params
            temp[i] = p.temperature
            topk[i] = p.top_k
            topp[i] = p.top_p
        if b > n:
            ids[n:b] = 0
            src[n:b] = -1
            pos_a[n:b] = 0
            slots[n:b] = -1
            lens[n:b] = 0
            temp[n:b] = 0
            topk[n:b] = 0
            topp[n:b] = 1
        n_el = _Staging.prefix(self.B, self.max_blocks_per_seq, b)  # the per-row fields + b block-table rows
        if publish is not None:
            publish(st.message(n, b, n_el))
        return self._launch_staged(st, n, b, n_el)

    def decode_launch_raw(self, n: int, b: int, n_el: int, words: np.ndarray) -> "DecodeHandle":
        """TP worker: launch the decode step the leader staged (its raw staging words)."""
        st = self.stage[self._stage_i]
        self._stage_i ^= 1
        st.raw[:n_el] = words
        return self._launch_staged(st, n, b, n_el)

    def _launch_staged(self, st: "_Staging", n: int, b: int, n_el: int) -> "DecodeHandle":
        gs = self.graphs.get(b)
        if gs is not None and self.graph_h2d:
            gs[st.idx].replay()  # its first node copies this staging buffer (n_el = the bucket's prefix)
        else:
            self.d_all[:n_el].copy_(st.h_all[:n_el], non_blocking=True)
            if gs is not None:
                gs[0].replay()
            else:
                self._decode_body(b)
        self.n_steps["decode"] += 1
        if self.on_launched is not None:
            self.on_launched()
        if not self.is_gpu:
            return DecodeHandle(n, None, self.d_out[:n].tolist())
        h = self.h_out[self._out_i]
        self._out_i ^= 1
        h[:n].copy_(self.d_out[:n], non_blocking=True)
        ev, prev = self._chain_event()
        return DecodeHandle(n, ev, h, prev)

    def _chain_event(self) -> tuple:
        """Record the end-of-step event (timing-enabled) and return it with the previous launched
        step's event IF that step was still running when this one was enqueued: the GPU then went
        from one step straight into the next, so the elapsed time between the two events is this
        step's GPU time (no host stall inside it) - the decode step-time samples of the admission
        model (EngineService.tpot).  Otherwise the previous event is dropped (None)."""
        prev = self._last_ev
        busy = prev is not None and not prev.query()
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self._last_ev = ev
        return ev, (prev if busy else None)

    @staticmethod
    def decode_collect(handle: "DecodeHandle") -> list[int]:
        if handle.event is None:
            return handle.out
        handle.event.synchronize()
        return handle.out[: handle.n].tolist()

    def memory_report(self) -> dict:
        kv = (self.k_cache.numel() + self.v_cache.numel()) * self.k_cache.element_size()
        return {"kv_cache_bytes": kv, "kv_blocks": self.num_blocks, "block_size": BLOCK_SIZE,
                "max_model_len": self.max_len, "graph_buckets": sorted(self.graphs)}


class _Staging:
    """Pinned host buffer for one decode step's inputs, with numpy views for cheap writes.

    One int32 buffer holds every field - ids, src, pos, slots, lens, top_k, temperature and top_p
    ([B] each; the two float fields bit-cast) followed by the block tables [B, max_blocks] - so the
    step's inputs reach the device in ONE copy of the per-row fields plus the live block-table rows
    (nine separate small copies were nine blit kernels of ~4.6 us each in front of every decode
    graph replay)."""

    NFIELDS = 8

    @staticmethod
    def size(B: int, max_blocks: int) -> int:
        return _Staging.NFIELDS * B + B * max_blocks

    @staticmethod
    def prefix(B: int, max_blocks: int, b: int) -> int:
        return _Staging.NFIELDS * B + b * max_blocks

    @staticmethod
    def views(buf, B: int, max_blocks: int) -> tuple:
        """(ids, src, pos, slots, lens, topk, temp, topp, bt) views of a buffer (torch or numpy)."""
        f = [buf[i * B:(i + 1) * B] for i in range(_Staging.NFIELDS)]
        as_f32 = (lambda a: a.view(torch.float32)) if isinstance(buf, torch.Tensor) else (lambda a: a.view(np.float32))
        f[6], f[7] = as_f32(f[6]), as_f32(f[7])
        bt = buf[_Staging.NFIELDS * B:_Staging.size(B, max_blocks)]
        bt = bt.view(B, max_blocks) if isinstance(buf, torch.Tensor) else bt.reshape(B, max_blocks)
        return (*f, bt)

    def __init__(self, B: int, max_blocks: int, pin: bool, idx: int = 0):
        from ..parallel.step_bus import DECODE_HDR, KIND_DECODE

        self.idx = idx
        # DECODE_HDR leading words hold the step-bus header, so a TP leader publishes
        # full[:DECODE_HDR + n_el] without a copy (parallel/step_bus.py)
        self.h_full = torch.zeros(DECODE_HDR + self.size(B, max_blocks), dtype=torch.int32, pin_memory=pin)
        self.h_all = self.h_full[DECODE_HDR:]
        self.full = self.h_full.numpy()
        self.full[0] = KIND_DECODE
        self.raw = self.full[DECODE_HDR:]
        (self.n_ids, self.n_src, self.n_pos, self.n_slots, self.n_lens, self.n_topk, self.n_temp, self.n_topp,
         self.n_bt) = self.views(self.raw, B, max_blocks)

    def message(self, n: int, b: int, n_el: int) -> np.ndarray:
        from ..parallel.step_bus import DECODE_HDR

        self.full[1:4] = (n, b, n_el)
        return self.full[:DECODE_HDR + n_el]


@dataclass
class DecodeHandle:
    n: int
    event: object  # torch.cuda.Event, None on the CPU
    out: object  # pinned host tensor (GPU) or the token list (CPU)
    prev_event: object = None  # the back-to-back predecessor's end event (ModelRunner._chain_event)

    def gpu_ms(self) -> Optional[float]:
        """This step's GPU time (after the event completed), or None when not measurable."""
        if self.prev_event is None or self.event is None:
            return None
        return float(self.prev_event.elapsed_time(self.event))


def kv_blocks_for(cfg_layers: int, hkv: int, D: int, gb: float) -> int:
    per_block = 2 * cfg_layers * hkv * D * BLOCK_SIZE * 2
    return int(math.floor(gb * (1 << 30) / per_block))
