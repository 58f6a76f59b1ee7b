"""Step bus: how the tensor-parallel leader hands each engine step to its TP workers (SURVEY.md
§2.12 C-6).

The leader owns the scheduler; every TP rank runs the identical forward.  Per step the workers need
the step's inputs:

* decode  - the leader's pinned staging buffer (ids, src rows, positions, slots, lengths, sampling
            parameters, block-table rows: ``engine/runner._Staging``) sent RAW - no pickling, and
            the worker copies it straight into its own staging and replays the same hipGraph;
* prefill / mixed / stop - a pickled plan (prefill steps are tens to hundreds of ms; pickling is
            noise there).

Transport: ``ShmStepBus`` - the native shared-memory ring (``runtime/csrc/step_channel.cpp``,
all TP ranks of a group live on one node) - by default; ``GlooStepBus`` - ``broadcast_object_list``
over the CPU gloo group - when the native runtime is missing or ``K8SLLM_STEP_BUS=gloo``.
Message framing: int32 kind, then the payload (decode: int32 [n, b, n_el] + n_el staging words).
"""
from __future__ import annotations

import os
import pickle
import struct
import uuid

import numpy as np
import torch.distributed as dist

KIND_DECODE = 1
KIND_PICKLE = 2
KIND_STOP = 3

DECODE_HDR = 4  # int32 words in front of a raw decode message: kind, n, b, n_el


class GlooStepBus:
    """``broadcast_object_list`` over the TP group's step-bus gloo group (``ps.bus_group``).  That
    group has no serving timeout: a worker sits in the broadcast for as long as the server is idle,
    so a bounded group would kill every worker after an idle gap (the TP collective groups get the
    short serving bound, parallel/state.py).  A dead leader still surfaces: gloo raises as soon as
    the leader's socket closes."""

    def __init__(self, ps):
        self.ps = ps
        self.src = ps.rank - ps.tp_rank
        self.group = getattr(ps, "bus_group", None) or ps.cpu_group

    def _bcast(self, obj):
        lst = [obj]
        dist.broadcast_object_list(lst, src=self.src, group=self.group)
        return lst[0]

    def send_raw(self, words: np.ndarray) -> None:
        self._bcast(words.tobytes())

    def send_obj(self, obj) -> None:
        self._bcast(struct.pack("<i", KIND_PICKLE) + pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL))

    def send_stop(self) -> None:
        self._bcast(struct.pack("<i", KIND_STOP))

    def recv(self) -> bytes:
        return self._bcast(None)

    def set_leader(self, ident: tuple) -> None:
        self.leader_ident = ident  # gloo's own broadcast fails when the leader's socket closes

    def close(self) -> None:
        pass


class ShmStepBus:
    """Leader publishes into a native shared-memory ring; worker ``tp_rank - 1`` is reader index
    ``tp_rank - 1``.  Collective over the TP group's CPU group (name exchange + barrier)."""

    def __init__(self, ps, slot_bytes: int, nslots: int = 4, timeout_s: float = 60.0, poll_s: float = 1.0,
                 beat_s: float = 1.0, silent_s: float = 30.0):
        """``timeout_s`` bounds the LEADER's publish back-pressure (a worker that stopped consuming).
        A worker waits for the next step without a deadline - an idle server publishes nothing for
        as long as no request arrives - and polls the leader's liveness every ``poll_s`` instead,
        so a dead leader still surfaces (ConnectionError) rather than hanging the worker: through
        /proc when the worker can see the leader's process, else through the ring's heartbeat word,
        which a leader thread bumps every ``beat_s`` (a leader silent for ``silent_s`` is gone)."""
        from ..runtime import native_runtime

        rt = native_runtime()
        if rt is None or not hasattr(rt, "StepChannel"):
            raise RuntimeError("native StepChannel unavailable")
        self.ps = ps
        self.timeout_s = timeout_s
        self.silent_s = silent_s  # worker's bound on a still heartbeat when it cannot observe the leader
        self.poll_s = poll_s
        self._beat_stop = None
        src = ps.rank - ps.tp_rank
        name = [f"/k8sllm_step_{os.getpid()}_{uuid.uuid4().hex[:12]}" if ps.tp_rank == 0 else None]
        ok = [True]
        if ps.tp_rank == 0:
            try:
                self.ch = rt.StepChannel(name[0], True, nslots, int(slot_bytes), ps.tp_size - 1)
            except Exception:  # noqa: BLE001 - no /dev/shm: tell the workers to fall back
                ok[0] = False
        dist.broadcast_object_list(name, src=src, group=ps.cpu_group)
        if ps.tp_rank != 0 and ok[0]:
            try:
                self.ch = rt.StepChannel(name[0], False)
            except Exception:  # noqa: BLE001
                ok[0] = False
        oks: list = [None] * ps.tp_size  # every rank learns whether every rank has the channel
        dist.all_gather_object(oks, ok[0], group=ps.cpu_group)
        self.leader_pid = int(name[0].split("_")[2])  # TP ranks share a node (shared memory)
        if ps.tp_rank == 0 and ok[0]:
            self.ch.unlink()  # every rank that could map it has: the name is no longer needed
        if not all(oks):
            if ok[0]:
                self.ch.close()
            raise RuntimeError("shared-memory step channel unavailable on some TP rank")
        self.reader = ps.tp_rank - 1
        if ps.tp_rank == 0:
            import threading

            self._beat_stop = threading.Event()
            self._beat = threading.Thread(target=self._beat_loop, args=(beat_s,), name="step-bus-heartbeat",
                                          daemon=True)
            self._beat.start()

    def _beat_loop(self, beat_s: float) -> None:
        while not self._beat_stop.wait(beat_s):
            self.ch.heartbeat()

    def _publish(self, data) -> None:
        if not self.ch.publish(data, self.timeout_s):
            raise TimeoutError("TP worker did not consume the previous step within the step-bus timeout")

    def send_raw(self, words: np.ndarray) -> None:
        self._publish(words)

    def send_obj(self, obj) -> None:
        self._publish(struct.pack("<i", KIND_PICKLE) + pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL))

    def send_stop(self) -> None:
        self._publish(struct.pack("<i", KIND_STOP))

    def set_leader(self, ident: tuple) -> None:
        """The leader's (pid, start time, host) from the engine's identity exchange: the /proc
        liveness poll below is used only if this worker can see that process (same host and pid
        namespace, matching start time); otherwise the ring's heartbeat word tells whether the
        leader still runs (``silent_s``)."""
        from .health import visible

        self.leader_ident = ident
        self.leader_visible = visible(ident)

    def recv(self) -> bytes:
        from .health import alive

        import time

        beat, t_beat = self.ch.beats, time.monotonic()
        while True:
            m = self.ch.recv(self.reader, self.poll_s)
            if m is not None:
                return m
            ident = getattr(self, "leader_ident", None)
            if ident is None:
                if not _pid_alive(self.leader_pid):
                    raise ConnectionError(f"TP leader (pid {self.leader_pid}) exited without sending STOP")
            elif self.leader_visible:
                if alive(ident) is False:
                    raise ConnectionError(f"TP leader (pid {ident[0]}) exited without sending STOP")
            else:
                b, now = self.ch.beats, time.monotonic()
                if b != beat:
                    beat, t_beat = b, now
                elif now - t_beat > self.silent_s:
                    raise ConnectionError(f"TP leader heartbeat silent for {self.silent_s:.0f} s "
                                          "(leader process not observable from this worker)")

    def close(self) -> None:
        if self._beat_stop is not None:  # the thread must be gone before the ring is unmapped
            self._beat_stop.set()
            self._beat.join()
        self.ch.close()


def _pid_alive(pid: int) -> bool:
    """False once ``pid`` has exited - including an exited but not yet reaped (zombie) process,
    which signal 0 would still report as present."""
    try:
        with open(f"/proc/{pid}/stat", "rb") as f:
            return f.read().rsplit(b")", 1)[1].split()[0] not in (b"Z", b"X")
    except FileNotFoundError:
        return False
    except OSError:  # no procfs: fall back to signal 0
        pass
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:  # exists, owned by someone else
        return True
    return True


def make_step_bus(ps, slot_bytes: int):
    """Collective over the TP group.  None at TP 1."""
    if ps.tp_size == 1:
        return None
    if os.environ.get("K8SLLM_STEP_BUS", "shm") != "gloo":
        try:
            return ShmStepBus(ps, slot_bytes)
        except Exception:  # noqa: BLE001 - every rank takes the same branch (the failure is broadcast)
            pass
    return GlooStepBus(ps)


def decode_message(buf: bytes) -> tuple:
    """(kind, payload): KIND_DECODE -> (n, b, n_el, int32 staging words); KIND_PICKLE -> object."""
    kind = struct.unpack_from("<i", buf, 0)[0]
    if kind == KIND_DECODE:
        w = np.frombuffer(buf, dtype=np.int32)
        n, b, n_el = int(w[1]), int(w[2]), int(w[3])
        return kind, (n, b, n_el, w[DECODE_HDR:DECODE_HDR + n_el])
    if kind == KIND_PICKLE:
        return kind, pickle.loads(buf[4:])
    return kind, None


def bus_slot_bytes(max_num_seqs: int, max_model_len: int, max_blocks: int) -> int:
    """Enough for the largest message: a raw decode step or a pickled prefill plan (chunk ids +
    block tables of every sequence)."""
    raw = 4 * (DECODE_HDR + 8 * max_num_seqs + max_num_seqs * max_blocks)
    pickled = max_num_seqs * (max_model_len * 6 + max_blocks * 6 + 256) + (1 << 16)
    return int(max(1 << 20, raw, pickled))

