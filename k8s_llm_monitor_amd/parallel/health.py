"""TP group failure detection (SURVEY.md §5 "Detect RCCL timeouts via NCCL_TIMEOUT-style watchdog";
the probe contract it serves: liveness / readiness on ``/health``,
``/root/reference/deployments/monitor-server.yaml:145-156``, and the 15 s write timeout,
``/root/reference/cmd/server/main.go:147-148``).

A tensor-parallel step is a chain of collectives: when one rank dies, the others block inside the
next all-reduce (RCCL waits on the GPU; only the process-group timeout would end it).  Three layers
turn that into a fast, visible failure instead of a silent hang:

* process identity - at engine setup every TP rank's (pid, process start time) is gathered over the
  CPU group (:func:`gather_identities`); the start time guards against pid reuse, and a rank whose
  peer is not visible in its /proc (separate pid namespaces) knows it cannot use the check;
* :class:`PeerMonitor` - a leader-side daemon thread that polls its workers' /proc entries and
  reports the first one that is gone (dead, zombie, or replaced);
* the engine service's step watchdog (``engine.EngineService``) - a step in flight longer than its
  bound marks the service unhealthy even when every process is alive (a wedged collective).

Either detector marks the service unhealthy: ``/health`` answers 503 (the liveness probe restarts
the pod) and every request in flight or queued fails at once with EngineUnavailable (HTTP 503)
instead of hanging until the process-group timeout.
"""
from __future__ import annotations

import os
import threading
from typing import Callable, Optional


def proc_start_time(pid: int) -> Optional[int]:
    """Field 22 of /proc/<pid>/stat (start time in clock ticks since boot), None when the process
    is not visible here or has exited (zombie / dead)."""
    try:
        with open(f"/proc/{pid}/stat", "rb") as f:
            rest = f.read().rsplit(b")", 1)[1].split()
    except (FileNotFoundError, ProcessLookupError, OSError):
        return None
    if rest[0] in (b"Z", b"X"):
        return None
    return int(rest[19])


def identity() -> tuple:
    """(pid, start time, host) of this process."""
    pid = os.getpid()
    return pid, proc_start_time(pid), os.uname().nodename


def gather_identities(ps) -> list:
    """Collective over the TP group's CPU group: every rank's :func:`identity`, by TP rank."""
    import torch.distributed as dist

    out: list = [None] * ps.tp_size
    dist.all_gather_object(out, identity(), group=ps.cpu_group)
    return out


def alive(ident: tuple) -> Optional[bool]:
    """True / False for a peer identity; None when this process cannot tell (another host, or
    another pid namespace: the peer's pid is not visible with its start time)."""
    pid, start, host = ident
    if host != os.uname().nodename or start is None:
        return None
    now = proc_start_time(pid)
    if now is None:
        return False if os.path.isdir("/proc/self") else None
    return now == start


def visible(ident: tuple) -> bool:
    return alive(ident) is True


class PeerMonitor:
    """Polls the identities of ``peers`` ({tp_rank: identity}) every ``poll_s`` on a daemon thread
    and calls ``on_dead(rank, identity)`` once, for the first peer found gone.  Peers this process
    cannot observe (:func:`alive` is None at start) are skipped - the step watchdog still covers
    them."""

    def __init__(self, peers: dict, on_dead: Callable[[int, tuple], None], poll_s: float = 0.5):
        self.peers = {r: ident for r, ident in peers.items() if alive(ident) is True}
        self.unobservable = sorted(set(peers) - set(self.peers))
        self.on_dead = on_dead
        self.poll_s = poll_s
        self.dead: Optional[tuple] = None
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._loop, name="tp-peer-monitor", daemon=True)
        if self.peers:
            self._thread.start()

    def _loop(self) -> None:
        while not self._stop.wait(self.poll_s):
            for r, ident in self.peers.items():
                if alive(ident) is False:
                    self.dead = (r, ident)
                    try:
                        self.on_dead(r, ident)
                    finally:
                        return

    def check(self) -> Optional[tuple]:
        """Synchronous poll (tests / callers without the thread): the first dead peer or None."""
        for r, ident in self.peers.items():
            if alive(ident) is False:
                return r, ident
        return None

    def stop(self) -> None:
        self._stop.set()
