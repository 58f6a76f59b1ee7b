"""Per-step TP control overhead: one-way latency of a decode step message from the TP leader to a
worker process (parallel/step_bus.py), shared-memory ring vs gloo broadcast_object_list.

The message is the real decode payload: the pinned staging words of a B-row step (ids, src,
positions, slots, lengths, sampling parameters) plus B block-table rows of max_blocks entries.
The leader stamps time.perf_counter() (CLOCK_MONOTONIC, common to both processes) into the
message; the worker records arrival - stamp after decoding the message into numpy views, which is
what the engine's worker does before its launch.  The leader paces messages 2 ms apart (a decode
step's cadence is ~3-7 ms) so the figure is latency, not queueing.

    python tools/bench_step_bus.py [--batch 64] [--max-blocks 512] [--steps 2000]
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _rank(rank: int, port: int, kind: str, B: int, mb: int, steps: int, q) -> None:
    import torch.distributed as dist

    from k8s_llm_monitor_amd.parallel.state import ParallelState
    from k8s_llm_monitor_amd.parallel.step_bus import (DECODE_HDR, KIND_DECODE, GlooStepBus, ShmStepBus,
                                                      decode_message)

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    ps = ParallelState(world_size=2, rank=rank, tp_size=2, tp_rank=rank, cpu_group=dist.group.WORLD)
    n_el = 8 * B + B * mb
    bus = ShmStepBus(ps, 4 * (DECODE_HDR + n_el) + 4096) if kind == "shm" else GlooStepBus(ps)
    if rank == 0:
        words = np.zeros(DECODE_HDR + n_el, dtype=np.int32)
        words[0], words[1], words[2], words[3] = KIND_DECODE, B, B, n_el
        stamp = words[DECODE_HDR:DECODE_HDR + 2].view(np.float64)
        for _ in range(steps):
            stamp[0] = time.perf_counter()
            bus.send_raw(words)
            time.sleep(0.002)
        bus.send_stop()
    else:
        lat = []
        while True:
            k, payload = decode_message(bus.recv())
            if k != KIND_DECODE:
                break
            t = payload[3][:2].view(np.float64)[0]
            lat.append((time.perf_counter() - t) * 1e6)
        lat = sorted(lat[10:])
        q.put({"bus": kind, "batch": B, "max_blocks": mb, "bytes": 4 * (DECODE_HDR + n_el), "steps": len(lat),
               "one_way_us_p50": round(lat[len(lat) // 2], 1), "one_way_us_p99": round(lat[int(len(lat) * 0.99)], 1)})
    bus.close()
    dist.destroy_process_group()


def main() -> None:
    import multiprocessing as mp

    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--max-blocks", type=int, default=512)
    ap.add_argument("--steps", type=int, default=2000)
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    for kind in ("shm", "gloo"):
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        q = ctx.Queue()
        ps = [ctx.Process(target=_rank, args=(r, port, kind, a.batch, a.max_blocks, a.steps, q)) for r in range(2)]
        for p in ps:
            p.start()
        print(json.dumps(q.get(timeout=600)), flush=True)
        for p in ps:
            p.join(60)


if __name__ == "__main__":
    main()
