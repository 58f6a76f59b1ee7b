"""ASan + UBSan build and threaded stress run of the native serving runtime (SURVEY.md §5 race
detection / sanitizers; VERDICT r1 missing #8).

Builds ``runtime/csrc/*.cpp`` (BlockPool prefix cache, BPE encoder, decode-batch packing, the
shared-memory StepChannel) with ``-fsanitize=address,undefined -fno-omit-frame-pointer`` into
``build/sanitize/`` - never over the production module - and runs :func:`stress` against it in a
child interpreter with the ASan runtime preloaded (CPython itself is not instrumented).  The stress
hammers every entry point from several threads (the BPE encoder releases the GIL; StepChannel
readers spin without it) and checks invariants, so any heap overflow, use-after-free, UB (shift /
overflow / misaligned access) or torn message aborts the child with a sanitizer report.

    python tools/sanitize_runtime.py            # build + run, exit code 0 = clean
"""
from __future__ import annotations

import importlib.util
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
SRC = ROOT / "k8s_llm_monitor_amd" / "runtime" / "csrc"
OUT = ROOT / "build" / "sanitize"
SO = OUT / ("_k8sllm_runtime" + sysconfig.get_config_var("EXT_SUFFIX"))
FLAGS = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"]


def build() -> Path:
    import pybind11

    OUT.mkdir(parents=True, exist_ok=True)
    srcs = sorted(SRC.glob("*.cpp"))
    cmd = ["g++", "-std=c++17", "-shared", "-fPIC", *FLAGS, f"-I{pybind11.get_include()}",
           f"-I{sysconfig.get_paths()['include']}", f"-I{SRC}", *map(str, srcs), "-o", str(SO), "-lrt"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("sanitizer build failed:\n" + r.stderr[-4000:])
    return SO


def _load(path: str):
    spec = importlib.util.spec_from_file_location("_k8sllm_runtime", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def stress(path: str) -> None:
    import random
    import threading

    rt = _load(path)
    rng = random.Random(0)

    # BlockPool: random allocate / match / publish / release against a shadow refcount model
    pool = rt.BlockPool(64)
    held: list = []
    for it in range(20000):
        op = rng.random()
        if op < 0.4:
            toks = [rng.randrange(50) for _ in range(rng.randrange(0, 80))]
            hs = rt.block_hashes(toks, 16, 0)
            assert pool.peek_idle(hs) <= pool.peek(hs) <= len(hs)
            got = pool.match(hs)
            need = rng.randrange(0, 4)
            fresh = pool.allocate(need)
            if fresh is None:
                pool.release(got)
                continue
            blocks = list(got) + list(fresh)
            for i, b in enumerate(fresh):
                if len(got) + i < len(hs):
                    pool.publish(b, hs[len(got) + i])
            held.append(blocks)
        elif held:
            pool.release(held.pop(rng.randrange(len(held))))
        assert 0 <= pool.num_free <= 64
    for b in held:
        pool.release(b)
    assert pool.num_free == 64
    try:
        pool.release([0])
        raise AssertionError("double free not detected")
    except RuntimeError:
        pass

    # BPE: concurrent encodes (GIL released inside) over a shared word cache
    left = list(range(256, 300))
    right = list(range(300, 344))
    bpe = rt.BPE([97 + (i % 26) for i in range(len(left))], [98 + (i % 25) for i in range(len(right))])
    texts = ["集群状态概览: node-%03d CPU=%.1f%% [资源压力] 'll 've  \n\t" % (i, i * 1.7) * 5 for i in range(64)]
    errs: list = []

    def enc(k):
        try:
            for _ in range(200):
                for t in texts[k::4]:
                    bpe.encode(t)
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=enc, args=(k,)) for k in range(4)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errs, errs

    # pack_decode over random batches
    import numpy as np

    for _ in range(500):
        n = rng.randrange(1, 9)
        W = 8
        tables = [[rng.randrange(100) for _ in range(rng.randrange(1, W + 1))] for _ in range(n)]
        num = [rng.randrange(1, 16 * len(t) + 1) for t in tables]
        ids = np.zeros(n + 3, np.int32)
        pos = np.zeros(n + 3, np.int32)
        slots = np.zeros(n + 3, np.int32)
        lens = np.zeros(n + 3, np.int32)
        bt = np.zeros((n + 3, W), np.int32)
        rt.pack_decode(ids, pos, slots, lens, bt, [1] * n, num, tables, n + 3, 16)
        assert (lens[:n] == np.asarray(num)).all() and (slots[n:] == -1).all()

    # StepChannel: 1 writer, 3 reader threads, variable-size messages through a 2-slot ring
    name = f"/k8sllm_asan_{os.getpid()}"
    w = rt.StepChannel(name, True, 2, 1 << 14, 3)
    readers = [rt.StepChannel(name, False) for _ in range(3)]
    w.unlink()
    got = [[] for _ in range(3)]

    def rd(i):
        while True:
            m = readers[i].recv(i, 10.0)
            assert m is not None, "reader timed out"
            if m == b"stop":
                return
            got[i].append(m)

    ts = [threading.Thread(target=rd, args=(i,)) for i in range(3)]
    [t.start() for t in ts]
    sent = []
    for k in range(3000):
        m = bytes([k % 251]) * rng.randrange(1, 1 << 14)
        assert w.publish(m, 10.0)
        sent.append(m)
    w.publish(b"stop", 10.0)
    [t.join() for t in ts]
    assert all(g == sent for g in got)
    for r in readers:
        r.close()
    w.close()
    print("sanitized runtime stress: clean")


def run() -> int:
    path = build()
    env = dict(os.environ)
    def lib(name: str) -> str:
        return subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()

    # libstdc++ right after the ASan runtime: CPython does not link it, and ASan's __cxa_throw
    # interceptor must find the real one at start-up (C++ exceptions cross the binding)
    env["LD_PRELOAD"] = f"{lib('libasan.so')} {lib('libstdc++.so')}"
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=1"  # CPython's arenas are not leak-clean
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    r = subprocess.run([sys.executable, __file__, "--child", str(path)], env=env, capture_output=True, text=True,
                       timeout=600)
    sys.stdout.write(r.stdout)
    sys.stderr.write(r.stderr[-8000:])
    return r.returncode


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        stress(sys.argv[2])
    else:
        sys.exit(run())
