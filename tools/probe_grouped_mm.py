"""Probe torch._grouped_mm on this ROCm build (MI355X): correctness against per-group matmuls,
whether it synchronises with the host (torch.cuda.set_sync_debug_mode), and its speed on a
Mixtral-shaped MoE prefill (T tokens x top-2 over 8 experts, d 4096, F 14336)."""
import json
import sys
import time

import torch


def main() -> None:
    dev = "cuda"
    E, d, F = 8, 4096, 14336
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    rows = T * 2
    torch.manual_seed(0)
    counts = torch.multinomial(torch.ones(E), rows, replacement=True).bincount(minlength=E)
    offs = counts.cumsum(0).to(torch.int32).to(dev)
    x = torch.randn(rows, d, device=dev, dtype=torch.bfloat16)
    w = torch.randn(E, 2 * F, d, device=dev, dtype=torch.bfloat16) * 0.02  # [E, N, K]
    res = {"T": T, "counts": counts.tolist()}
    try:
        y = torch._grouped_mm(x, w.transpose(1, 2), offs=offs)  # [rows, N]
        torch.cuda.synchronize()
        ref = []
        o = 0
        for e in range(E):
            n = int(counts[e])
            ref.append(x[o:o + n] @ w[e].t())
            o += n
        ref = torch.cat(ref)
        res["max_err"] = float((y.float() - ref.float()).abs().max())
        res["ok"] = True
    except Exception as ex:  # noqa: BLE001
        res["ok"] = False
        res["error"] = repr(ex)[:300]
        print(json.dumps(res))
        return
    try:
        torch.cuda.set_sync_debug_mode("error")
        torch._grouped_mm(x, w.transpose(1, 2), offs=offs)
        torch.cuda.set_sync_debug_mode(0)
        res["host_sync"] = False
    except Exception as ex:  # noqa: BLE001
        torch.cuda.set_sync_debug_mode(0)
        res["host_sync"] = True
        res["sync_error"] = repr(ex)[:200]
    flops = 2 * rows * d * 2 * F
    for name, fn in (("grouped_mm", lambda: torch._grouped_mm(x, w.transpose(1, 2), offs=offs)),
                     ("loop_mm", lambda: [x[a:b] @ w[e].t() for e, (a, b) in enumerate(
                         zip([0] + counts.cumsum(0).tolist()[:-1], counts.cumsum(0).tolist()))])):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 10
        res[name + "_ms"] = round(dt * 1e3, 3)
        res[name + "_PFps"] = round(flops / dt / 1e15, 3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
