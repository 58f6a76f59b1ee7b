#!/usr/bin/env python
"""Which PyTorch (non-k8sllm) kernels run inside the headline's engine steps, and from which aten
op: torch.profiler over one wave of the headline workload (64 ~1.6k-token prompts, 16 decode
steps), listing every aten op whose device kernels are not ours, with total device time.

    python tools/torch_ops_in_step.py [--rows 64 --tokens 16]"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--rows", type=int, default=64)
    ap.add_argument("--tokens", type=int, default=16)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    from torch.profiler import ProfilerActivity, profile

    from k8s_llm_monitor_amd.engine import EngineConfig, LLMEngine, SamplingParams
    from k8s_llm_monitor_amd.llm.synthetic import synthetic_cluster_prompt

    eng = LLMEngine(EngineConfig(model=a.model, max_num_seqs=a.rows, max_model_len=8192, kv_cache_gb=48.0, seed=1),
                    device="cuda")
    eng.warmup()
    prompts = [synthetic_cluster_prompt(s) for s in range(a.rows)]
    sp = SamplingParams(max_tokens=a.tokens, temperature=0.1, ignore_eos=True)
    eng.generate(prompts[:8], sp)  # first-use paths outside the profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        eng.generate(prompts, sp)
        torch.cuda.synchronize()
    rows = []
    for ev in prof.key_averages():
        dev_us = getattr(ev, "device_time_total", None)
        if dev_us is None:
            dev_us = getattr(ev, "cuda_time_total", 0)
        if dev_us <= 0 or not ev.key.startswith("aten::"):
            continue
        rows.append((dev_us, ev.key, ev.count))
    rows.sort(reverse=True)
    kern = []
    for ev in prof.key_averages():
        dev_us = getattr(ev, "self_device_time_total", None)
        if dev_us is None:
            dev_us = getattr(ev, "self_cuda_time_total", 0)
        if dev_us > 0 and not ev.key.startswith("aten::") and "k8sllm" not in ev.key:
            kern.append((dev_us, ev.key[:110], ev.count))
    kern.sort(reverse=True)
    for us, k, n in rows[: a.top]:
        print(json.dumps({"aten_op": k, "calls": n, "device_us_total": round(us, 1)}))
    for us, k, n in kern[: a.top]:
        print(json.dumps({"non_k8sllm_kernel": k, "calls": n, "device_us_total": round(us, 1)}))


if __name__ == "__main__":
    main()
