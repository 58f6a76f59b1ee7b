"""The batched CPU serving attention (ops/cpu_attn.py, config 1) against the fp32 oracle of
ops/reference.py: ragged lengths, an empty sequence, GQA, unused block-table entries (-1), a cached
prefix (paged prefill) - and the runner's auto-sized KV pool (kv_cache_gb <= 0)."""
import pytest
import torch

from k8s_llm_monitor_amd.ops import cpu_attn
from k8s_llm_monitor_amd.ops import reference as ref


def _cache(dt, Hkv=2, D=64, bs=16, nblocks=64, seed=0):
    g = torch.Generator().manual_seed(seed)
    kc = torch.randn(nblocks, Hkv, D // 8, bs, 8, generator=g).to(dt)
    vc = torch.randn(nblocks, Hkv, D, bs, generator=g).to(dt)
    return kc, vc


@pytest.mark.parametrize("dt,tol", [(torch.float32, 1e-5), (torch.bfloat16, 2e-2)])
@pytest.mark.parametrize("Hq,Hkv", [(8, 2), (4, 4)])
def test_paged_decode_matches_oracle(dt, tol, Hq, Hkv):
    D = 64
    kc, vc = _cache(dt, Hkv=Hkv)
    g = torch.Generator().manual_seed(1)
    lens = torch.tensor([1, 17, 40, 0, 100, 128], dtype=torch.int32)
    bt = torch.stack([torch.randperm(64, generator=g)[:8] for _ in range(6)]).int()
    bt[3] = -1
    bt[0, 1:] = -1
    q = torch.randn(6, Hq * D, generator=g).to(dt)
    a = ref.paged_decode(q, kc, vc, bt, lens, Hq, Hkv, D, 0.125)
    b = cpu_attn.paged_decode(q, kc, vc, bt, lens, Hq, Hkv, D, 0.125)
    assert b.dtype == q.dtype and b.shape == a.shape
    assert torch.all(b[3] == 0)
    assert (a.float() - b.float()).abs().max().item() <= tol


def test_prefill_forms_match_oracle():
    Hq, Hkv, D = 8, 2, 64
    kc, vc = _cache(torch.float32)
    g = torch.Generator().manual_seed(2)
    cu = torch.tensor([0, 5, 38, 38, 60])
    qkv = torch.randn(60, (Hq + 2 * Hkv) * D, generator=g)
    a = ref.flash_prefill(qkv, cu, Hq, Hkv, D, 0.125)
    b = cpu_attn.flash_prefill(qkv, cu, Hq, Hkv, D, 0.125)
    torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-5)
    cs = torch.tensor([10, 30, 0, 7])
    bt = torch.stack([torch.randperm(64, generator=g)[:8] for _ in range(4)]).int()
    a = ref.paged_prefill(qkv, cu, cs, kc, vc, bt, Hq, Hkv, D, 0.125)
    b = cpu_attn.paged_prefill(qkv, cu, cs, kc, vc, bt, Hq, Hkv, D, 0.125)
    torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-5)


def test_runner_auto_kv_pool_holds_every_sequence():
    from k8s_llm_monitor_amd.engine import EngineConfig, LLMEngine

    eng = LLMEngine(EngineConfig(model="llama-tiny-d128", max_num_seqs=8, max_model_len=256, kv_cache_gb=0.0,
                                 use_graphs=False, seed=0, dtype="float32"), device="cpu")
    r = eng.runner
    assert r.num_blocks == 8 * r.max_blocks_per_seq + 1
