"""Real-weight checkpoints (models/checkpoint.py): Hugging Face safetensors directories written by
``transformers`` itself load into CausalLM and reproduce the Hugging Face forward (fp32, CPU) -
parity of the model math (RoPE pairing, GQA, RMSNorm, SwiGLU, MoE routing, GPT-2 Conv1D layout)
against the reference implementation of each architecture, plus save -> load round trips and the
engine / tokenizer wiring."""
import json

import pytest
import torch

from k8s_llm_monitor_amd.models import AttnMeta, CausalLM, config_from_hf, load_checkpoint, save_checkpoint
from k8s_llm_monitor_amd.models.config import get_config

transformers = pytest.importorskip("transformers")


def _prefill_logits(model, ids):
    n = len(ids)
    meta = AttnMeta(is_prefill=True, positions=torch.arange(n, dtype=torch.int32),
                    slot_mapping=torch.full((n,), -1, dtype=torch.int32),
                    cu_seqlens=torch.tensor([0, n], dtype=torch.int32))
    return model.forward(torch.tensor(ids, dtype=torch.int32), meta, None).float()


def _hf_tiny(kind: str):
    torch.manual_seed(0)
    if kind == "llama":
        cfg = transformers.LlamaConfig(vocab_size=320, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                                       num_attention_heads=4, num_key_value_heads=2, head_dim=32,
                                       max_position_embeddings=256, rope_theta=500000.0, rms_norm_eps=1e-5,
                                       tie_word_embeddings=False, bos_token_id=1, eos_token_id=2)
        return transformers.LlamaForCausalLM(cfg)
    if kind == "llama31":  # Llama-3.1 rope frequency remap
        cfg = transformers.LlamaConfig(vocab_size=320, hidden_size=128, intermediate_size=256, num_hidden_layers=1,
                                       num_attention_heads=4, num_key_value_heads=1, max_position_embeddings=512,
                                       rope_theta=500000.0, tie_word_embeddings=True, bos_token_id=1, eos_token_id=2,
                                       rope_scaling={"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                                                     "high_freq_factor": 4.0,
                                                     "original_max_position_embeddings": 64})
        return transformers.LlamaForCausalLM(cfg)
    if kind == "mixtral":
        cfg = transformers.MixtralConfig(vocab_size=320, hidden_size=128, intermediate_size=192, num_hidden_layers=2,
                                         num_attention_heads=4, num_key_value_heads=2, head_dim=32,
                                         num_local_experts=4, num_experts_per_tok=2, max_position_embeddings=256,
                                         rope_theta=1e6, bos_token_id=1, eos_token_id=2)
        return transformers.MixtralForCausalLM(cfg)
    cfg = transformers.GPT2Config(vocab_size=300, n_embd=96, n_layer=2, n_head=4, n_positions=128,
                                  bos_token_id=0, eos_token_id=0)
    return transformers.GPT2LMHeadModel(cfg)


def _randomize(hf):
    """Non-trivial norms / biases (HF inits them to 1 / 0, which would hide layout mistakes)."""
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for n, p in hf.named_parameters():
            if p.dim() == 1:
                p.copy_(1.0 + 0.1 * torch.randn(p.shape, generator=g) if "norm" in n or "ln" in n
                        else 0.05 * torch.randn(p.shape, generator=g))
    return hf


@pytest.mark.parametrize("kind", ["llama", "llama31", "mixtral", "gpt2"])
def test_hf_checkpoint_matches_transformers_forward(tmp_path, kind):
    hf = _randomize(_hf_tiny(kind)).float().eval()
    hf.save_pretrained(tmp_path, safe_serialization=True)
    cfg = config_from_hf(tmp_path)
    assert cfg.arch == ("gpt2" if kind == "gpt2" else "llama")
    assert cfg.is_moe == (kind == "mixtral")
    m = CausalLM(cfg, device="cpu", dtype=torch.float32, init="empty")
    unused = load_checkpoint(m, tmp_path)
    assert unused == []
    ids = [1, 17, 33, 250, 5, 99, 140, 7, 61, 200, 3, 45]
    ours = _prefill_logits(m, ids)
    with torch.no_grad():
        ref = hf(torch.tensor([ids])).logits[0].float()
    err = (ours - ref).abs().max().item()
    assert err < 2e-3 * max(1.0, ref.abs().max().item()), f"{kind}: max |logit diff| {err}"
    assert torch.equal(ours.argmax(-1), ref.argmax(-1))


@pytest.mark.parametrize("model", ["llama-tiny", "mixtral-tiny", "gpt2-tiny"])
def test_save_load_roundtrip(tmp_path, model):
    cfg = get_config(model)
    a = CausalLM(cfg, device="cpu", dtype=torch.float32, seed=5)
    save_checkpoint(a, tmp_path, max_shard_bytes=200_000)  # force several shards + an index
    assert (tmp_path / "config.json").exists()
    assert len(list(tmp_path.glob("*.safetensors"))) > 1 and (tmp_path / "model.safetensors.index.json").exists()
    cfg2 = config_from_hf(tmp_path)
    for f in ("vocab_size", "d_model", "n_layers", "n_heads", "n_kv_heads", "head_dim", "ffn_dim", "n_experts",
              "tie_embeddings", "bos_id"):
        assert getattr(cfg2, f) == getattr(cfg, f), f
    b = CausalLM(cfg2, device="cpu", dtype=torch.float32, seed=99)  # different random init, then overwritten
    load_checkpoint(b, tmp_path)
    ids = [3, 9, 27, 81, 243 % cfg.vocab_size, 11]
    assert torch.equal(_prefill_logits(a, ids), _prefill_logits(b, ids))


def test_tp_shards_from_checkpoint(tmp_path):
    """Each TP rank cuts its own shard out of the same checkpoint: the rank-local tensors equal
    the corresponding slices of the TP=1 model (fused qkv / gate-up layout per rank)."""
    from k8s_llm_monitor_amd.parallel.state import ParallelState

    cfg = get_config("llama-tiny")
    full = CausalLM(cfg, device="cpu", dtype=torch.float32, seed=2)
    save_checkpoint(full, tmp_path)
    D, F = full.D, cfg.ffn_dim
    nq, nk = cfg.n_heads * D, cfg.n_kv_heads * D
    for r in range(2):
        ps = ParallelState(rank=r, world_size=2, tp_size=2, tp_rank=r, dp_rank=0, device=torch.device("cpu"))
        m = CausalLM(cfg, device="cpu", dtype=torch.float32, pstate=ps, init="empty")
        load_checkpoint(m, tmp_path)
        L, L0 = m.layers[0], full.layers[0]
        q = L0["wqkv"][:nq].chunk(2)[r]
        k = L0["wqkv"][nq:nq + nk].chunk(2)[r]
        v = L0["wqkv"][nq + nk:].chunk(2)[r]
        assert torch.equal(L["wqkv"], torch.cat([q, k, v]))
        from k8s_llm_monitor_amd import ops

        def canon(model, w):  # resident w13 is gate/up-interleaved per 128 rows when F allows
            return ops.deinterleave_gate_up(w) if model._w13_il else w

        w0 = canon(full, L0["w13"])
        assert torch.equal(canon(m, L["w13"]), torch.cat([w0[:F].chunk(2)[r], w0[F:].chunk(2)[r]]))
        assert torch.equal(L["wo"], L0["wo"].chunk(2, dim=1)[r])
        assert torch.equal(m.embed, full.embed.chunk(2)[r])


def test_engine_serves_checkpoint_dir_with_hf_tokenizer(tmp_path):
    """EngineConfig.weights: config, weights and tokenizer.json all come from the directory."""
    tokenizers = pytest.importorskip("tokenizers")
    from k8s_llm_monitor_amd.engine import EngineConfig, LLMEngine, SamplingParams
    from k8s_llm_monitor_amd.engine.tokenizer import HFTokenizer

    cfg = get_config("llama-tiny")
    save_checkpoint(CausalLM(cfg, device="cpu", dtype=torch.float32, seed=4), tmp_path)
    tok = tokenizers.Tokenizer(tokenizers.models.BPE(unk_token="<unk>"))
    tok.pre_tokenizer = tokenizers.pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = tokenizers.decoders.ByteLevel()
    tok.train_from_iterator(["pod default/api-gateway CrashLoopBackOff on node-003 " * 20],
                            tokenizers.trainers.BpeTrainer(vocab_size=300, special_tokens=["<unk>", "<s>", "</s>"]))
    tok.save(str(tmp_path / "tokenizer.json"))
    eng = LLMEngine(EngineConfig(model="unused-preset-name", weights=str(tmp_path), max_num_seqs=2, max_model_len=128,
                                 num_blocks=32, use_graphs=False, dtype="float32"), device="cpu")
    assert isinstance(eng.tokenizer, HFTokenizer)
    assert eng.model_cfg.d_model == cfg.d_model
    text = "pod default/api-gateway CrashLoopBackOff"
    ids = eng.tokenizer.encode(text)
    assert ids[0] == cfg.bos_id and eng.tokenizer.decode(ids) == text
    seqs = eng.generate([text], SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True))
    assert len(seqs[0].output_ids) == 4


def test_config_from_hf_transformers5_rope_parameters():
    c = config_from_hf({"model_type": "llama", "vocab_size": 128256, "hidden_size": 4096, "num_hidden_layers": 32,
                        "num_attention_heads": 32, "num_key_value_heads": 8, "intermediate_size": 14336,
                        "rope_parameters": {"rope_type": "llama3", "rope_theta": 500000.0, "factor": 8.0,
                                            "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                                            "original_max_position_embeddings": 8192},
                        "bos_token_id": 128000, "eos_token_id": [128001, 128008, 128009]})
    assert c.rope_theta == 500000.0 and c.rope_scaling["factor"] == 8.0 and c.head_dim == 128
    assert c.eos_ids == (128001, 128008, 128009)
    with pytest.raises(ValueError):
        config_from_hf({"model_type": "falcon"})
    json.dumps(c.rope_scaling)


@pytest.mark.gpu
def test_gpu_engine_on_hf_checkpoint_matches_transformers(tmp_path):
    """A transformers-written Llama checkpoint (head_dim 128, GQA) served by the engine on the GPU
    in bf16 - flash prefill, hipGraph decode, skinny GEMMs, sampler - greedily generates what the
    fp32 transformers model generates (allowing near-ties from bf16 rounding)."""
    from k8s_llm_monitor_amd import ops
    from k8s_llm_monitor_amd.engine import EngineConfig, LLMEngine, SamplingParams

    ops.native()
    torch.manual_seed(0)
    cfg = transformers.LlamaConfig(vocab_size=1024, hidden_size=512, intermediate_size=1024, num_hidden_layers=2,
                                   num_attention_heads=8, num_key_value_heads=2, head_dim=128,
                                   max_position_embeddings=1024, rope_theta=500000.0, tie_word_embeddings=False,
                                   bos_token_id=1, eos_token_id=2)
    hf = _randomize(transformers.LlamaForCausalLM(cfg)).float().eval()
    with torch.no_grad():  # larger weights: decisive logits, so bf16 rounding rarely flips a choice
        for p in hf.parameters():
            if p.dim() == 2:
                p.mul_(3.0)
    hf.save_pretrained(tmp_path, safe_serialization=True)
    eng = LLMEngine(EngineConfig(weights=str(tmp_path), max_num_seqs=4, max_model_len=512, num_blocks=64, seed=0),
                    device="cuda:0")
    eng.warmup()
    prompts = [[1, 17, 33, 250, 5, 99, 140, 7, 61, 200, 3, 45] * 3, [1, 900, 12, 12, 4, 700, 31]]
    n_new = 12
    seqs = eng.generate(prompts, SamplingParams(max_tokens=n_new, temperature=0.0, ignore_eos=True))
    agree = total = 0
    for s, p in zip(seqs, prompts):
        with torch.no_grad():
            out = hf.generate(torch.tensor([p]), max_new_tokens=n_new, do_sample=False,
                              attention_mask=torch.ones(1, len(p), dtype=torch.long))[0, len(p):].tolist()
        for a, b in zip(s.output_ids, out):
            total += 1
            agree += int(a == b)
            if a != b:
                break  # the continuations diverge after the first differing token
    assert agree >= 0.8 * total, (agree, total)
