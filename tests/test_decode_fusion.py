"""The decode-step fusion (CausalLM.set_decode_fusion: the row-complete o projection) is a
drop-in replacement for add_norm_partial: on the CPU (their fp32 reference forms, the same control flow the GPU takes)
an engine generates the same greedy tokens with each of them as with the default path.  The
kernels themselves are checked bit for bit against the default path in
tests/test_gemm_decode_gpu.py."""
import pytest
import torch

from k8s_llm_monitor_amd.engine import EngineConfig, LLMEngine, SamplingParams


def _run(rc) -> list:
    eng = LLMEngine(EngineConfig(model="llama-tiny-d128", max_num_seqs=4, max_model_len=256, num_blocks=64,
                                 use_graphs=False, seed=3, dtype="float32"), device="cpu")
    eng.model.set_decode_fusion(rc=rc)
    assert bool(eng.model._rc_o) == (rc is None or bool(rc))
    assert eng.model._skinny_ws is not None  # the decode steps take the fused-tail (skinny) path
    sp = SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True)
    seqs = eng.generate(["node-003 NotReady: kubelet stopped posting status", "pod default/api CrashLoopBackOff"], sp)
    return [s.output_ids for s in seqs]


@pytest.mark.parametrize("rc", [True, None, 2])
def test_decode_fusions_match_default(rc):
    torch.manual_seed(0)
    assert _run(rc) == _run(False)


def test_rc_auto_only_small_buckets():
    eng = LLMEngine(EngineConfig(model="llama-tiny-d128", max_num_seqs=4, max_model_len=256, num_blocks=64,
                                 use_graphs=False, seed=3, dtype="float32"), device="cpu")
    m = eng.model
    assert m._rc_o == m.RC_O_MAX_ROWS  # the default: the smallest buckets only
    m.set_decode_fusion(rc=False)
    assert m._rc_o == 0
    m.set_decode_fusion(rc=True)
    assert m._rc_o >= 1 << 20
