"""C++ runtime (block allocator, BPE encoder, decode packing) and the tokenizer."""
import random

import numpy as np
import pytest

from k8s_llm_monitor_amd.engine.block_manager import BlockManager, PyBlockPool, py_block_hashes
from k8s_llm_monitor_amd.engine.sequence import SamplingParams, Sequence
from k8s_llm_monitor_amd.engine.tokenizer import ByteBPETokenizer, tokenizer_for, train_bpe
from k8s_llm_monitor_amd.llm.synthetic import synthetic_cluster_prompt
from k8s_llm_monitor_amd.models import get_config
from k8s_llm_monitor_amd.runtime import native_runtime

rt = native_runtime()
needs_rt = pytest.mark.skipif(rt is None, reason="C++ runtime not built")


@needs_rt
def test_native_allocator_matches_python_and_catches_double_free():
    a, b = rt.BlockAllocator(16), PyBlockPool(16)
    for n in (3, 5, 2):
        assert a.allocate(n) == b.allocate(n)
    assert a.allocate(100) is None and a.num_free == b.num_free == 6
    a.free([0, 1])
    with pytest.raises(RuntimeError, match="double free"):
        a.free([1])


@pytest.mark.parametrize("native", [True, False])
def test_block_pool_prefix_cache(native):
    if native and rt is None:
        pytest.skip("C++ runtime not built")
    p = rt.BlockPool(6) if native else PyBlockPool(6)
    hashes = rt.block_hashes if native else py_block_hashes
    toks = list(range(40))
    h = hashes(toks, 16, 0)
    assert len(h) == 2 and h == py_block_hashes(toks, 16, 0)  # native and Python chains agree
    assert hashes(toks[:16] + [99] * 16, 16, 0)[0] == h[0] != hashes(toks[:16] + [99] * 16, 16, 0)[1]
    b = p.allocate(3)
    for blk, hh in zip(b, h):
        p.publish(blk, hh)
    assert p.peek(h) == 2 and p.num_cached == 2
    m = p.match(h)  # second reference on the two prefix blocks
    assert m == b[:2] and p.refcount(b[0]) == 2
    p.release(b)
    assert p.num_free == 4 and p.refcount(b[0]) == 1
    p.release(m)  # last references: the prefix blocks stay cached but are evictable
    assert p.num_free == 6 and p.num_cached == 2
    got = p.allocate(5)  # 4 plain free + 1 eviction (least recently used cached block)
    assert len(got) == 5 and p.num_cached == 1 and p.stats()["evictions"] == 1
    with pytest.raises(RuntimeError, match="double free"):
        p.release([b[2]]) if b[2] not in got else p.release([got[0], got[0]])


def test_block_manager_slots():
    bm = BlockManager(8, use_native=False)
    s = Sequence(prompt_ids=list(range(20)), params=SamplingParams())
    assert bm.can_allocate(s) and bm.allocate(s) and len(s.block_table) == 2
    s.output_ids = [1] * 12  # 32 tokens -> the next write needs a third block
    assert bm.ensure_slot(s) and len(s.block_table) == 3
    bm.free(s)
    assert bm.num_free == 8


@pytest.mark.parametrize("native", [True, False])
def test_block_manager_prefix_sharing(native):
    if native and rt is None:
        pytest.skip("C++ runtime not built")
    bm = BlockManager(32, use_native=native)
    a = Sequence(prompt_ids=list(range(50)), params=SamplingParams())
    b = Sequence(prompt_ids=list(range(40)) + [7] * 5, params=SamplingParams())
    c = Sequence(prompt_ids=list(range(32)), params=SamplingParams())  # exactly 2 full blocks
    assert bm.allocate(a) and a.num_cached == 0
    assert bm.cached_prefix_tokens(b) == 0  # published only when a prefill step computes them
    bm.publish_computed(a, 16)  # chunked prefill: a's first chunk covers one block
    assert bm.cached_prefix_tokens(b) == 16
    bm.publish_computed(a, a.num_tokens)
    assert bm.cached_prefix_tokens(b) == 32 and bm.allocate(b) and b.num_cached == 32
    bm.publish_computed(b, b.num_tokens)
    assert b.block_table[:2] == a.block_table[:2] and b.block_table[2] != a.block_table[2]
    # a fully cached prompt still runs its last token: only the first block is reused
    assert bm.allocate(c) and c.num_cached == 16
    bm.free(a)
    bm.free(b)
    bm.free(c)
    assert bm.num_free == 32
    assert bm.stats()["prefix_cached_tokens"] == 48


@needs_rt
def test_native_bpe_parity_with_python():
    tok = tokenizer_for(get_config("llama-3-8b"))
    assert tok._native is not None
    py = ByteBPETokenizer(tok.merges, bos_id=tok.bos_id)
    py._native = None
    r = random.Random(0)
    texts = [synthetic_cluster_prompt(s) for s in range(5)]
    alphabet = ["a", "Z", "1", " ", "  ", "\n", "\t", "'", "s", "中", "!", "-", "　", "\xa0", "é", "re", "ll"]
    texts += ["".join(r.choice(alphabet) for _ in range(r.randrange(1, 40))) for _ in range(500)]
    for t in texts:
        assert tok.encode(t) == py.encode(t), repr(t)


def test_tokenizer_roundtrip_and_vocab_bounds():
    for name in ("llama-3-8b", "mixtral-8x7b", "llama-tiny", "gpt2-small"):
        cfg = get_config(name)
        tok = tokenizer_for(cfg)
        text = synthetic_cluster_prompt(1)
        ids = tok.encode(text)
        assert ids[0] == cfg.bos_id and max(ids) < cfg.vocab_size
        assert tok.decode(ids) == text
        # a random-init model samples anywhere in the vocab: decode must never fail
        assert isinstance(tok.decode(list(range(cfg.vocab_size - 50, cfg.vocab_size))), str)
    tok = tokenizer_for(get_config("llama-3-8b"))
    assert len(tok.encode(synthetic_cluster_prompt(2))) < len(synthetic_cluster_prompt(2).encode()) / 2.5


def test_train_bpe_small():
    m = train_bpe(["aaab aaab aaab", "ab ab"], num_merges=10)
    t = ByteBPETokenizer(m)
    assert t.decode(t.encode("aaab ab", bos=False)) == "aaab ab"
    assert len(t.encode("aaab", bos=False)) < 4


@needs_rt
def test_pack_decode():
    B, W = 4, 8
    ids, pos, slots, lens = (np.zeros(B, np.int32) for _ in range(4))
    bt = np.full((B, W), 7, np.int32)
    rt.pack_decode(ids, pos, slots, lens, bt, [5, 6], [17, 3], [[4, 9], [2]], 3, 16)
    assert list(ids[:3]) == [5, 6, 0] and list(pos[:3]) == [16, 2, 0]
    assert list(slots[:3]) == [9 * 16 + 0, 2 * 16 + 2, -1] and list(lens[:3]) == [17, 3, 0]
    assert list(bt[0, :3]) == [4, 9, 0] and bt[3, 0] == 7
