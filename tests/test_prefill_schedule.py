"""Q-block schedule of the flash prefill kernel (CPU): every 128-row block of every sequence is
listed exactly once under both orders; the sequence-major order keeps a sequence's blocks together,
heaviest first, longest sequence first."""
import pytest

from k8s_llm_monitor_amd import ops


@pytest.mark.parametrize("order", ["seq", "work"])
def test_qblocks_cover_every_block_once(order):
    lens, starts = [300, 1609, 7, 128, 1000], [0, 0, 50, 4096, 0]
    cu = [0]
    for n in lens:
        cu.append(cu[-1] + n)
    seqs, firsts = ops.prefill_qblocks(cu, ctx_starts=starts, order=order)
    want = sorted((i, s) for i, n in enumerate(lens) for s in range(0, n, 128))
    assert sorted(zip(seqs, firsts)) == want
    work = [starts[i] + s for i, s in zip(seqs, firsts)]
    if order == "work":
        assert work == sorted(work, reverse=True)
    else:
        runs = [seqs[0]]
        for i in seqs[1:]:
            if i != runs[-1]:
                assert i not in runs  # one contiguous run per sequence
                runs.append(i)
        tot = [starts[i] + lens[i] for i in runs]
        assert tot == sorted(tot, reverse=True)
        for i in runs:
            w = [starts[i] + s for j, s in zip(seqs, firsts) if j == i]
            assert w == sorted(w, reverse=True)
