"""CPU proof of the paged-decode operand layout (ops/csrc/paged_decode.hip, `issue` / `compute`):
the QK tile rows are ordered so that, for every lane, the 8 score values that become the PV
product's B operand belong to the same 8 tokens as the V fragment that lane loads with ONE 16-byte
read from the v_perm-ordered V cache.  Mirrors the kernel's index formulas; no GPU needed."""


def v_perm(t: int) -> int:  # common.h: swap bits 2 and 3 of the in-block token index (involution)
    return (t & ~12) | ((t & 4) << 1) | ((t & 8) >> 1)


def k_row_token(c: int, j: int) -> int:
    """Token (within a 32-token PV step) that QK tile 2s + j row c holds (the K load of lane c)."""
    return 16 * (c >> 3) + 8 * j + 4 * ((c >> 2) & 1) + (c & 3)


def test_v_perm_is_an_involution():
    assert all(v_perm(v_perm(t)) == t for t in range(16))
    assert sorted(v_perm(t) for t in range(16)) == list(range(16))


def test_score_lanes_match_one_16_byte_v_fragment():
    for kg in range(4):  # lane group = MFMA k-group
        # B operand (P): element e = sacc[2s + (e >> 2)][e & 3] = score of output row 4 kg + (e & 3)
        p_tokens = [k_row_token(4 * kg + (e & 3), e >> 2) for e in range(8)]
        # A operand (V^T): one 16-byte load = positions 8 (kg & 1) .. + 7 of block 2s + (kg >> 1)
        v_tokens = [16 * (kg >> 1) + v_perm(8 * (kg & 1) + e) for e in range(8)]
        assert p_tokens == v_tokens, (kg, p_tokens, v_tokens)


def test_each_tile_pair_covers_the_step_once():
    toks = sorted(k_row_token(c, j) for j in range(2) for c in range(16))
    assert toks == list(range(32))
    # a K load row stays inside one 16-token cache block: block index c >> 3
    for j in range(2):
        for c in range(16):
            assert k_row_token(c, j) // 16 == c >> 3


def test_mask_index_matches_the_row_mapping():
    # compute(): t = wtok0 + 32 (i >> 1) + 16 (kg >> 1) + 8 (i & 1) + 4 (kg & 1) + r for sacc[i][r]
    for i in range(4):
        for kg in range(4):
            for r in range(4):
                t = 32 * (i >> 1) + 16 * (kg >> 1) + 8 * (i & 1) + 4 * (kg & 1) + r
                assert t == 32 * (i >> 1) + k_row_token(4 * kg + r, i & 1)
