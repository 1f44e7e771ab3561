"""The fast path sums checksums in the little-endian domain (v_dot2_u32_u16 over raw words)
and byte-swaps once at the end (gpd_kernels.hip fold_le_not).  This pins the identity it
relies on against tcpipChecksum's own fold (layers/tcpip.go:52-70): for any word sequence
whose sums do not wrap 2^32, ~fold(sum of big-endian words) == swap16(~fold(sum of
byte-swapped words)) — including the all-zero and 0xFFFF-multiple representatives."""
import numpy as np


def _go_fold_not(s: int) -> int:  # tcpip.go:66-69
    s &= 0xFFFFFFFF
    while s > 0xFFFF:
        s = (s >> 16) + (s & 0xFFFF)
    return ~s & 0xFFFF


def _le_fold_not(words) -> int:  # fold_le_not over the LE-domain sum
    s = int(sum(((w & 0xFF) << 8) | (w >> 8) for w in words))
    s = (s >> 16) + (s & 0xFFFF)
    s = (s >> 16) + (s & 0xFFFF)
    r = ~s & 0xFFFF
    return ((r & 0xFF) << 8) | (r >> 8)


def test_le_domain_fold_matches_go_fold():
    rng = np.random.default_rng(0x5EED)
    cases = [[], [0], [0] * 9, [0xFFFF], [0xFFFF] * 7, [0x1234, 0xEDCB], [0x8000] * 2]
    for _ in range(20000):
        n = int(rng.integers(0, 48))
        kind = rng.random()
        if kind < 0.1:
            ws = [0xFFFF] * n
        elif kind < 0.2:
            ws = [int(x) for x in rng.integers(0xFF00, 0x10000, n)]
        else:
            ws = [int(x) for x in rng.integers(0, 0x10000, n)]
        cases.append(ws)
    for ws in cases:
        assert _go_fold_not(sum(ws)) == _le_fold_not(ws), ws


def test_two_folds_reach_16_bits():
    for s in [0, 1, 0xFFFF, 0x10000, 0x1FFFE, 0xFFFFFFFF, 0x8000FFFF, 0xFFFF0001]:
        r = (s >> 16) + (s & 0xFFFF)
        r = (r >> 16) + (r & 0xFFFF)
        assert r <= 0xFFFF
        assert _go_fold_not(s) == ~r & 0xFFFF
