"""The index maps the frame-pair spectral kernels rely on (CPU; restated from
csrc/fft_pair.h pair_bin_lane, csrc/fft_pair512.h pair512_bin and the comments of
csrc/pair_mask.hip / csrc/pair_stft.hip), checked exhaustively:

  * the bin of (lane l, register d) is q(l) + 64 d with q an involution;
  * its partner bin N - k sits in register E-1-d of lane q(64 - q(l)), except in
    lane 0, where it is register (E - d) mod E of lane 0 (ds_bpermute + readlane);
  * the forward split stores every real bin 0 .. N/2 exactly once (registers
    d < E/2 in every lane, register E/2 in lane 0);
  * the inverse's scrambled reads (buf + q + 64 d for d < E/2, buf - q + N - 64 d
    above) land on the real bin min(k, N - k), conjugated above N/2.
"""
import pytest


def q1024(l):
    return (l & 3) + 4 * (l >> 4) + 16 * ((l >> 2) & 3)


def q512(l):
    return (l >> 3) + 8 * (l & 7)


@pytest.mark.parametrize("n,E,q", [(1024, 16, q1024), (512, 8, q512)])
def test_pair_bin_maps(n, E, q):
    lanes = range(64)
    assert sorted(q(l) for l in lanes) == list(range(64))
    assert all(q(q(l)) == l for l in lanes)  # involution
    where = {q(l) + 64 * d: (l, d) for l in lanes for d in range(E)}
    assert sorted(where) == list(range(n))
    for l in lanes:
        partner = q((64 - q(l)) & 63)
        for d in range(E):
            kb = q(l) + 64 * d
            want = where[(n - kb) % n]
            got = (0, (E - d) % E) if l == 0 else (partner, E - 1 - d)
            assert got == want, (n, l, d)
    # the forward split's stores: bins 0 .. N/2, each once
    stored = [q(l) + 64 * d for l in lanes for d in range(E // 2)] + [q(0) + 64 * (E // 2)]
    assert sorted(stored) == list(range(n // 2 + 1))
    # the inverse's scrambled reads of the staged real bins
    for l in lanes:
        for d in range(E):
            kb = q(l) + 64 * d
            idx = q(l) + 64 * d if d < E // 2 else -q(l) + n - 64 * d
            assert idx == min(kb, n - kb), (n, l, d)
            assert 0 <= idx <= n // 2


def test_pair15_bin_map():
    """N = 960 (csrc/fft_pair15.h pair15_bin, csrc/pair15_spec.hip q15_partner): bin
    k1 + 15 k' in lane l, register d, k1 = (l & 3) + 4 (l >> 4) (15: the zero row),
    k' = ((l >> 2) & 3) + 4 d; the partner N - k in register 15 - d of
    q15_partner(l), lane 0 its own register (16 - d) mod 16; the stores of bins
    0 .. N/2 (registers d < 8 of the bin lanes, register 8 of lane 0) each once."""
    n = 960

    def k1(l):
        return (l & 3) + 4 * (l >> 4)

    def b15(l, d):
        return k1(l) + 15 * (((l >> 2) & 3) + 4 * d)

    def partner(l):
        j = (l >> 2) & 3
        if k1(l) == 15:
            return l
        if k1(l) == 0:
            return 0 if j == 0 else 4 * (4 - j)
        kp = 15 - k1(l)
        return (kp & 3) + 4 * (3 - j) + 16 * (kp >> 2)

    live = [l for l in range(64) if k1(l) != 15]
    assert len(live) == 60
    where = {b15(l, d): (l, d) for l in live for d in range(16)}
    assert sorted(where) == list(range(n))
    for l in live:
        for d in range(16):
            want = where[(n - b15(l, d)) % n]
            got = (0, (16 - d) % 16) if l == 0 else (partner(l), 15 - d)
            assert got == want, (l, d)
    stored = [b15(l, d) for l in live for d in range(8)] + [b15(0, 8)]
    assert sorted(stored) == list(range(n // 2 + 1))


def test_pair15h_bin_map():
    """N = 480 (csrc/fft_pair15.h pair15h_bin, csrc/pair15_spec.hip Q15<32>::partner):
    half-lane h holds bin k1 + 15 (c + 2 e), k1 = (h & 7) + 8 (h >> 4) (15: the zero
    row), c = (h >> 3) & 1; the partner N - k in register 15 - e of partner(h)
    (half-lane 0: its own register (16 - e) mod 16); bins 0 .. N/2 stored once."""
    n = 480

    def k1(h):
        return (h & 7) + 8 * (h >> 4)

    def b(h, e):
        return k1(h) + 15 * (((h >> 3) & 1) + 2 * e)

    def partner(h):
        if k1(h) in (0, 15):
            return h
        c, kp = (h >> 3) & 1, 15 - k1(h)
        return (kp & 7) + 8 * (1 - c) + 16 * (kp >> 3)

    live = [h for h in range(32) if k1(h) != 15]
    assert len(live) == 30
    where = {b(h, e): (h, e) for h in live for e in range(16)}
    assert sorted(where) == list(range(n))
    for h in live:
        for e in range(16):
            want = where[(n - b(h, e)) % n]
            got = (0, (16 - e) % 16) if h == 0 else (partner(h), 15 - e)
            assert got == want, (h, e)
    stored = [b(h, e) for h in live for e in range(8)] + [b(0, 8)]
    assert sorted(stored) == list(range(n // 2 + 1))
