"""dsp::Framer drop-in (crlot_framer_*, a host object in the product library)
against the reference's own compiled framer.cc outputs (tests/golden/ref_tables.npz,
26 push/pop cases with available_frames traces) and the behaviours
tests/framer_test.cc checks.  Host code only: runs without a GPU."""
import numpy as np
import pytest

from test_oracle_pins import _framer_case


def run_product_framer(pkg, x, T, C, n, h, mode, chunk=0):
    """framer_run's loop (oracle/oracle.py) on the product Framer."""
    f = pkg.Framer()
    f.set_params(n, h, C, mode)
    frames, avail = [], []
    pos, chunk = 0, chunk or T
    while pos < T:
        m = min(chunk, T - pos)
        assert f.push(x[pos * C:(pos + m) * C], m)
        pos += m
        avail.append(f.available_frames())
        while True:
            fr = f.pop()
            if fr is None:
                break
            frames.append(fr.copy())
    fr = np.concatenate(frames) if frames else np.zeros(0, np.float32)
    return fr, np.array(avail, np.uint64)


def test_framer_bit_exact_vs_reference_build(pkg, ref_tables):
    n_cases = 0
    for key in ref_tables.files:
        if not key.startswith("framer_") or key.endswith("_avail"):
            continue
        tag = key[len("framer_"):]
        mode = pkg.DROP if tag.endswith("_drop") or "_drop_" in tag else pkg.ZERO_PAD
        x, T, C, N, H, chunk = _framer_case(tag)
        fr, av = run_product_framer(pkg, x, T, C, N, H, mode, chunk)
        assert np.array_equal(fr, ref_tables[key]), tag
        assert np.array_equal(av, ref_tables[key + "_avail"]), tag
        n_cases += 1
    assert n_cases == 26


def test_framer_matches_oracle_random_chunks(pkg, oracle):
    rng = np.random.default_rng(7)
    for _ in range(40):
        n = int(rng.integers(1, 40))
        h = int(rng.integers(1, n + 3))
        C = int(rng.integers(1, 4))
        T = int(rng.integers(0, 200))
        mode = int(rng.integers(0, 2))
        chunk = int(rng.integers(0, 30))
        x = rng.standard_normal(T * C).astype(np.float32)
        a = run_product_framer(pkg, x, T, C, n, h, mode, chunk) if T else (np.zeros(0), [])
        b = oracle.framer_run(x, T, C, n, h, mode, chunk) if T else (np.zeros(0), [])
        assert np.array_equal(a[0], b[0]) and np.array_equal(np.asarray(a[1]), np.asarray(b[1]))


def test_framer_api_behaviour(pkg):
    """framer_test.cc:100-321 (BasicPushPop, InterleavedChannels, VeryShortLengths,
    BoundaryConditions, FramingCompatibilityFormula, MemoryEfficiency) and the
    set_params / push / pop guards (framer.cc:15-67)."""
    sine = np.sin(2 * np.pi * np.arange(1000) / 50.0).astype(np.float32)
    f = pkg.Framer()
    assert f.pop() is None and f.available_frames() == 0           # params unset
    assert not f.push(sine, 10)
    for bad in ((0, 1, 1), (1, 0, 1), (1, 1, 0)):
        with pytest.raises(ValueError):
            f.set_params(*bad)
    f.set_params(64, 16, 1)
    assert f.push(sine) and f.available_frames() > 0 and f.pop() is not None
    st = pkg.Framer()
    st.set_params(32, 8, 2)
    stereo = np.stack([sine, np.cos(2 * np.pi * np.arange(1000) / 30.0).astype(np.float32)], 1)
    assert st.push(stereo.reshape(-1)[:200], 100)
    fr = st.pop()
    assert fr.size == 64 and st.channels() == 2
    assert np.array_equal(fr, stereo.reshape(-1)[:64])
    v = pkg.Framer()
    v.set_params(32, 8, 1)
    assert v.push(None, 0) and v.available_frames() == 0
    assert v.push(np.ones(1, np.float32), 1) and v.push(np.full(7, 0.5, np.float32))
    assert not v.push(None, 3)                                      # null with frames > 0
    zp, dr = pkg.Framer(), pkg.Framer()
    zp.set_params(32, 16, 1, pkg.ZERO_PAD)
    dr.set_params(32, 16, 1, pkg.DROP)
    short = np.ones(20, np.float32)
    assert zp.push(short) and dr.push(short)
    got = zp.pop()
    assert got is not None and np.all(got[20:] == 0) and np.all(got[:20] == 1)
    assert dr.pop() is None
    c = pkg.Framer()
    c.set_params(64, 16, 1)
    c.push(np.ones(200, np.float32))
    assert c.available_frames() == (200 - 64) // 16 + 1
    m = pkg.Framer()
    m.set_params(1024, 256, 2)
    b0 = m.buffer_size()
    assert b0 == 2 * 1024 * 2
    m.push(np.ones(20000, np.float32), 10000)
    assert m.buffer_size() >= b0
    k = 0
    while m.pop() is not None and k < 100:
        k += 1
    assert k > 0
    m.reset()
    assert m.available_frames() == 0 and m.buffer_size() == b0
    assert (m.frame_size(), m.hop_size(), m.channels(), m.boundary_mode()) == (1024, 256, 2, pkg.ZERO_PAD)
