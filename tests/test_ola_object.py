"""dsp::OLAAccumulator drop-in (crlot_ola_*: device rings, host counters) against
the oracle's OLAAccumulator restatement, re-expressing the reference's own test
groups (tests/ola_accumulator_test.cc):

  :143-191  construction / invalid configuration / window setting
  :194-437  SoA / AoS, single / multi channel, start offset, empty requests,
            error conditions, reset
  :439-548  AoS == SoA within +-1 ULP over N in {1024, 2048, 4096} x
            H in {N/4, N/2} x C in {1, 2, 4} x {hann, hamming, rect} x
            gain {0.5, 1, 2} -- here additionally bit-exact against the oracle
  :551-635  AoS == SoA edge cases (H = N, H = N/8, impulses)
  :638-905  large frames, extreme hops, memory pressure, produce() larger than
            the ring, real-time streaming
  :1033-1076 gain

Bar: bit-exact with the oracle (same scalar FMA kernels, IEEE division), the
counters (produced_samples, read_pos) equal, the peak meter equal.  The oracle's
OLA is the reference's arithmetic restated (OLAAccumulator.cc is not buildable
here: Highway is absent), pinned by test_oracle_pins.py.
"""
import numpy as np
import pytest

# ---------------------------------------------------------------- helpers


def hann(n):   # ola_accumulator_test.cc:115-121 (double expression, one rounding)
    i = np.arange(n, dtype=np.float64)
    return (0.5 * (1.0 - np.cos(2.0 * np.pi * i / (n - 1)))).astype(np.float32)


def hamming(n):  # :123-129
    i = np.arange(n, dtype=np.float64)
    return (0.54 - 0.46 * np.cos(2.0 * np.pi * i / (n - 1))).astype(np.float32)


def rect(n):
    return np.ones(n, np.float32)


WINDOWS = {"hann": hann, "hamming": hamming, "rectangular": rect}


def cfg(pkg, n=256, h=64, c=1, inside=True, eps=1e-8):
    return pkg.OLAConfig(sample_rate=48000, frame_size=n, hop_size=h, channels=c, eps=eps,
                         apply_window_inside=inside)


def pair(pkg, oracle, n=256, h=64, c=1, inside=True, window=None):
    d = pkg.OLAAccumulator(cfg(pkg, n, h, c, inside))
    o = oracle.Ola(n, h, c, 1e-8, inside)
    if window is not None:
        d.set_window(window)
        o.set_window(window)
    return d, o


def produce_both(d, o, n, c):
    od = [np.zeros(max(n, 1), np.float32) for _ in range(c)]
    oo = [np.zeros(max(n, 1), np.float32) for _ in range(c)]
    gd, _ = d.produce(n, od)
    go = o.produce_into(n, oo)
    assert gd == go
    for a, b in zip(od, oo):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    return gd, od


def same_state(d, o):
    assert d.produced_samples() == o.produced
    assert d.read_pos() == o.read_pos
    assert d.meter_peak() == o.meter_peak


def ulp_equal(a, b, max_ulp=1):
    ia = a.view(np.int32).astype(np.int64)
    ib = b.view(np.int32).astype(np.int64)
    return bool(np.all(((ia ^ ib) >= 0) & (np.abs(ia - ib) <= max_ulp)))


# ---------------------------------------------------------------- CPU: validation


def test_invalid_configuration_raises(pkg):
    """:155-176 (checked before any device call, so this runs without a GPU)."""
    for kw in ({"frame_size": 0}, {"hop_size": 0}, {"channels": 0}, {"eps": 0.0},
               {"sample_rate": 0}):
        c = cfg(pkg)
        for k, v in kw.items():
            setattr(c, k, v)
        assert not c.isValid()
        with pytest.raises(ValueError, match="Invalid OLA configuration"):
            pkg.OLAAccumulator(c)


# ---------------------------------------------------------------- GPU


@pytest.mark.gpu
def test_basic_construction_and_window(torch_cuda, pkg, oracle):
    """:143-153, :178-191."""
    d = pkg.OLAAccumulator(cfg(pkg))
    assert d.config().frame_size == 256 and d.config().hop_size == 64
    assert d.ring_size() == oracle.ring_len(256, 64) > 0
    assert not d.has_window()
    w = np.full(256, 0.5, np.float32)
    d.set_window(w)
    assert d.has_window()
    with pytest.raises(ValueError, match="Window pointer cannot be null"):
        d.set_window(None, 256)
    with pytest.raises(ValueError, match="Window size must match frame size"):
        d.set_window(np.zeros(257, np.float32))
    o = oracle.Ola(256, 64)
    o.set_window(w)
    assert np.array_equal(d.norm(), o.norm())


@pytest.mark.gpu
@pytest.mark.parametrize("c", [1, 2])
def test_soa_aos_single_multi_channel(torch_cuda, pkg, oracle, c):
    """:194-250 (SoA), :334-390 (AoS), :392-437 (AoS vs SoA, EXPECT_FLOAT_EQ)."""
    n = 256
    w = rect(n)
    vals = [0.5, 0.3][:c]
    frames = [np.full(n, v, np.float32) for v in vals]
    aos = np.stack(frames, 1).reshape(-1)
    d1, o1 = pair(pkg, oracle, n, 64, c, window=w)
    d1.add_frame_SoA(frames, w, 0, 0, n, 1.0)
    o1.add_frame_soa(frames, 0, 0, n, 1.0, window=w)
    g1, out_soa = produce_both(d1, o1, n, c)
    assert g1 > 0 and d1.produced_samples() == n and d1.read_pos() == g1
    same_state(d1, o1)
    d2, o2 = pair(pkg, oracle, n, 64, c, window=w)
    d2.push_frame_AoS(aos, w, 0, 0, n, 1.0)
    o2.push_frame_aos(aos, 0, 0, n, 1.0, window=w)
    g2, out_aos = produce_both(d2, o2, n, c)
    same_state(d2, o2)
    for a, b in zip(out_soa, out_aos):
        assert np.array_equal(a, b)


@pytest.mark.gpu
def test_start_offset_and_empty_requests(torch_cuda, pkg, oracle):
    """:252-292."""
    n = 256
    w = rect(n)
    d, o = pair(pkg, oracle, n, 64, 1, window=w)
    f = np.ones(n, np.float32)
    d.add_frame_SoA([f], w, 0, 32, n - 32, 1.0)
    o.add_frame_soa([f], 0, 32, n - 32, 1.0, window=w)
    g, _ = produce_both(d, o, n, 1)
    assert g > 0 and d.produced_samples() == n - 32
    same_state(d, o)
    e = pkg.OLAAccumulator(cfg(pkg))
    e.add_frame_SoA([None], None, 0, 0, 0, 1.0)        # size 0: nothing, no throw
    assert e.produce(0, [None])[0] == 0
    assert e.produced_samples() == 0


@pytest.mark.gpu
def test_error_conditions(torch_cuda, pkg):
    """:294-305, :807-844 (null pointers throw std::invalid_argument)."""
    d = pkg.OLAAccumulator(cfg(pkg))
    with pytest.raises(ValueError, match="Channel frame pointer cannot be null"):
        d.add_frame_SoA([None], None, 0, 0, 1, 1.0)
    with pytest.raises(ValueError, match="Channel frames pointer cannot be null"):
        d.add_frame_SoA(None, None, 0, 0, 1, 1.0)
    with pytest.raises(ValueError, match="Output channel buffer cannot be null"):
        d.produce(1, [None])
    with pytest.raises(ValueError, match="Interleaved input pointer cannot be null"):
        d.push_frame_AoS(None, None, 0, 0, 1, 1.0)


@pytest.mark.gpu
def test_null_second_channel_adds_first_then_throws(torch_cuda, pkg, oracle):
    """OLAAccumulator.cc:74-82: the channel loop adds channel 0, then throws at
    channel 1 and leaves produced_ unchanged -- the ring keeps channel 0's add."""
    n = 256
    w = hann(n)
    d, o = pair(pkg, oracle, n, 64, 2, window=w)
    f = np.linspace(-1, 1, n, dtype=np.float32)
    with pytest.raises(ValueError):
        d.add_frame_SoA([f, None], None, 0, 0, n, 1.0)
    assert d.produced_samples() == 0
    # an add of zeros that sets produced_ exposes the ring: channel 0 holds f*w
    z = np.zeros(n, np.float32)
    d.add_frame_SoA([z, z], None, 0, 0, n, 1.0)
    o1 = oracle.Ola(n, 64, 1)
    o1.set_window(w)
    o1.add_frame_soa([f], 0, 0, n, 1.0)
    o1.add_frame_soa([z], 0, 0, n, 1.0)
    got, out = d.produce(n)
    ref = o1.produce(n)[0]
    assert got == n and np.array_equal(out[0][:n], ref) and not out[1][:n].any()


@pytest.mark.gpu
def test_reset(torch_cuda, pkg, oracle):
    """:307-332."""
    n = 256
    w = rect(n)
    d, o = pair(pkg, oracle, n, 64, 1, window=w)
    f = np.full(n, 0.5, np.float32)
    d.add_frame_SoA([f], w, 0, 0, n, 1.0)
    o.add_frame_soa([f], 0, 0, n, 1.0, window=w)
    produce_both(d, o, n, 1)
    assert d.meter_peak() > 0
    d.reset()
    o.reset()
    assert d.produced_samples() == 0 and d.read_pos() == 0
    assert d.meter_peak() == 0.0 and not d.has_window()
    assert np.array_equal(d.norm(), o.norm()) and np.all(d.norm() == 1.0)
    # after reset: no window, ring cleared -> the next frame is added unwindowed
    d.add_frame_SoA([f], None, 0, 0, n, 1.0)
    o.add_frame_soa([f], 0, 0, n, 1.0)
    produce_both(d, o, n, 1)
    same_state(d, o)


@pytest.mark.gpu
def test_aos_soa_equivalence_grid(torch_cuda, pkg, oracle):
    """:439-548: N x H x C x window x gain, AoS == SoA (+-1 ULP in the
    reference; here bit-exact, and both bit-exact against the oracle)."""
    rng = np.random.default_rng(439)
    n_cases = 0
    for n in (1024, 2048, 4096):
        for ratio in (4, 2):
            h = n // ratio
            for c in (1, 2, 4):
                for wname, wf in WINDOWS.items():
                    w = wf(n)
                    for gain in (0.5, 1.0, 2.0):
                        tf = rng.uniform(-1, 1, n * c).astype(np.float32)
                        soa = [tf[ch * n:(ch + 1) * n] for ch in range(c)]
                        aos = np.stack(soa, 1).reshape(-1)
                        da, oa = pair(pkg, oracle, n, h, c, window=w)
                        ds, _ = pair(pkg, oracle, n, h, c, window=w)
                        da.push_frame_AoS(aos, w, 0, 0, n, gain)
                        ds.add_frame_SoA(soa, w, 0, 0, n, gain)
                        oa.push_frame_aos(aos, 0, 0, n, gain, window=w)
                        ga, outa = produce_both(da, oa, n, c)
                        gs, outs = ds.produce(n)
                        assert ga == gs == n
                        for a, b in zip(outa, outs):
                            assert ulp_equal(a[:n], b[:n], 1), (n, h, c, wname, gain)
                            assert np.array_equal(a[:n], b[:n])
                        n_cases += 1
    assert n_cases == 162


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,c", [(1024, 1024, 1), (2048, 256, 2), (4096, 512, 4), (960, 240, 2), (882, 441, 3)])
def test_aos_soa_edge_cases(torch_cuda, pkg, oracle, n, h, c):
    """:551-635: impulse on channel 0, H = N and H = N/8."""
    w = hann(n)
    tf = np.zeros(n * c, np.float32)
    tf[0] = 1.0
    soa = [tf[ch * n:(ch + 1) * n] for ch in range(c)]
    aos = np.stack(soa, 1).reshape(-1)
    da, oa = pair(pkg, oracle, n, h, c, window=w)
    ds, os_ = pair(pkg, oracle, n, h, c, window=w)
    da.push_frame_AoS(aos, w, 0, 0, n, 1.0)
    oa.push_frame_aos(aos, 0, 0, n, 1.0, window=w)
    ds.add_frame_SoA(soa, w, 0, 0, n, 1.0)
    os_.add_frame_soa(soa, 0, 0, n, 1.0, window=w)
    ga, outa = produce_both(da, oa, n, c)
    gs, outs = produce_both(ds, os_, n, c)
    assert ga == gs == n
    for a, b in zip(outa, outs):
        assert ulp_equal(a[:n], b[:n], 1)


@pytest.mark.gpu
def test_large_frames_and_extreme_hops(torch_cuda, pkg, oracle):
    """:638-738: N in {4096, 8192} at H = N/4; N = 2048, C = 2, H in {N, N/8}
    (H = N reconstructs the input within 1e-6)."""
    for n in (4096, 8192):
        w = hann(n)
        d, o = pair(pkg, oracle, n, n // 4, 1, window=w)
        f = np.full(n, 0.1, np.float32)
        d.add_frame_SoA([f], w, 0, 0, n, 1.0)
        o.add_frame_soa([f], 0, 0, n, 1.0, window=w)
        g, out = produce_both(d, o, n, 1)
        assert g == n and d.produced_samples() == n and np.all(np.isfinite(out[0]))
    n = 2048
    w = hamming(n)
    for h in (n, n // 8):
        d, o = pair(pkg, oracle, n, h, 2, window=w)
        f0, f1 = np.full(n, 0.5, np.float32), np.full(n, -0.3, np.float32)
        d.add_frame_SoA([f0, f1], w, 0, 0, n, 1.0)
        o.add_frame_soa([f0, f1], 0, 0, n, 1.0, window=w)
        g, out = produce_both(d, o, n, 2)
        assert g == n and all(np.all(np.isfinite(x)) for x in out)
        if h == n:
            assert np.allclose(out[0], f0, atol=1e-6) and np.allclose(out[1], f1, atol=1e-6)


@pytest.mark.gpu
def test_memory_pressure_sequence(torch_cuda, pkg, oracle):
    """:740-805: 100 frames x 4 channels at 4096/512, produce(N) every 10th
    frame (the ring wraps), then a final produce -- every output bit-exact."""
    n, h, c = 4096, 512, 4
    w = hann(n)
    d, o = pair(pkg, oracle, n, h, c, window=w)
    for k in range(100):
        fr = [np.full(n, k / 100.0, np.float32) for _ in range(c)]
        d.add_frame_SoA(fr, w, k * h, 0, n, 1.0)
        o.add_frame_soa(fr, k * h, 0, n, 1.0, window=w)
        if k % 10 == 0:
            g, _ = produce_both(d, o, n, c)
            assert g > 0
    g, _ = produce_both(d, o, n, c)
    assert g > 0
    same_state(d, o)


@pytest.mark.gpu
def test_produce_larger_than_ring(torch_cuda, pkg, oracle):
    """:807-844: produce(10 N) asks for more than the ring holds: split() clamps
    the work to ring_len while the count and read_pos advance by the request
    (OLAAccumulator.cc:195-213, ring_buffer.cc:55-58); the caller's buffer tail
    stays as it was, and the peak meter reads it."""
    n, h = 1024, 256
    w = hann(n)
    d, o = pair(pkg, oracle, n, h, 1, window=w)
    f = np.ones(n, np.float32)
    d.add_frame_SoA([f], w, 0, 0, n, 1.0)
    o.add_frame_soa([f], 0, 0, n, 1.0, window=w)
    d.flush()
    o.flush()
    d.add_frame_SoA([f], w, 20 * n, 0, n, 1.0)   # produced_ far beyond the ring
    o.add_frame_soa([f], 20 * n, 0, n, 1.0, window=w)
    big = 10 * n
    tail = np.linspace(-3, 3, big, dtype=np.float32)
    od, oo = [tail.copy()], [tail.copy()]
    gd, _ = d.produce(big, od)
    go = o.produce_into(big, oo)
    assert gd == go == big
    assert np.array_equal(od[0], oo[0])
    assert np.array_equal(od[0][d.ring_size():], tail[d.ring_size():])
    same_state(d, o)


@pytest.mark.gpu
def test_realtime_streaming_sequence(torch_cuda, pkg, oracle):
    """:846-905: 50 iterations of add(frame at iter*H) then produce(H), C = 2."""
    n, h, c = 512, 128, 2
    w = hann(n)
    d, o = pair(pkg, oracle, n, h, c, window=w)
    total = 0
    for it in range(50):
        fr = [np.full(n, np.sin(np.float32(it * 0.1)), np.float32),
              np.full(n, np.cos(np.float32(it * 0.1)), np.float32)]
        d.add_frame_SoA(fr, w, it * h, 0, n, 1.0)
        o.add_frame_soa(fr, it * h, 0, n, 1.0, window=w)
        g, out = produce_both(d, o, h, c)
        total += g
        if it > 5:
            assert 0 < g <= 2 * h
        assert all(np.all(np.isfinite(x[:g])) for x in out)
    assert 0 < total <= 2 * 50 * h
    same_state(d, o)


@pytest.mark.gpu
def test_gain(torch_cuda, pkg, oracle):
    """:1033-1076: impulse with gain g; first output = impulse * w[0] * g."""
    n, h = 2048, 512
    w = hann(n)
    for gain in (0.1, 0.5, 1.0, 2.0, 10.0):
        d, o = pair(pkg, oracle, n, h, 1, window=w)
        imp = np.zeros(n, np.float32)
        imp[0] = 1.0
        d.add_frame_SoA([imp], w, 0, 0, n, gain)
        o.add_frame_soa([imp], 0, 0, n, gain, window=w)
        g, out = produce_both(d, o, n, 1)
        assert g > 0 and abs(out[0][0] - imp[0] * w[0] * gain) <= 1e-6


@pytest.mark.gpu
def test_external_window_and_aos_window_offset(torch_cuda, pkg, oracle):
    """apply_window_inside = false: the caller's window is used (and the norm is
    all ones); push_frame_AoS with start_off > 0 reads that window from index 0
    (it calls add_frame_SoA with start_off = 0, OLAAccumulator.cc:146-159),
    add_frame_SoA from start_off."""
    n, h, c = 512, 128, 2
    w = hann(n)
    rng = np.random.default_rng(5)
    d, o = pair(pkg, oracle, n, h, c, inside=False)
    assert np.all(d.norm() == 1.0)
    for k in range(6):
        aos = rng.uniform(-1, 1, n * c).astype(np.float32)
        soa = [rng.uniform(-1, 1, n).astype(np.float32) for _ in range(c)]
        off = [0, 37, 100][k % 3]
        d.push_frame_AoS(aos, w, k * h, off, n - off, 0.75)
        o.push_frame_aos(aos, k * h, off, n - off, 0.75, window=w)
        d.add_frame_SoA(soa, w if k % 2 else None, k * h + 3, off, n, 1.25)
        o.add_frame_soa(soa, k * h + 3, off, n, 1.25, window=w if k % 2 else None)
        produce_both(d, o, h, c)
    same_state(d, o)


@pytest.mark.gpu
def test_random_call_sequences_match_oracle(torch_cuda, pkg, oracle):
    """Differential fuzz of whole call sequences: random adds (SoA / AoS,
    start_sample / start_off / size / gain / window), produce(n) of random n,
    flush, reset, set_window -- outputs, counters and the peak meter bit-exact."""
    rng = np.random.default_rng(2024)
    for trial in range(6):
        n = int(rng.choice([64, 256, 1000, 1024]))
        h = int(rng.choice([n // 4, n // 2, n, max(1, n // 3)]))
        c = int(rng.choice([1, 2, 3]))
        inside = bool(rng.integers(0, 2))
        d, o = pair(pkg, oracle, n, h, c, inside=inside, window=hann(n) if rng.integers(0, 2) else None)
        pos = 0
        for step in range(60):
            op = rng.integers(0, 10)
            if op < 5:
                off = int(rng.integers(0, n + 2)) if rng.random() < 0.3 else 0
                size = int(rng.integers(0, n + 5)) if rng.random() < 0.3 else n
                gain = float(np.float32(rng.choice([1.0, 0.5, rng.uniform(-2, 2)])))
                win = hamming(n) if rng.random() < 0.5 else None
                if rng.random() < 0.5:
                    fr = [rng.uniform(-1, 1, n).astype(np.float32) for _ in range(c)]
                    d.add_frame_SoA(fr, win, pos, off, size, gain)
                    o.add_frame_soa(fr, pos, off, size, gain, window=win)
                else:
                    a = rng.uniform(-1, 1, n * c).astype(np.float32)
                    d.push_frame_AoS(a, win, pos, off, size, gain)
                    o.push_frame_aos(a, pos, off, size, gain, window=win)
                pos += int(rng.choice([h, h, 0, 2 * h]))
            elif op < 8:
                produce_both(d, o, int(rng.choice([h, 1, n, 3 * h + 1])), c)
            elif op == 8:
                d.flush()
                o.flush()
            else:
                if rng.random() < 0.3:
                    d.reset()
                    o.reset()
                    pos = 0
                else:
                    w = hann(n) * np.float32(rng.uniform(0.5, 1.5))
                    d.set_window(w)
                    o.set_window(w)
            assert d.produced_samples() == o.produced and d.read_pos() == o.read_pos
        same_state(d, o)


@pytest.mark.gpu
def test_device_forms_match_host_forms(torch_cuda, pkg, oracle):
    """push_frame_AoS_device / add_frame_SoA_device / produce_device on HBM
    tensors equal the oracle; mixing them with host-pointer calls keeps order."""
    torch = torch_cuda
    n, h, c = 1024, 256, 2
    w = hann(n)
    rng = np.random.default_rng(9)
    d, o = pair(pkg, oracle, n, h, c, window=w)
    out = torch.zeros((c, 3 * h), dtype=torch.float32, device="cuda:0")
    for k in range(12):
        a = rng.uniform(-1, 1, n * c).astype(np.float32)
        if k % 3 == 0:
            d.push_frame_AoS(a, None, k * h, 0, n, 1.0)
        elif k % 3 == 1:
            d.push_frame_AoS_device(torch.from_numpy(a).cuda(), None, k * h, 0, n, 1.0)
        else:
            soa = torch.from_numpy(a.reshape(n, c).T.copy()).cuda()
            d.add_frame_SoA_device(soa, None, k * h, 0, n, 1.0)
        o.push_frame_aos(a, k * h, 0, n, 1.0)
        if k % 2:
            g = d.produce_device(out, h)
            ref = o.produce(h)
            got = out.cpu().numpy()
            assert g == len(ref[0])
            for ch in range(c):
                assert np.array_equal(got[ch, :g], ref[ch])
        else:
            produce_both(d, o, h, c)
    same_state(d, o)
