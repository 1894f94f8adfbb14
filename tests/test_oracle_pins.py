"""Pin the oracle (CPU restatement) before trusting it.

1. bit-exact against the reference's own compiled WindowLUT.cc / norm_builder.cc /
   framer.cc / FrameQueue.cc outputs and its OLA primitives -- the scalar kernels
   of kernels.cc, RingBuffer::split (ring_buffer.cc) and deinterleave_to_scratch
   (aos_to_soa.cc) -- (tests/golden/ref_tables.npz, via oracle/_ref/ref_dump);
2. kissfft restatement bit-exact against an independent kissfft build
   (tests/golden/kiss_gst.npz);
3. the reference's own known-answer tests, re-expressed:
   tests/fft_test.cc, tests/norm_builder_test.cc, tests/kernels_test.cc,
   tests/ola_accumulator_test.cc, tests/framer_test.cc.
"""
import re

import numpy as np
import pytest

TYPES = {"hann": 0, "hamming": 1, "blackman": 2, "rect": 3}


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


# ----------------------------------------------------------------- vs reference build
def test_windows_bit_exact_vs_reference(oracle, ref_tables):
    n_checked = 0
    for key in ref_tables.files:
        m = re.match(r"window_(\w+?)_p(\d)_n(\d+)_norm(\d)$", key)
        if not m:
            continue
        t, per, n, nm = TYPES[m[1]], int(m[2]), int(m[3]), int(m[4])
        w = oracle.window(t, n, bool(per), nm)
        assert np.array_equal(bits(w), bits(ref_tables[key])), key
        n_checked += 1
    assert n_checked >= 100
    # GetWindowSafe path == ctor path (e2e_benchmark.cc:51-53)
    assert np.array_equal(bits(ref_tables["window_getsafe_hann_1024"]),
                          bits(oracle.window(0, 1024)))


def test_norm_tables_bit_exact_vs_reference(oracle, ref_tables):
    n_checked = 0
    for key in ref_tables.files:
        m = re.match(r"norm_hann_p(\d)_n(\d+)_h(\d+)_r(\d+)$", key)
        if not m:
            continue
        per, n, h, r = (int(v) for v in m.groups())
        assert oracle.ring_len(n, h) == r  # calculate_ring_size
        w = oracle.window(0, n, bool(per))
        got = np.zeros(r, np.float32)
        oracle.lib().or_build_norm_linear(got, w, r, n, h)
        assert np.array_equal(bits(got), bits(ref_tables[key])), key
        n_checked += 1
    assert n_checked == 16


def test_norm_quirk_q1_nonuniform(ref_tables):
    """the norm sums w (not w^2) over more frame starts than the ring holds."""
    t = ref_tables["norm_hann_p1_n1024_h256_r6144"]
    slots = t[::256]
    assert slots[0] == pytest.approx(4.0, abs=1e-4)
    assert slots[10] == pytest.approx(2.0, abs=1e-4)
    assert len(set(np.round(slots, 4))) > 3


def _framer_case(tag):
    if tag.startswith("ramp20_n8_h2"):
        x = np.arange(1, 21, dtype=np.float32)
        return x, 20, 1, 8, 2, int(tag.split("_c")[-1])
    if tag.startswith("ramp20_st"):
        return np.arange(1, 21, dtype=np.float32), 10, 2, 4, 2, 0
    if tag.startswith("edge_t"):
        T = int(re.match(r"edge_t(\d+)", tag)[1])
        x = (np.arange(T) % 1000).astype(np.float32) / np.float32(1024) - np.float32(0.5)
        return x, T, 1, 1024, 256, 0
    x = np.arange(3000, dtype=np.float32)
    if tag.startswith("n512_h128"):
        return x, 3000, 1, 512, 128, 128
    return x, 1000, 1, 100, 30, 0


def test_framer_bit_exact_vs_reference(oracle, ref_tables):
    n = 0
    for key in ref_tables.files:
        if not key.startswith("framer_") or key.endswith("_avail"):
            continue
        tag = key[len("framer_"):]
        mode = oracle.DROP if tag.endswith("_drop") or "_drop_" in tag else oracle.ZERO_PAD
        x, T, C, N, H, chunk = _framer_case(tag)
        fr, av = oracle.framer_run(x, T, C, N, H, mode, chunk)
        assert np.array_equal(fr, ref_tables[key]), tag
        assert np.array_equal(av, ref_tables[key + "_avail"]), tag
        n += 1
    assert n == 26


def test_framer_counts_match_formula(oracle, ref_tables):
    """ZERO_PAD whole push: ceil(T/H) frames; DROP: floor((T-N)/H)+1 (framer_test.cc:299-321)."""
    for T in (1, 255, 1023, 1024, 1025, 4173):
        for mode, tag in ((oracle.ZERO_PAD, "zpad"), (oracle.DROP, "drop")):
            fr = ref_tables[f"framer_edge_t{T}_{tag}"]
            assert fr.size // 1024 == oracle.frame_count(T, 1024, 256, mode)


# ----------------------------------------------------------------- FrameQueue
def _fq_cases(ref_tables):
    for key in sorted(ref_tables.files):
        if key.startswith("fq_") and key.endswith("_meta"):
            base = key[:-5]
            T, N, H, c, m, F = (int(v) for v in ref_tables[key])
            yield base, T, N, H, c, m, F


def test_framequeue_bit_exact_vs_reference(oracle, ref_tables):
    """FrameQueue.cc / Indexing.h restatement vs the reference's own FrameQueue
    (ref_dump): frame counts and every frame value, all pad modes, centre on/off,
    signals shorter than the pad (multi-bounce reflect101), T = 0."""
    n = 0
    for base, T, N, H, c, m, F in _fq_cases(ref_tables):
        x = ref_tables[base + "_x"]
        assert oracle.fq_count(T, N, H, bool(c)) == F, base
        got = oracle.fq_frames(x, N, H, bool(c), m)
        assert np.array_equal(got.reshape(-1), ref_tables[base + "_frames"]), base
        n += 1
    assert n == 48


def test_ola_kernels_bit_exact_vs_reference(oracle, ref_tables):
    """axpy_scalar / axpy_windowed_scalar / normalize_and_clear_scalar
    (kernels.cc:18-36), compiled from the reference unchanged, against the
    oracle's or_axpy / or_axpy_windowed / or_normalize_and_clear on the same
    seeded data (mt19937(42) U(-10, 10) as kernels_test.cc:219; norms on both
    sides of the eps guard)."""
    n_checked = 0
    for key in ref_tables.files:
        m = re.match(r"(k_n\d+_g\d)_dst$", key)
        if not m:
            continue
        k = m[1]
        dst, src, win = (ref_tables[f"{k}_{s}"] for s in ("dst", "src", "win"))
        g = float(ref_tables[f"{k}_gain"][0])
        assert np.array_equal(bits(oracle.axpy(dst, src, g)), bits(ref_tables[f"{k}_axpy"])), k
        assert np.array_equal(bits(oracle.axpy(dst, src, g, win)), bits(ref_tables[f"{k}_axpyw"])), k
        out, acc = oracle.normalize_and_clear(dst, ref_tables[f"{k}_norm"], float(ref_tables[f"{k}_eps"][0]))
        assert np.array_equal(bits(out), bits(ref_tables[f"{k}_out"])), k
        assert np.array_equal(bits(acc), bits(ref_tables[f"{k}_acc"])), k
        n_checked += 1
    assert n_checked == 28


def test_ring_split_vs_reference(oracle, ref_tables):
    """RingBuffer::split (ring_buffer.cc:44-85): start mod capacity, length
    clamped to the capacity, at most two spans -- the oracle's ring_split, which
    its add_frame_SoA / produce use, gives the same spans for every case."""
    rows = ref_tables["ring_split_rows"].reshape(-1, 7).astype(np.int64)
    assert len(rows) == 5 * 7 * 7
    for cap, start, length, o1, l1, o2, l2 in rows:
        s1, m1, m2 = oracle.ring_split(int(cap), int(start), int(length))
        assert (m1, m2) == (l1, l2), (cap, start, length)
        if l1:
            assert s1 == o1, (cap, start, length)
        assert o2 == 0  # the second span always starts at the ring's origin


def test_deinterleave_vs_reference(oracle, ref_tables):
    """deinterleave_to_scratch (aos_to_soa.cc:7-18), push_frame_AoS's first step."""
    for c in (1, 2, 3, 5, 16):
        x = ref_tables[f"deint_c{c}_x"]
        assert np.array_equal(bits(oracle.deinterleave(x, x.size // c, c)), bits(ref_tables[f"deint_c{c}_s"])), c


def test_reflect101_is_the_reference_mixed_rule(oracle):
    """Indexing.h:18-37 as written: the left side reflects about -1/2 (-1 -> 0),
    the right side about n-1 (n -> n-2); the doc comment's example differs."""
    L = oracle.lib()
    assert [L.or_fq_reflect101(i, 4) for i in range(-4, 8)] == [3, 2, 1, 0, 0, 1, 2, 3, 2, 1, 0, 0]
    assert L.or_fq_reflect101(-9, 1) == 0 and L.or_fq_reflect101(5, 0) == 0


def test_framequeue_golden_reproduces(oracle, fq_gold):
    names = sorted({k.split("/")[0] for k in fq_gold.files})
    for name in names:
        n, h, c, pm, aw, S, T = (int(v) for v in fq_gold[f"{name}/meta"])
        x = fq_gold[f"{name}/x"]
        for s in range(S):
            y, fr = oracle.roundtrip_ex(x[s], n, h, mode=oracle.FRAMEQUEUE, center=bool(c),
                                        pad_mode=pm, analysis_window=bool(aw), want_frames=True)
            assert np.array_equal(y, fq_gold[f"{name}/y"][s]), name
            assert np.array_equal(fr, fq_gold[f"{name}/frames"][s]), name


# ----------------------------------------------------------------- kissfft
def test_kissfft_bit_exact_vs_independent_build(oracle, kiss_gst):
    for key in kiss_gst.files:
        if not key.startswith("x_"):
            continue
        n = int(key[2:])
        k = oracle.KissR(n)
        X = k.rfft_raw(kiss_gst[f"x_{n}"])
        assert np.array_equal(bits(X.view(np.float32)), bits(kiss_gst[f"X_{n}"])), n
        y = k.irfft_raw(kiss_gst[f"Y_{n}"].view(np.complex64))
        assert np.array_equal(bits(y), bits(kiss_gst[f"y_{n}"])), n


@pytest.mark.parametrize("n", [8, 12, 30, 64, 96, 512, 1000, 1024, 4096])
def test_kissfft_vs_float64_dft(oracle, n):
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n).astype(np.float32)
    X = oracle.KissR(n).rfft_raw(x)
    ref = np.fft.rfft(x.astype(np.float64))
    assert np.linalg.norm(X - ref) / np.linalg.norm(ref) < 3e-7
    z = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
    Z = oracle.KissC(n).forward(z)
    refz = np.fft.fft(z.astype(np.complex128))
    assert np.linalg.norm(Z - refz) / np.linalg.norm(refz) < 3e-7


# fft_test.cc:57-129 round trip
@pytest.mark.parametrize("n,f", [(512, 10), (1024, 20), (2048, 40)])
def test_ref_fft_roundtrip_rms(oracle, n, f):
    t = np.arange(n, dtype=np.float32) / np.float32(n)
    x = np.sin(np.float32(2 * np.pi) * np.float32(f / n) * np.float32(n) * t).astype(np.float32)
    k = oracle.KissR(n)
    y = k.inverse(k.forward(x))
    assert np.sqrt(np.mean((x - y) ** 2)) < 1e-5


# fft_test.cc:131-197, 344-381 known answers
def test_ref_fft_known_answers(oracle):
    k = oracle.KissR(512)
    X = k.forward(np.ones(512, np.float32))
    assert abs(abs(X[0]) - 512) < 1e-3 and abs(np.angle(X[0])) < 1e-3
    assert np.all(np.abs(X[1:]) < 1e-3)
    k = oracle.KissR(1024)
    t = np.arange(1024, dtype=np.float32) / np.float32(1024)
    x = (2 * np.cos(2 * np.pi * 10 * t)).astype(np.float32)
    X = k.forward(x)
    assert abs(abs(X[10]) - 1024) < 1e-3 * 1024 and abs(np.angle(X[10])) < 1e-3
    assert abs(X[0]) < 1e-3 and abs(X[512]) < 1e-3
    ny = np.where(np.arange(1024) % 2 == 0, 1.0, -1.0).astype(np.float32)
    X = k.forward(ny)
    assert abs(X[512]) > 500 and abs(X[0]) < 1e-3


# fft_test.cc:199-221 NaN / Inf / denormal
def test_ref_fft_sanitize(oracle):
    k = oracle.KissR(512)
    x = np.zeros(512, np.float32)
    x[0], x[1], x[2] = np.nan, 1e-40, np.inf
    y = k.inverse(k.forward(x))
    assert np.all(np.isfinite(y))


# fft_test.cc:251-288 complex round trip
def test_ref_complex_roundtrip(oracle):
    n = 256
    t = np.arange(n, dtype=np.float32) / np.float32(n)
    z = (np.cos(2 * np.pi * 10 * t) + 1j * np.sin(2 * np.pi * 10 * t)).astype(np.complex64)
    k = oracle.KissC(n)
    back = k.inverse(k.forward(z))
    assert np.max(np.abs(back - z)) < 1e-5


# ----------------------------------------------------------------- norm builder
def _norm_scalar(window, ring_len, n, h):
    """norm_builder_test.cc:13-53 scalar triple loop (float accumulation, max 1e-8)."""
    out = np.zeros(ring_len, np.float32)
    kmin = -int(np.ceil(n / h))
    kmax = int(np.ceil((ring_len + n - 1) / h))
    for pos in range(ring_len):
        acc = np.float32(0)
        for fo in range(kmin, kmax + 1):
            st = fo * h
            for t in range(n):
                if (st + t) % ring_len == pos:
                    acc = np.float32(acc + window[t])
        out[pos] = max(acc, np.float32(1e-8))
    return out


def test_ref_norm_builder_grid(ref_tables):
    """norm_builder_test.cc:87-128: linear == scalar within 1e-5 on the reference's grid."""
    for key in ref_tables.files:
        m = re.match(r"normgrid_n(\d+)_h(\d+)_r(\d+)$", key)
        if not m:
            continue
        n, h, r = (int(v) for v in m.groups())
        if n * r > 300_000:  # keep the pure-Python loop small
            continue
        w = ref_tables[f"window_hann_p0_n{n}_norm0"] if f"window_hann_p0_n{n}_norm0" in ref_tables.files else None
        if w is None:
            w = (0.5 * (1 - np.cos(2 * np.pi * np.arange(n) / (n - 1)))).astype(np.float32)
        assert np.max(np.abs(_norm_scalar(w, r, n, h) - ref_tables[key])) < 1e-5


# ----------------------------------------------------------------- OLA kernels / accumulator
def test_ref_kernels_values(oracle):
    """kernels_test.cc:67-207 axpy / axpy_windowed / normalize_and_clear."""
    L = oracle.lib()
    import ctypes as C
    f = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
    L.or_axpy_windowed.argtypes = [f, f, f, C.c_float, C.c_size_t]
    L.or_normalize_and_clear.argtypes = [f, f, f, C.c_float, C.c_size_t]
    rng = np.random.default_rng(42)
    for n in (0, 1, 7, 8, 15, 16, 31, 64, 1023, 4096):
        d = rng.uniform(-10, 10, n).astype(np.float32)
        s = rng.uniform(-10, 10, n).astype(np.float32)
        w = rng.uniform(0, 1, n).astype(np.float32)
        exp = (d.astype(np.float64) + (s * w).astype(np.float64) * 0.5).astype(np.float32)
        L.or_axpy_windowed(d, s, w, 0.5, n)
        assert np.all(np.abs(d - exp) <= np.abs(exp) * 2.4e-7 + 1e-30)
        acc = rng.uniform(-10, 10, n).astype(np.float32)
        nm = rng.uniform(-1, 2, n).astype(np.float32)
        out = np.zeros(n, np.float32)
        exp = acc / np.maximum(nm, np.float32(1e-8))
        L.or_normalize_and_clear(out, acc, nm, 1e-8, n)
        assert np.array_equal(out, exp) and not acc.any()


def test_ref_ola_h_equals_n_reconstruction(oracle):
    """ola_accumulator_test.cc:681-737: H == N with the window inside reconstructs the frame."""
    n = 2048
    w = (0.54 - 0.46 * np.cos(2 * np.pi * np.arange(n) / (n - 1))).astype(np.float32)
    ola = oracle.Ola(n, n, 1, 1e-8, True)
    ola.set_window(w)
    fr = np.full(n, 0.5, np.float32)
    ola.push_frame_aos(fr, 0)
    (y,) = ola.produce(n)
    assert y.size == n and np.max(np.abs(y - 0.5)) < 1e-6


def test_ref_ola_streaming_semantics(oracle):
    """ola_accumulator_test.cc:846-904: produce(H) after every push; no NaN; ring size."""
    n, h = 512, 128
    ola = oracle.Ola(n, h, 2, 1e-8, True)
    assert ola.ring_size == (4 + 20) * 128
    w = oracle.window(0, n)
    ola.set_window(w)
    tot = 0
    for it in range(50):
        fr = np.stack([np.full(n, np.sin(it * 0.1), np.float32),
                       np.full(n, np.cos(it * 0.1), np.float32)], 1).reshape(-1)
        ola.push_frame_aos(fr, it * h)
        outs = ola.produce(h)
        assert outs[0].size == h
        assert np.all(np.isfinite(outs[0])) and np.all(np.isfinite(outs[1]))
        tot += outs[0].size
    assert tot == 50 * h


def test_oracle_roundtrip_equals_batch_formula(oracle):
    """The streaming-interleaved object walk == the closed-form batch formula."""
    n, h, T = 1024, 256, 5000
    x = oracle.synth(T, 3)
    y, frames = oracle.roundtrip(x, n, h, want_frames=True)
    w = oracle.window(0, n)
    nt = oracle.norm_table(w, n, h)
    F = frames.shape[0]
    acc = np.zeros(F * h + n, np.float32)
    for k in range(F):
        a = (frames[k] * w).astype(np.float32)
        acc[k * h:k * h + n] = (acc[k * h:k * h + n] + a).astype(np.float32)
    den = np.maximum(nt, np.float32(1e-8))
    yy = acc[:F * h] / den[np.arange(F * h) % nt.size]
    assert np.array_equal(bits(yy), bits(y))


def test_oracle_q2_double_window_snr(oracle):
    """analysis window + inside window, normalised by sum(w): ~7 dB vs the input."""
    n, h, T = 1024, 256, 48000
    x = oracle.synth(T, 11)
    y = oracle.roundtrip(x, n, h)[:T]
    snr = 10 * np.log10(np.sum(x.astype(np.float64) ** 2) / np.sum((x - y).astype(np.float64) ** 2))
    assert 3.0 < snr < 12.0


def test_oracle_batch_threads_match_single(oracle):
    x = oracle.synth_streams(5, 3000, config_id=9)
    y1 = oracle.roundtrip_batch(x, 1024, 256, nthreads=1)
    y3 = oracle.roundtrip_batch(x, 1024, 256, nthreads=3)
    assert np.array_equal(y1, y3)
    assert np.array_equal(y1[2], oracle.roundtrip(x[2], 1024, 256))


def test_e2e_golden_reproduces(oracle, e2e_gold):
    """The committed end-to-end vectors are reproducible by the pinned oracle."""
    names = sorted({k.split("/")[0] for k in e2e_gold.files})
    for name in names:
        n, h, mode, S, T = (int(v) for v in e2e_gold[f"{name}/meta"])
        x = e2e_gold[f"{name}/x"]
        for s in range(S):
            y = oracle.roundtrip(x[s], n, h, mode=mode)
            assert np.array_equal(bits(y), bits(e2e_gold[f"{name}/y"][s])), name


@pytest.mark.parametrize("n,h,mode", [(1024, 256, 0), (4096, 1024, 1), (512, 128, 2), (960, 240, 0)])
def test_oracle_spectral_step_reduces_to_pinned_loops(oracle, n, h, mode):
    """or_roundtrip_mask (the checker of crlot_stft / crlot_istft_ola / the masked
    round trip) on the pinned loops: a mask of ones is or_roundtrip_ex, mask rows
    equal to one gain are or_roundtrip_gain (ZERO_PAD), and its raw spectra are
    IFftPlan::forward (the adapter restatement) of the windowed frames."""
    T = 7 * n + 33
    x = oracle.synth(T, 5 + n)
    F = oracle.frames_for(T, n, h, mode)
    bins = n // 2 + 1
    y0 = oracle.roundtrip_ex(x, n, h, mode=mode)
    y1, spec = oracle.roundtrip_mask(x, n, h, mask=np.ones((F, bins), np.float32), mode=mode, want_spec=True)
    assert np.array_equal(bits(y0), bits(y1))
    w = oracle.window(oracle.HANN, n)
    if mode == oracle.FRAMEQUEUE:
        fr = oracle.fq_frames(x, n, h).reshape(-1, n)
    else:
        fr = np.zeros((F, n), np.float32)
        for k in range(F):
            seg = x[k * h:k * h + n]
            fr[k, :seg.size] = seg
    direct = oracle.bench_rfft((fr * w).astype(np.float32), n)
    assert np.array_equal(bits(spec.view(np.float32)), bits(direct.view(np.float32)))
    if mode == oracle.ZERO_PAD:
        g = np.linspace(0.25, 1.75, bins).astype(np.float32)
        yg = oracle.roundtrip_gain(x, n, h, g)
        assert np.array_equal(bits(yg), bits(oracle.roundtrip_mask(x, n, h, bin_gain=g)))
        assert np.array_equal(bits(yg), bits(oracle.roundtrip_mask(x, n, h, mask=np.tile(g, (F, 1)))))


def test_oracle_harness_order_loop_replays_the_objects(oracle):
    """or_roundtrip_harness_order (bench.py's CPU leg for e2e_benchmark.cc:152-179's
    literal order) equals the oracle's Framer / kissfft adapter / OLAAccumulator
    objects driven call by call in that order: every push, then produce(T - got)
    until it returns 0 -- ring aliasing and the clamped first read included."""
    n, h = 1024, 256
    x = oracle.synth(12_000, 5)
    T = x.size
    y = oracle.roundtrip_harness_order(x, n, h)
    w = oracle.window(oracle.HANN, n)
    fr, _ = oracle.framer_run(x, T, 1, n, h, oracle.ZERO_PAD)
    kr = oracle.KissR(n)
    ola = oracle.Ola(n, h, 1, eps=1e-8, inside=True)
    ola.set_window(w)
    for k, f in enumerate(fr.reshape(-1, n)):
        ola.push_frame_aos(kr.inverse(kr.forward(f * w)), k * h, 0, n, 1.0)
    out = np.zeros(T, np.float32)
    got = 0
    while got < T:
        buf = np.zeros(T - got, np.float32)
        s = ola.produce_into(T - got, [buf])
        if s == 0:
            break
        out[got:got + s] = buf[:s]
        got += s
    assert y.size == got
    assert np.array_equal(y.view(np.uint32), out[:got].view(np.uint32))
