"""The round trip split at its spectral step: crlot_stft,
crlot_istft_ola and the per-frame spectral mask, through the C ABI.

The reference leaves the step as the identity (bench/e2e_benchmark.cc:160-162);
the oracle applies the same edit in its e2e loop (oracle/crlot_oracle.c
or_roundtrip_mask: kissfft_adapter.cc forward -> spectrum * gain * mask row k ->
inverse -> OLAAccumulator push / produce), so the masked results are pinned to
the oracle's restatement of the reference chain ("parity unpinned" for the edit
itself: the reference has no non-identity step).

Bars (tests/test_gpu_parity.py):
  * spectra and outputs vs the oracle: the float32 FFT tolerance
    (rel-L2 <= 1e-6, max-abs <= 4e-6 of the input / spectrum scale);
  * bit-exact: crlot_stft vs crlot_rfft_batched of the windowed frames,
    crlot_istft_ola vs crlot_irfft_batched of the stepped spectra +
    crlot_ola_gather, the per-frame masked crlot_roundtrip vs
    crlot_istft_ola(crlot_stft), the walkers vs their staged fallbacks, every
    chunking, and the frame-pair masked walk under a mask of ones vs
    the unmasked frame-pair round trip;
  * the frame-pair masked walk vs the per-frame one: the FFT tolerance.
"""
import numpy as np
import pytest

from test_gpu_parity import assert_close, bits, dev, host, rel_l2

pytestmark = pytest.mark.gpu

SHAPES = [(1024, 256), (4096, 1024), (512, 128)]
# the spectral entries as frame pairs (K_pair_stft / K_pair_istft, frame pairing on: the default)
PAIR_SPEC = {(1024, 128), (1024, 256), (1024, 512), (512, 128), (512, 256),
             (2048, 256), (2048, 512), (2048, 1024), (4096, 512), (4096, 1024), (4096, 2048)}  # (N >= 2048: one workgroup per walk)


def assert_spec_close(X, ref, what=""):
    X = np.asarray(X, np.complex64)
    ref = np.asarray(ref, np.complex64)
    assert X.shape == ref.shape, (what, X.shape, ref.shape)
    assert np.all(np.isfinite(X.view(np.float32))), what
    scale = float(np.max(np.abs(ref))) if ref.size else 0.0
    r = rel_l2(X, ref)
    m = float(np.max(np.abs(X.astype(np.complex128) - ref))) if X.size else 0.0
    assert r <= 1e-6 or np.linalg.norm(ref) < 1e-20, f"{what}: rel-L2 {r:.3e}"
    assert m <= 4e-6 * max(scale, 1e-30), f"{what}: max-abs {m:.3e} (scale {scale:.3e})"


def frames_np(oracle, x, n, h, mode, center=True, pad_mode=0):
    """Raw frames of one stream: the Framer (whole push) or the FrameQueue."""
    if mode == oracle.FRAMEQUEUE:
        return oracle.fq_frames(x, n, h, center, pad_mode).reshape(-1, n)
    T = x.size
    F = oracle.frame_count(T, n, h, mode)
    out = np.zeros((F, n), np.float32)
    for k in range(F):
        seg = x[k * h:k * h + n]
        out[k, :seg.size] = seg
    return out


def special(x):
    """NaN / Inf bursts, sub-threshold and denormal stretches, a huge sample."""
    x = x.copy()
    T = x.shape[1]
    x[0, 100:110] = np.nan
    x[0, min(2000, T - 1)] = np.inf
    x[0, min(2100, T - 2)] = -np.inf
    if x.shape[0] > 1:
        x[1, 300:900] = 1e-35
        x[1, 1000:1010] = 1e-42
        x[1, min(5000, T - 3)] = 3e30
    return x


def finite_scale(xs):
    """(max |x|, ||x||) over the finite samples: the tolerance scale of a stream."""
    f = np.where(np.isfinite(xs), xs, 0).astype(np.float64)
    return float(np.max(np.abs(f))) if f.size else 0.0, float(np.linalg.norm(f))


def stepped(spec, gain=None, mask=None):
    """spectrum * gain[b] then * mask[k, b] in float32, re and im each (the oracle's step)."""
    f = np.ascontiguousarray(spec, np.complex64).view(np.float32).reshape(spec.shape + (2,)).copy()
    if gain is not None:
        f *= np.asarray(gain, np.float32)[..., None]
    if mask is not None:
        f *= np.asarray(mask, np.float32)[..., None]
    return f.view(np.complex64).reshape(spec.shape)


@pytest.mark.parametrize("n,h", SHAPES + [(256, 128), (2048, 512), (1024, 300)])
@pytest.mark.parametrize("mode", [0, 1, 2])  # ZERO_PAD, DROP, FRAMEQUEUE (centre, reflect)
def test_stft_vs_oracle_and_rfft(pkg, oracle, torch_cuda, n, h, mode):
    torch = torch_cuda
    S, T = 3, 9 * n + 77
    x = special(oracle.synth_streams(S, T, config_id=61))
    kw = dict(center=True, pad_mode=pkg.PAD_REFLECT) if mode == 2 else {}
    plan = pkg.Plan(frame_size=n, hop_size=h, boundary_mode=mode, **kw)
    xd = dev(torch, x)
    paired = (n, h) in PAIR_SPEC  # K_pair_stft (frame pairing on, the default)
    spec = host(plan.stft(xd))
    assert plan.last_launch()["kernels"] == ["k_pair_stft" if paired else "k_stft"]
    if paired:  # ... and the per-frame kernel beside it, the one the bit-exact check below holds for
        plan.set_frame_pairing(False)
        spec_pf = host(plan.stft(xd))
        assert plan.last_launch()["kernels"] == ["k_stft"]
        plan.set_frame_pairing(True)
    else:
        spec_pf = spec
    F = plan.frame_count(T)
    assert spec.shape == (S, F, n // 2 + 1)
    w = oracle.window(oracle.HANN, n)
    for s in range(S):
        _, ref = oracle.roundtrip_mask(x[s], n, h, mode=mode, pad_mode=kw.get("pad_mode", 0), want_spec=True)
        assert_spec_close(spec[s], ref, f"{n}/{h} mode {mode} stream {s}")
        assert_spec_close(spec_pf[s], ref, f"{n}/{h} mode {mode} stream {s} per frame")
        assert np.all(spec[s][:, 0].imag == 0) and np.all(spec[s][:, -1].imag == 0)
        fr = frames_np(oracle, x[s], n, h, mode, True, kw.get("pad_mode", 0))
        direct = host(plan.rfft(dev(torch, (fr * w).astype(np.float32))))
        assert np.array_equal(bits(spec_pf[s].view(np.float32)), bits(direct.view(np.float32))), (n, h, mode, s)


@pytest.mark.parametrize("n,h", SHAPES + [(2048, 1024), (1024, 128)])
def test_istft_ola_bit_exact_vs_irfft_gather(pkg, oracle, torch_cuda, n, h):
    torch = torch_cuda
    S, T = 3, 11 * n + 5
    bins = n // 2 + 1
    x = oracle.synth_streams(S, T, config_id=62)
    plan = pkg.Plan(frame_size=n, hop_size=h)
    spec = plan.stft(dev(torch, x))
    F = spec.shape[1]
    rng = np.random.default_rng(n + h)
    gain = rng.uniform(0.0, 2.0, bins).astype(np.float32)
    mask = rng.uniform(-1.5, 1.5, (S, F, bins)).astype(np.float32)
    paired = (n, h) in PAIR_SPEC  # K_pair_istft (frame pairing on, the default)
    for g, m in ((None, None), (gain, None), (None, mask), (gain, mask)):
        plan.set_spectral_gain(g)
        plan.set_spectral_mask(None if m is None else dev(torch, m))
        X = dev(torch, stepped(host(spec), g, m))
        fr = plan.irfft(X.reshape(S * F, bins)).reshape(S, F, n)
        ref = host(plan.ola_gather(fr))
        if paired:
            yp = host(plan.istft_ola(spec))
            assert plan.last_launch()["kernels"] == ["k_pair_istft"]
            for s in range(S):
                assert_close(yp[s], ref[s], float(np.max(np.abs(ref[s]))), f"{n}/{h} pair istft stream {s}",
                             float(np.linalg.norm(ref[s])))
            plan.set_frame_pairing(False)
        y = host(plan.istft_ola(spec))
        assert plan.last_launch()["kernels"] == ["k_istft"]
        assert np.array_equal(bits(y), bits(ref)), (n, h, g is not None, m is not None)
        plan.set_frame_pairing(True)
    plan.set_spectral_gain(None)
    plan.set_spectral_mask(None)


@pytest.mark.parametrize("n,h", SHAPES)
@pytest.mark.parametrize("shared", [False, True])
@pytest.mark.parametrize("pairing", [True, False])
def test_masked_roundtrip(pkg, oracle, torch_cuda, n, h, shared, pairing):
    """crlot_roundtrip with a per-frame mask: one walk over HBM -- per frame
    (k_stft_masked) bit-identical to crlot_istft_ola(crlot_stft(x)); at the PAIR_SPEC shapes
    with frame pairing (the default) as frame pairs (k_pair_mask) within the FFT
    tolerance of it -- and the oracle's masked e2e loop within the FFT tolerance,
    with NaN, Inf, tiny and huge samples in the input."""
    if not pairing and (n, h) not in PAIR_SPEC:
        pytest.skip("frame pairing only changes the frame-pair shapes' walk")
    torch = torch_cuda
    S, T = 4, 13 * n + 31
    bins = n // 2 + 1
    x = special(oracle.synth_streams(S, T, config_id=63))
    plan = pkg.Plan(frame_size=n, hop_size=h)
    plan.set_frame_pairing(pairing)
    F = plan.frame_count(T)
    rng = np.random.default_rng(7 * n + h)
    m = rng.uniform(0.0, 1.0, (F, bins) if shared else (S, F, bins)).astype(np.float32)
    m[..., ::17] = 0.0
    plan.set_spectral_mask(dev(torch, m))
    xd = dev(torch, x)
    y = host(plan.roundtrip(xd))
    paired = pairing and (n, h) in PAIR_SPEC  # (the frame-pair masked walk takes the same shapes)
    assert plan.last_launch()["kernels"] == ["k_pair_mask" if paired else "k_stft_masked"]
    y2 = host(plan.istft_ola(plan.stft(xd)))
    assert np.all(np.isfinite(y))
    if not paired and not (pairing and (n, h) in PAIR_SPEC):
        assert np.array_equal(bits(y), bits(y2))
    for s in range(S):
        ms = m if shared else m[s]
        ref = oracle.roundtrip_mask(x[s], n, h, mask=ms)
        xmax, xnorm = finite_scale(x[s])
        assert_close(y[s], ref, xmax, f"{n}/{h} masked stream {s}", xnorm)
        assert_close(y[s], y2[s], xmax, f"{n}/{h} masked vs istft(stft) stream {s}", xnorm)
    plan.set_spectral_mask(None)


@pytest.mark.parametrize("n,h", sorted(PAIR_SPEC))
def test_pair_mask_walk(pkg, oracle, torch_cuda, n, h):
    """K_pair_mask (N = 512 - 4096): frames 2j, 2j+1 share one transform and the step
    separates them (c1 Z + c2 conj Z[-k]).  A mask of ones gives K_pair's own bits
    (with and without a spectral gain, NaN / Inf / huge samples included); a
    time-varying signed mask with zero, NaN, tiny and huge (unpaired regime)
    values matches the oracle and the per-frame walk within the FFT tolerance;
    the bits do not depend on the chunking; odd frame counts."""
    torch = torch_cuda
    S = 4
    T = 29 * n + 18  # (even rows: the unmasked N = 512 round trip takes K_pair512; F odd at every hop here)
    bins = n // 2 + 1
    x = special(oracle.synth_streams(S, T, config_id=68))
    plan = pkg.Plan(frame_size=n, hop_size=h)
    F = plan.frame_count(T)
    xd = dev(torch, x)
    gain = np.linspace(0.5, 1.5, bins).astype(np.float32)
    ones = dev(torch, np.ones((F, bins), np.float32))
    for g in (None, gain):
        plan.set_spectral_gain(g)
        plan.set_spectral_mask(None)
        y0 = host(plan.roundtrip(xd))
        assert plan.last_launch()["kernels"][0].startswith("k_pair"), plan.last_launch()
        plan.set_spectral_mask(ones)
        y1 = host(plan.roundtrip(xd))
        assert plan.last_launch()["kernels"] == ["k_pair_mask"]
        assert np.array_equal(bits(y1), bits(y0)), (h, g is not None)
    rng = np.random.default_rng(h)
    m = rng.uniform(-1.0, 1.5, (S, F, bins)).astype(np.float32)
    m[..., ::13] = 0.0
    m[1, 5, 40] = np.nan
    m[1, 20, :] = 1e-30
    m[2, 9, 100] = 1e25
    m[3, F - 1, 3] = 2.0 ** 21  # the last frame's (odd F: its own pair)
    plan.set_spectral_mask(dev(torch, m))
    y = host(plan.roundtrip(xd))
    assert plan.last_launch()["kernels"] == ["k_pair_mask"]
    for c in (1, 2, 5, F):
        plan.set_chunks(c)
        assert np.array_equal(bits(host(plan.roundtrip(xd))), bits(y)), c
    plan.set_chunks(0)
    plan.set_frame_pairing(False)
    yf = host(plan.roundtrip(xd))
    assert plan.last_launch()["kernels"] == ["k_stft_masked"]
    plan.set_frame_pairing(True)
    for s in range(S):
        ref = oracle.roundtrip_mask(x[s], n, h, bin_gain=gain, mask=m[s])
        ymax, ynorm = finite_scale(ref)
        assert_close(y[s], ref, ymax, f"{h} pair mask stream {s}", ynorm)
        assert_close(y[s], yf[s], ymax, f"{h} pair vs per-frame stream {s}", ynorm)
    plan.set_spectral_mask(None)
    plan.set_spectral_gain(None)


@pytest.mark.parametrize("n,h", SHAPES)
def test_masked_roundtrip_chunking_and_fallbacks(pkg, oracle, torch_cuda, n, h):
    """The bits do not depend on the chunking, nor on whether the walk or the
    staged path (spectra through HBM, k_spec_step + irfft + gather) runs."""
    torch = torch_cuda
    S, T = 3, 17 * n + 9
    bins = n // 2 + 1
    x = oracle.synth_streams(S, T, config_id=64)
    plan = pkg.Plan(frame_size=n, hop_size=h)
    plan.set_frame_pairing(False)  # (the per-frame walk; test_pair_mask_walk covers K_pair_mask)
    F = plan.frame_count(T)
    m = np.random.default_rng(3).uniform(0.2, 1.2, (S, F, bins)).astype(np.float32)
    plan.set_spectral_mask(dev(torch, m))
    plan.set_spectral_gain(np.linspace(0.5, 1.5, bins).astype(np.float32))
    xd = dev(torch, x)
    y0 = host(plan.roundtrip(xd))
    for c in (1, 2, 5, F):
        plan.set_chunks(c)
        assert np.array_equal(bits(host(plan.roundtrip(xd))), bits(y0)), c
        assert np.array_equal(bits(host(plan.istft_ola(plan.stft(xd)))), bits(y0)), c
    plan.set_chunks(0)
    # x rows 4-byte aligned only: still the one walk (its frame loads check the alignment)
    xo = torch.zeros((S, T + 1), device="cuda")
    xo[:, :T] = xd
    xv = xo[:, :T]
    assert np.array_equal(bits(host(plan.roundtrip(xv))), bits(y0))
    assert plan.last_launch()["kernels"] == ["k_stft_masked"]
    # output rows 4-byte aligned only: spectra through HBM, k_spec_step + irfft + gather
    yo = torch.zeros((S, F * h + 1), device="cuda")
    plan.roundtrip(xv, yo[:, :F * h])
    ks = plan.last_launch()["kernels"]
    assert ks[:2] == ["k_stft", "k_spec_step"] and "k_gather" in ks[-1], ks
    assert np.array_equal(bits(host(yo[:, :F * h])), bits(y0))
    spec = plan.stft(xv)
    yo.zero_()
    assert np.array_equal(bits(host(plan.istft_ola(spec, yo[:, :F * h]))), bits(y0))
    assert plan.last_launch()["kernels"][0] == "k_spec_step"
    plan.set_spectral_mask(None)
    plan.set_spectral_gain(None)


@pytest.mark.parametrize("n,h", [(960, 240), (882, 441), (1024, 200), (480, 120), (1000, 250)])
def test_other_sizes(pkg, oracle, torch_cuda, n, h):
    """Frame sizes / hops outside the walkers: the staged forms (windowed frames ->
    mixed-radix rfft; spectral step -> irfft -> gather) against the oracle (frame
    pairing off: these sizes have frame-pair kernels, test_anysize_pair_spectral_entries)."""
    torch = torch_cuda
    S, T = 3, 12 * n + 13
    bins = n // 2 + 1
    x = special(oracle.synth_streams(S, T, config_id=65))
    plan = pkg.Plan(frame_size=n, hop_size=h)
    plan.set_frame_pairing(False)
    xd = dev(torch, x)
    spec = plan.stft(xd)
    F = spec.shape[1]
    m = np.random.default_rng(n).uniform(0.0, 1.0, (S, F, bins)).astype(np.float32)
    specn = host(spec)
    for s in range(S):
        _, ref = oracle.roundtrip_mask(x[s], n, h, want_spec=True)
        assert_spec_close(specn[s], ref, f"{n}/{h} stream {s}")
    plan.set_spectral_mask(dev(torch, m))
    y = host(plan.istft_ola(spec))
    yr = host(plan.roundtrip(xd))
    assert np.array_equal(bits(y), bits(yr))
    for s in range(S):
        xmax, xnorm = finite_scale(x[s])
        ref = oracle.roundtrip_mask(x[s], n, h, mask=m[s])
        assert_close(y[s], ref, xmax, f"{n}/{h} stream {s}", xnorm)
    plan.set_spectral_mask(None)


def test_framequeue_pipeline_masked(pkg, oracle, torch_cuda):
    """performance_benchmark.cc:174-246's framing (FrameQueue, centre, reflect, no
    analysis window) with a per-frame mask."""
    torch = torch_cuda
    n, h, S, T = 1024, 256, 2, 20000
    x = oracle.synth_streams(S, T, config_id=66)
    plan = pkg.Plan(frame_size=n, hop_size=h, boundary_mode=pkg.FRAMEQUEUE, analysis_window=False,
                    pad_mode=pkg.PAD_REFLECT)
    F = plan.frame_count(T)
    m = np.random.default_rng(9).uniform(0.0, 1.0, (F, n // 2 + 1)).astype(np.float32)
    plan.set_spectral_mask(dev(torch, m))
    xd = dev(torch, x)
    y = host(plan.roundtrip(xd))
    assert plan.last_launch()["kernels"] == ["k_pair_mask"]
    plan.set_frame_pairing(False)
    yf = host(plan.roundtrip(xd))
    assert np.array_equal(bits(yf), bits(host(plan.istft_ola(plan.stft(xd)))))
    for s in range(S):
        assert_close(y[s], yf[s], 0.5, f"framequeue pair vs per-frame stream {s}")
        ref = oracle.roundtrip_mask(x[s], n, h, mask=m, mode=oracle.FRAMEQUEUE, pad_mode=oracle.PAD_REFLECT,
                                    analysis_window=False)
        assert_close(y[s], ref, 0.5, f"framequeue stream {s}")


@pytest.mark.parametrize("n,h", [(1024, 256), (4096, 1024), (2048, 256)])
def test_short_and_empty_streams(pkg, oracle, torch_cuda, n, h):
    """Streams of one or two frames, a hop either side of the frame edges, an
    empty batch; the masked walk as well (one pair, a lone last frame)."""
    torch = torch_cuda
    plan = pkg.Plan(frame_size=n, hop_size=h)
    for T in (1, 2, 5, h - 1, h, h + 1, n - 1, n + 1):
        x = oracle.synth_streams(2, T, config_id=67)
        xd = dev(torch, x)
        spec = host(plan.stft(xd))
        y = host(plan.istft_ola(plan.stft(xd)))
        F = plan.frame_count(T)
        m = np.random.default_rng(T).uniform(0.0, 1.0, (F, n // 2 + 1)).astype(np.float32)
        plan.set_spectral_mask(dev(torch, m))
        ym = host(plan.roundtrip(xd))
        plan.set_spectral_mask(None)
        for s in range(2):
            yr, ref = oracle.roundtrip_mask(x[s], n, h, want_spec=True)
            assert_spec_close(spec[s], ref, f"{n}/{h} T={T}")
            assert_close(y[s], yr, 0.5, f"{n}/{h} T={T}", float(np.linalg.norm(x[s])))
            assert_close(ym[s], oracle.roundtrip_mask(x[s], n, h, mask=m), 0.5, f"{n}/{h} masked T={T}",
                         float(np.linalg.norm(x[s])))
    empty = torch.zeros((2, 0), device="cuda")
    assert plan.stft(empty).shape == (2, 0, n // 2 + 1)


def test_abi_validation(pkg, torch_cuda):
    torch = torch_cuda
    L = pkg.lib()
    plan = pkg.Plan(frame_size=1024, hop_size=256)
    x = torch.zeros((2, 4096), device="cuda")
    R = 1026  # N + 2 floats: one spectrum row
    spec = torch.zeros((2, 16, R), device="cuda")
    y = torch.zeros((2, 4096), device="cuda")
    xp, sp, yp = x.data_ptr(), spec.data_ptr(), y.data_ptr()
    assert L.crlot_stft(None, xp, sp, 2, 4096, 4096, 16 * R, R, None) == pkg.EINVAL
    assert L.crlot_stft(plan._h, xp, sp, 2, 4096, 4096, 16 * R, R - 2, None) == pkg.EINVAL
    assert L.crlot_stft(plan._h, xp, sp + 4, 2, 4096, 4096, 16 * R, R, None) == pkg.EINVAL
    assert L.crlot_stft(plan._h, xp, sp, 2, 4096, 4096, 15 * R, R, None) == pkg.EINVAL
    assert L.crlot_stft(plan._h, xp, sp, 2, 4096, 4095, 16 * R, R, None) == pkg.EINVAL
    assert L.crlot_istft_ola(plan._h, sp, yp, 2, 16, 16 * R, R + 1, 4096, None) == pkg.EINVAL
    assert L.crlot_istft_ola(plan._h, sp, yp, 2, 16, 16 * R, R, 4095, None) == pkg.EINVAL
    assert L.crlot_istft_ola(plan._h, None, yp, 2, 16, 16 * R, R, 4096, None) == pkg.EINVAL
    assert L.crlot_plan_set_spectral_mask(plan._h, sp, 512, 0) == pkg.EINVAL
    assert L.crlot_plan_set_spectral_mask(plan._h, sp, 513, -1) == pkg.EINVAL
    assert L.crlot_plan_set_spectral_mask(plan._h, sp + 2, 513, 0) == pkg.EINVAL
    assert L.crlot_stft(plan._h, xp, sp, 2, 4096, 4096, 16 * R, R, None) == 0
    assert L.crlot_istft_ola(plan._h, sp, yp, 2, 16, 16 * R, R, 4096, None) == 0
    assert L.crlot_stft(plan._h, xp, sp, 0, 4096, 4096, 16 * R, R, None) == 0  # nothing to do
    torch.cuda.synchronize()


@pytest.mark.parametrize("n,h", [(1024, 256), (4096, 1024)])
def test_full_size_stft_istft(pkg, oracle, torch_cuda, n, h):
    """At BASELINE scale (1024 x 480000, the headline's 1024/256 and config 3's
    4096/1024; 7.9 GB of spectra): istft_ola(stft(x)) within the parity bar of
    crlot_roundtrip(x) on sampled streams and of the oracle; an all-ones shared
    mask gives the masked walk the same bits; determinism."""
    torch = torch_cuda
    S, T = 1024, 480_000
    g = torch.Generator(device="cuda").manual_seed(4321)
    x = (torch.rand((S, T), generator=g, device="cuda") * 2 - 1) * 0.5
    plan = pkg.Plan(frame_size=n, hop_size=h)
    spec = plan.stft(x)  # frame pairs (K_pair_stft / K_pair_istft)
    y = plan.istft_ola(spec)
    assert torch.equal(y, plan.istft_ola(plan.stft(x)))
    plan.set_frame_pairing(False)  # per frame (K_stft / K_istft)
    spec = plan.stft(x)
    y_pf = plan.istft_ola(spec)
    plan.set_frame_pairing(True)
    del spec
    yr = plan.roundtrip(x)
    F = plan.frame_count(T)
    ones = torch.ones((F, n // 2 + 1), device="cuda")
    plan.set_spectral_mask(ones)
    ym = plan.roundtrip(x)  # frame pairs (K_pair_mask): K_pair's bits
    assert torch.equal(ym, yr)
    plan.set_frame_pairing(False)
    ym = plan.roundtrip(x)  # per frame: istft(stft)'s bits
    assert torch.equal(ym, y_pf)
    plan.set_frame_pairing(True)
    plan.set_spectral_mask(None)
    for s in (0, 700, 1023):
        xs = host(x[s])
        ref = oracle.roundtrip(xs, n, h)
        for yy, what in ((y, "pairs"), (y_pf, "per frame")):
            assert_close(host(yy[s]), ref, 0.5, f"stft+istft ({what}) stream {s}", float(np.linalg.norm(xs)))
            assert_close(host(yy[s]), host(yr[s]), 0.5, f"vs roundtrip ({what}) stream {s}", float(np.linalg.norm(xs)))
    del x, y, y_pf, yr, ym
    torch.cuda.empty_cache()


@pytest.mark.parametrize("n,h", [(960, 240), (1920, 480), (882, 441)])
def test_full_size_anysize_stft_istft(pkg, oracle, torch_cuda, n, h):
    """The any-size frame-pair entries (K_pair15's / K_pairN's transforms) at
    1024 x 480000: istft_ola(stft(x)) deterministic, within the parity bar of the
    per-frame entries, of crlot_roundtrip(x) and of the oracle on sampled streams;
    the masked walk under an all-ones shared mask within the bar of the round trip."""
    torch = torch_cuda
    S, T = 1024, 480_000
    g = torch.Generator(device="cuda").manual_seed(8765)
    x = (torch.rand((S, T), generator=g, device="cuda") * 2 - 1) * 0.5
    plan = pkg.Plan(frame_size=n, hop_size=h)
    y = plan.istft_ola(plan.stft(x))
    assert torch.equal(y, plan.istft_ola(plan.stft(x)))
    plan.set_frame_pairing(False)
    y_pf = plan.istft_ola(plan.stft(x))
    plan.set_frame_pairing(True)
    yr = plan.roundtrip(x)
    F = plan.frame_count(T)
    plan.set_spectral_mask(torch.ones((F, n // 2 + 1), device="cuda"))  # (one row per frame, shared)
    ym = plan.roundtrip(x)
    plan.set_spectral_mask(None)
    assert bool(torch.isfinite(y).all()) and bool(torch.isfinite(ym).all())
    for s in (0, 511, 1023):
        xs = host(x[s])
        nx = float(np.linalg.norm(xs))
        ref = oracle.roundtrip(xs, n, h)
        assert_close(host(y[s]), ref, 0.5, f"stft+istft pairs stream {s}", nx)
        assert_close(host(y[s]), host(y_pf[s]), 0.5, f"pairs vs per frame stream {s}", nx)
        assert_close(host(y[s]), host(yr[s]), 0.5, f"pairs vs roundtrip stream {s}", nx)
        assert_close(host(ym[s]), host(yr[s]), 0.5, f"masked (ones) vs roundtrip stream {s}", nx)
    del x, y, y_pf, yr, ym
    torch.cuda.empty_cache()


@pytest.mark.parametrize("n,h", sorted(PAIR_SPEC))
def test_pair_stft_istft(pkg, oracle, torch_cuda, n, h):
    """K_pair_stft / K_pair_istft (N = 512 - 4096, frame pairing on): spectra and the
    split round trip vs the oracle and vs the per-frame kernels within the FFT
    tolerance, with NaN / Inf / tiny / huge samples (the forward's per-frame
    regime) and NaN / Inf / 1e30 spectrum values (the inverse's); the bits do not
    depend on the chunking; odd frame counts; gain + mask."""
    torch = torch_cuda
    S = 4
    T = 23 * n + 57
    bins = n // 2 + 1
    x = special(oracle.synth_streams(S, T, config_id=69))
    plan = pkg.Plan(frame_size=n, hop_size=h)
    F = plan.frame_count(T)
    xd = dev(torch, x)
    spec = plan.stft(xd)
    assert plan.last_launch()["kernels"] == ["k_pair_stft"]
    sh = host(spec)
    for c in (1, 2, 5, F):
        plan.set_chunks(c)
        assert np.array_equal(bits(host(plan.stft(xd)).view(np.float32)), bits(sh.view(np.float32))), c
    plan.set_chunks(0)
    plan.set_frame_pairing(False)
    spf = host(plan.stft(xd))
    plan.set_frame_pairing(True)
    for s in range(S):
        _, ref = oracle.roundtrip_mask(x[s], n, h, want_spec=True)
        assert_spec_close(sh[s], ref, f"{h} pair stft stream {s}")
        assert_spec_close(sh[s], spf[s], f"{h} pair vs per-frame stft stream {s}")
    # the inverse: a gain, a signed mask, and edited spectra that leave the paired regime
    rng = np.random.default_rng(h + 1)
    gain = np.linspace(0.5, 1.5, bins).astype(np.float32)
    m = rng.uniform(-1.0, 1.5, (S, F, bins)).astype(np.float32)
    se = sh.copy()
    se[1, 3, 17] = np.nan
    se[2, 8, 100] = np.inf
    se[3, 11, 40] = 1e30
    se[3, F - 1, 5] = 1e25
    sed = dev(torch, se)
    for g, mm in ((None, None), (gain, None), (gain, m)):
        plan.set_spectral_gain(g)
        plan.set_spectral_mask(None if mm is None else dev(torch, mm))
        y = host(plan.istft_ola(sed))
        assert plan.last_launch()["kernels"] == ["k_pair_istft"]
        for c in (1, 3, F):
            plan.set_chunks(c)
            assert np.array_equal(bits(host(plan.istft_ola(sed))), bits(y)), c
        plan.set_chunks(0)
        plan.set_frame_pairing(False)
        ypf = host(plan.istft_ola(sed))
        assert plan.last_launch()["kernels"] == ["k_istft"]
        plan.set_frame_pairing(True)
        assert np.all(np.isfinite(y))
        for s in range(S):
            ymax, ynorm = finite_scale(ypf[s])
            assert_close(y[s], ypf[s], ymax, f"{h} pair vs per-frame istft stream {s}", ynorm)
    plan.set_spectral_gain(None)
    plan.set_spectral_mask(None)
    # the split round trip of plain input vs the fused one and the oracle
    xp = oracle.synth_streams(S, T, config_id=70)
    xpd = dev(torch, xp)
    y2 = host(plan.istft_ola(plan.stft(xpd)))
    yr = host(plan.roundtrip(xpd))
    for s in range(S):
        ref = oracle.roundtrip(xp[s], n, h)
        assert_close(y2[s], ref, 0.5, f"{h} pair split vs oracle stream {s}", float(np.linalg.norm(xp[s])))
        assert_close(y2[s], yr[s], 0.5, f"{h} pair split vs roundtrip stream {s}", float(np.linalg.norm(xp[s])))


@pytest.mark.parametrize("seed", range(10))
def test_spectral_entries_random_shapes(pkg, oracle, torch_cuda, seed):
    """Random shapes through crlot_stft / crlot_istft_ola / the masked round trip:
    frame sizes with and without frame-pair kernels, every framing, stream counts
    and lengths (short streams, odd frame counts), leading dimensions with slack;
    frame pairs vs per frame within the FFT tolerance, per frame bit-exact between
    the split and the fused masked walk, one stream vs the oracle."""
    torch = torch_cuda
    rng = np.random.default_rng(1000 + seed)
    n, h = [(1024, 256), (1024, 128), (1024, 512), (512, 128), (512, 256), (2048, 512), (256, 128),
            (4096, 1024), (960, 240), (960, 320), (480, 120), (882, 441)][int(rng.integers(12))]
    mode = int(rng.integers(3))
    kw = dict(center=bool(rng.integers(2)), pad_mode=int(rng.integers(3))) if mode == 2 else {}
    S = int(rng.integers(1, 6))
    T = int(rng.integers(n // 2, 9 * n))
    plan = pkg.Plan(frame_size=n, hop_size=h, boundary_mode=mode, **kw)
    F = plan.frame_count(T)
    if F == 0:
        pytest.skip("no frames")
    bins = n // 2 + 1
    x = oracle.synth_streams(S, T, config_id=80 + seed)
    ldx = T + int(rng.integers(0, 5))
    xs = torch.zeros((S, ldx), device="cuda")
    xs[:, :T] = dev(torch, x)
    xv = xs[:, :T]
    m = rng.uniform(0.0, 1.2, (S, F, bins)).astype(np.float32)
    outs = {}
    for pairing in (True, False):
        plan.set_frame_pairing(pairing)
        spec = plan.stft(xv)
        plan.set_spectral_mask(dev(torch, m))
        y_split = host(plan.istft_ola(spec))
        y_walk = host(plan.roundtrip(xv))
        plan.set_spectral_mask(None)
        outs[pairing] = (host(spec), y_split, y_walk)
    sp, ysp, ywp = outs[True]
    sf, ysf, ywf = outs[False]
    assert np.array_equal(bits(ysf), bits(ywf)), (n, h, mode, S, T)  # per frame: split == fused walk
    for s in range(S):
        assert_spec_close(sp[s], sf[s], f"{n}/{h} pairs vs per frame, stream {s}")
        ymax, ynorm = finite_scale(ysf[s])
        for yy, what in ((ysp, "split"), (ywp, "walk")):
            assert_close(yy[s], ysf[s], max(ymax, 1e-30), f"{n}/{h} {what} vs per frame, stream {s}", ynorm)
    ref = oracle.roundtrip_mask(x[0], n, h, mask=m[0], mode=mode, center=kw.get("center", True),
                                pad_mode=kw.get("pad_mode", 0))
    assert_close(ysf[0], ref, max(finite_scale(ref)[0], 1e-30), f"{n}/{h} mode {mode} vs oracle",
                 finite_scale(ref)[1])


@pytest.mark.parametrize("n,h", [(960, 240), (960, 480), (960, 320), (960, 100), (480, 120), (480, 240), (480, 100),
                                 (882, 441), (882, 220), (1000, 250), (640, 320), (400, 160), (320, 160),
                                 (1764, 441), (1920, 480), (1920, 455)])
def test_anysize_pair_spectral_entries(pkg, oracle, torch_cuda, n, h):
    """The any-size frame pairs: N = 960 / 480 (20 / 10 ms at 48 kHz) on K_pair15's
    transforms (at 480 the two halves of a wave walk two streams, an odd stream
    count here) and 882 (20 ms at 44.1 kHz), 1000, 640, 400, 320, 1764, 1920 (two waves
    per transform; 1920 at an even hop with a twiddle table of its own beside K_pair30's)
    on K_pairN's (any hop):
    crlot_stft, crlot_istft_ola and the masked round trip vs the oracle and vs the
    per-frame staged forms (frame pairing off) within the FFT tolerance, with NaN /
    Inf / tiny / huge samples (the per-frame regime), edited spectra and signed /
    NaN / huge mask values; the bits do not depend on the chunking; odd F."""
    torch = torch_cuda
    S = 3
    T = 21 * n + 37
    bins = n // 2 + 1
    x = special(oracle.synth_streams(S, T, config_id=71))
    plan = pkg.Plan(frame_size=n, hop_size=h)
    F = plan.frame_count(T)
    xd = dev(torch, x)
    spec = plan.stft(xd)
    assert plan.last_launch()["kernels"] == ["k_pair_stft"]
    sh = host(spec)
    for c in (1, 3, F):
        plan.set_chunks(c)
        assert np.array_equal(bits(host(plan.stft(xd)).view(np.float32)), bits(sh.view(np.float32))), c
    plan.set_chunks(0)
    plan.set_frame_pairing(False)
    spf = host(plan.stft(xd))
    plan.set_frame_pairing(True)
    for s in range(S):
        _, ref = oracle.roundtrip_mask(x[s], n, h, want_spec=True)
        assert_spec_close(sh[s], ref, f"{n}/{h} pair stft stream {s}")
        assert_spec_close(sh[s], spf[s], f"{n}/{h} pair vs per-frame stft stream {s}")
        assert np.all(sh[s][:, 0].imag == 0) and np.all(sh[s][:, -1].imag == 0)
    # the inverse: gain, signed mask, edited spectra that leave the paired regime
    rng = np.random.default_rng(h)
    gain = np.linspace(0.5, 1.5, bins).astype(np.float32)
    m = rng.uniform(-1.0, 1.5, (S, F, bins)).astype(np.float32)
    se = sh.copy()
    se[1, 3, 17] = np.nan
    se[2, 8, 100] = np.inf
    se[2, F - 1, 5] = 1e25
    sed = dev(torch, se)
    for g, mm in ((None, None), (gain, None), (gain, m)):
        plan.set_spectral_gain(g)
        plan.set_spectral_mask(None if mm is None else dev(torch, mm))
        y = host(plan.istft_ola(sed))
        assert plan.last_launch()["kernels"] == ["k_pair_istft"]
        for c in (1, 3, F):
            plan.set_chunks(c)
            assert np.array_equal(bits(host(plan.istft_ola(sed))), bits(y)), c
        plan.set_chunks(0)
        plan.set_frame_pairing(False)
        ypf = host(plan.istft_ola(sed))
        plan.set_frame_pairing(True)
        assert np.all(np.isfinite(y))
        for s in range(S):
            ymax, ynorm = finite_scale(ypf[s])
            assert_close(y[s], ypf[s], ymax, f"{n}/{h} pair vs per-frame istft stream {s}", ynorm)
    plan.set_spectral_gain(None)
    # the masked round trip: one walk, vs the oracle's masked loop and the per-frame form
    m[..., ::13] = 0.0
    m[1, 5, 40] = np.nan
    m[1, 9, :] = 1e-30
    m[2, 2, 100] = 1e25
    m[0, F - 1, 3] = 2.0 ** 21
    plan.set_spectral_mask(dev(torch, m))
    plan.set_spectral_gain(gain)
    y = host(plan.roundtrip(xd))
    assert plan.last_launch()["kernels"] == ["k_pair_mask"]
    for c in (1, 2, 5, F):
        plan.set_chunks(c)
        assert np.array_equal(bits(host(plan.roundtrip(xd))), bits(y)), c
    plan.set_chunks(0)
    plan.set_frame_pairing(False)
    yf = host(plan.roundtrip(xd))
    plan.set_frame_pairing(True)
    for s in range(S):
        ref = oracle.roundtrip_mask(x[s], n, h, bin_gain=gain, mask=m[s])
        ymax, ynorm = finite_scale(ref)
        assert_close(y[s], ref, ymax, f"{n}/{h} pair mask stream {s}", ynorm)
        assert_close(y[s], yf[s], ymax, f"{n}/{h} pair vs per-frame mask stream {s}", ynorm)
    plan.set_spectral_mask(None)
    plan.set_spectral_gain(None)
    # plain input: the split round trip vs the fused one and the oracle
    xp = oracle.synth_streams(S, T, config_id=72)
    xpd = dev(torch, xp)
    y2 = host(plan.istft_ola(plan.stft(xpd)))
    yr = host(plan.roundtrip(xpd))
    for s in range(S):
        ref = oracle.roundtrip(xp[s], n, h)
        assert_close(y2[s], ref, 0.5, f"{n}/{h} pair split vs oracle stream {s}", float(np.linalg.norm(xp[s])))
        assert_close(y2[s], yr[s], 0.5, f"{n}/{h} pair split vs roundtrip stream {s}", float(np.linalg.norm(xp[s])))
