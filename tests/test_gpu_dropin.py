"""The reference's remaining drop-in surfaces on the device, against the oracle:

* dsp::axpy / axpy_windowed / normalize_and_clear (ola/kernels.h:28-53): the
  batched device forms and the host-pointer forms (resident call kernel),
  BIT-EXACT with the scalar kernels (kernels.cc:18-36) -- the reference's own
  bar is +-1 ULP between its Highway and scalar forms (tests/kernels_test.cc:
  214-429) -- at the reference test's sizes {0, 1, 7, ..., 4096} and at a
  batched size, plus kernels_test.cc's known values;
* dsp::FrameQueue (FrameQueue.h:35-59): the object and the batched device form,
  BIT-EXACT against the 48 fixtures dumped from the reference's own compiled
  FrameQueue.cc (tests/golden/ref_tables.npz fq_*), its exceptions;
* IFftPlan host-pointer calls on the resident call kernel: bit-identical to the
  launched device kernels (the same arithmetic), speculation hits and misses,
  strides, both domains, the staged fallback for other sizes; within the parity
  tolerance of the kissfft restatement.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SIZES = [0, 1, 7, 8, 15, 16, 31, 32, 63, 64, 127, 128, 255, 256, 511, 512, 1023, 1024, 4096]


def bits(a):
    """Bit patterns of a float32 array; complex64 spectra as their (re, im) pairs."""
    if np.iscomplexobj(a):
        return np.ascontiguousarray(a, np.complex64).view(np.float32).view(np.uint32)
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    return t.detach().cpu().numpy()


# ------------------------------------------------------------------ OLA kernels
def test_kernels_known_values(pkg, torch_cuda):
    """kernels_test.cc:67-207 values through the host-pointer forms."""
    dst = np.ones(10, np.float32)
    pkg.axpy_host(dst, np.full(10, 2, np.float32), 0.5)
    assert np.all(dst == 2.0)
    dst = np.ones(10, np.float32)
    pkg.axpy_host(dst, np.full(10, 2, np.float32), 0.0)
    assert np.all(dst == 1.0)
    dst = np.ones(1000, np.float32)
    pkg.axpy_host(dst, np.full(1000, 2, np.float32), 0.5)
    assert np.all(dst == 2.0)
    dst = np.ones(10, np.float32)
    pkg.axpy_host(dst, np.full(10, 2, np.float32), 1.0, win=np.full(10, 0.5, np.float32))
    assert np.all(dst == 2.0)
    acc = np.full(10, 4, np.float32)
    out = np.zeros(10, np.float32)
    pkg.normalize_and_clear_host(out, acc, np.full(10, 2, np.float32), 1e-8)
    assert np.all(out == 2.0) and np.all(acc == 0.0)
    acc = np.full(10, 1, np.float32)
    pkg.normalize_and_clear_host(out, acc, np.zeros(10, np.float32), 1e-3)  # eps guard
    assert np.all(out == np.float32(1.0) / np.float32(1e-3))


@pytest.mark.parametrize("n", SIZES)
def test_kernels_bit_exact_vs_scalar(pkg, oracle, torch_cuda, n):
    torch = torch_cuda
    rng = np.random.default_rng(42 + n)  # kernels_test.cc:219 mt19937(42), U(-10, 10)
    d, s, w = (rng.uniform(-10, 10, n).astype(np.float32) for _ in range(3))
    nrm = rng.uniform(-1, 3, n).astype(np.float32)  # some below eps
    nrm[::5] = 0.0
    for g in (1.0, 0.5, -1.75):
        want = oracle.axpy(d, s, g)
        want_w = oracle.axpy(d, s, g, win=w)
        # host-pointer forms (resident call kernel)
        a = d.copy()
        pkg.axpy_host(a, s, g)
        assert np.array_equal(bits(a), bits(want)), (n, g)
        a = d.copy()
        pkg.axpy_host(a, s, g, win=w)
        assert np.array_equal(bits(a), bits(want_w)), (n, g)
        if n == 0:
            continue
        # device forms, one row
        dd = dev(torch, d)
        pkg.axpy(dd, dev(torch, s), g)
        assert np.array_equal(bits(host(dd)), bits(want)), (n, g)
        dd = dev(torch, d)
        pkg.axpy(dd, dev(torch, s), g, win=dev(torch, w))
        assert np.array_equal(bits(host(dd)), bits(want_w)), (n, g)
    out_w, acc_w = oracle.normalize_and_clear(d, nrm, 0.25)
    out, acc = np.zeros(n, np.float32), d.copy()
    pkg.normalize_and_clear_host(out, acc, nrm, 0.25)
    assert np.array_equal(bits(out), bits(out_w)) and np.array_equal(acc, acc_w)
    if n:
        do, da = dev(torch, np.zeros(n, np.float32)), dev(torch, d)
        pkg.normalize_and_clear(do, da, dev(torch, nrm), 0.25)
        assert np.array_equal(bits(host(do)), bits(out_w)) and np.all(host(da) == 0)


def test_kernels_batched_rows_and_leading_dims(pkg, oracle, torch_cuda):
    """Batched device forms: B rows with padded leading dimensions (scalar and
    16-byte paths), the shared window / norm row, against the scalar kernels."""
    torch = torch_cuda
    rng = np.random.default_rng(3)
    for B, n, ld in ((64, 1024, 1024), (33, 1000, 1003), (5, 4096, 4100)):
        d = rng.uniform(-10, 10, (B, ld)).astype(np.float32)
        s = rng.uniform(-10, 10, (B, ld)).astype(np.float32)
        w = rng.uniform(0, 1, n).astype(np.float32)
        nrm = rng.uniform(0, 4, n).astype(np.float32)
        dd = dev(torch, d)
        pkg.axpy(dd[:, :n], dev(torch, s)[:, :n], 0.5, win=dev(torch, w))
        got = host(dd)
        for b in range(B):
            assert np.array_equal(bits(got[b, :n]), bits(oracle.axpy(d[b, :n], s[b, :n], 0.5, win=w))), (B, n, b)
        assert np.array_equal(got[:, n:], d[:, n:])  # padding untouched
        da = dev(torch, d)
        do = torch.zeros((B, ld), dtype=torch.float32, device="cuda")
        pkg.normalize_and_clear(do[:, :n], da[:, :n], dev(torch, nrm), 1e-8)
        go, ga = host(do), host(da)
        for b in range(B):
            ow, aw = oracle.normalize_and_clear(d[b, :n], nrm, 1e-8)
            assert np.array_equal(bits(go[b, :n]), bits(ow)) and np.array_equal(ga[b, :n], aw)
        assert np.array_equal(ga[:, n:], d[:, n:])


# ------------------------------------------------------------------ FrameQueue
def _fq_cases(ref_tables):
    for key in sorted(ref_tables.files):
        if key.startswith("fq_") and key.endswith("_meta"):
            base = key[:-5]
            T, N, H, c, m, F = (int(v) for v in ref_tables[key])
            yield base, T, N, H, c, m, F


def test_framequeue_object_bit_exact_vs_reference(pkg, torch_cuda, ref_tables):
    """All 48 fixtures of the reference's compiled FrameQueue (3 pad modes, centre
    on / off, signals shorter than the pad, T = 0): counts and every frame."""
    torch = torch_cuda
    cases = 0
    for base, T, N, H, c, m, F in _fq_cases(ref_tables):
        x = ref_tables[base + "_x"]
        want = ref_tables[base + "_frames"]
        q = pkg.FrameQueue(x, N, H, center=bool(c), pad_mode=m)
        assert q.getNumFrames() == F and q.getFrameSize() == N and q.getHopSize() == H, base
        assert np.array_equal(bits(q.getAllFrames()), bits(want)), base
        for k in {0, F // 2, F - 1} if F else ():
            assert np.array_equal(bits(q.getFrame(k)), bits(want[k * N:(k + 1) * N])), (base, k)
            buf = np.zeros(N, np.float32)
            q.copyFrame(k, buf)
            assert np.array_equal(bits(buf), bits(want[k * N:(k + 1) * N]))
        with pytest.raises(IndexError):
            q.getFrame(F)
        # the batched device form, two copies of the stream, padded rows
        if T:
            xd = torch.zeros((2, T + 3), dtype=torch.float32, device="cuda")
            xd[:, :T] = dev(torch, x)
            fr = host(pkg.framequeue_frames(xd[:, :T], N, H, center=bool(c), pad_mode=m))
            assert fr.shape == (2, F, N)
            for s in range(2):
                assert np.array_equal(bits(fr[s].reshape(-1)), bits(want)), base
        cases += 1
    assert cases == 48


def test_framequeue_errors(pkg, torch_cuda):
    """FrameQueue.cc:13-22, 49-67: the reference's exceptions."""
    x = np.arange(100, dtype=np.float32)
    with pytest.raises(ValueError):
        pkg.FrameQueue(x, 0, 4)
    with pytest.raises(ValueError):
        pkg.FrameQueue(x, 8, 0)
    with pytest.raises(ValueError):  # null input with len > 0
        pkg._check(pkg.lib().crlot_framequeue_create(None, 5, 8, 4, 1, 0, -1, pkg.C.byref(pkg.C.c_void_p())))
    q = pkg.FrameQueue(x, 16, 4, center=True)
    with pytest.raises(IndexError):
        q.copyFrame(q.getNumFrames(), np.zeros(16, np.float32))
    with pytest.raises(ValueError):
        q.copyFrame(0, None)
    e = pkg.FrameQueue(np.zeros(0, np.float32), 16, 4, center=False)
    assert e.getNumFrames() == 0 and e.getAllFrames().size == 0


# ------------------------------------------------------------------ IFftPlan host calls
@pytest.mark.parametrize("nfft", [256, 512, 1024, 2048, 4096])
def test_fft_host_calls_equal_device_kernels(pkg, oracle, torch_cuda, nfft):
    """forward_host / inverse_host (resident call kernel) give the launched device
    kernels' bits; an unchanged spectrum takes the speculated inverse, a changed
    one a real call -- both the device inverse's bits; the kissfft restatement
    agrees within the parity tolerance."""
    torch = torch_cuda
    rng = np.random.default_rng(nfft)
    plan = pkg.FftPlan(nfft)
    for B in (1, 3, 4, 16):
        x = rng.standard_normal((B, nfft)).astype(np.float32)
        X = plan.forward_host(x)
        Xd = host(plan.forward(dev(torch, x)))
        assert np.array_equal(X.view(np.uint32), Xd.view(np.uint32)), (nfft, B)
        ref = oracle.bench_rfft(x, nfft)
        assert np.linalg.norm(X - ref) <= 1e-6 * np.linalg.norm(ref)
        y_dev = host(plan.inverse(dev(torch, X)))
        y = plan.inverse_host(X)  # speculation hit (batch <= 4, nfft <= 2048) or a real call
        assert np.array_equal(bits(y), bits(y_dev)), (nfft, B)
        X2 = X.copy()
        X2[:, 3] *= 2.0  # a processed spectrum: the speculation must not serve it
        plan.forward_host(x)
        y2 = plan.inverse_host(X2)
        assert np.array_equal(bits(y2), bits(host(plan.inverse(dev(torch, X2))))), (nfft, B)
        # another call between forward and inverse also voids the speculation
        plan.forward_host(x)
        plan.forward_host(x[::-1].copy())
        y3 = plan.inverse_host(X)
        assert np.array_equal(bits(y3), bits(y_dev)), (nfft, B)


@pytest.mark.parametrize("nfft", [960, 882, 480, 1764, 1920, 1000, 130, 6, 2, 8192, 16384])
def test_fft_host_calls_any_size(pkg, oracle, torch_cuda, nfft):
    """Sizes outside the power-of-two call kernels run on the any-size call
    server (K_call<-1>: fft_any.h's passes, one transform per wave; 16384 has no
    room for its buffers and stages through launches): the launched k_fft_any's
    bits for forward, inverse and the complex forms, the speculated inverse
    served only for the unchanged spectrum, the kissfft restatement within the
    parity tolerance."""
    torch = torch_cuda
    rng = np.random.default_rng(nfft + 5)
    plan = pkg.FftPlan(nfft)
    for B in (1, 3, 4, 9):
        x = rng.standard_normal((B, nfft)).astype(np.float32)
        X = plan.forward_host(x)
        assert np.array_equal(X.view(np.uint32), host(plan.forward(dev(torch, x))).view(np.uint32)), (nfft, B)
        ref = oracle.bench_rfft(x, nfft)
        assert np.linalg.norm(X - ref) <= 1e-6 * np.linalg.norm(ref), (nfft, B)
        y_dev = host(plan.inverse(dev(torch, X)))
        assert np.array_equal(bits(plan.inverse_host(X)), bits(y_dev)), (nfft, B)  # speculated when B <= waves
        X2 = X.copy()
        X2[:, nfft // 4] *= 0.5
        plan.forward_host(x)
        y2 = plan.inverse_host(X2)
        assert np.array_equal(bits(y2), bits(host(plan.inverse(dev(torch, X2))))), (nfft, B)
        assert np.linalg.norm(y_dev - x) <= 1e-5 * np.linalg.norm(x), (nfft, B)
    if nfft <= 8192:
        cp = pkg.FftPlan(nfft, domain=pkg.FFT_COMPLEX)
        z = (rng.standard_normal((3, nfft)) + 1j * rng.standard_normal((3, nfft))).astype(np.complex64)
        Z = cp.forward_complex_host(z)
        assert np.array_equal(Z.view(np.uint32), host(cp.forward_complex(dev(torch, z))).view(np.uint32)), nfft
        zi = cp.inverse_complex_host(Z)
        assert np.array_equal(zi.view(np.uint32), host(cp.inverse_complex(dev(torch, Z))).view(np.uint32)), nfft


def test_fft_host_strides_complex_and_fallback(pkg, oracle, torch_cuda):
    """The reference's stride semantics (kissfft_adapter.cc:97-98, 139-140): batch b
    at b*stride*len, element i at i*stride, untouched elements kept; the complex
    domain; a size without a call-kernel instantiation (staged launches)."""
    torch = torch_cuda
    rng = np.random.default_rng(9)
    n, B, st = 1024, 4, 2
    plan = pkg.FftPlan(n)
    x = rng.standard_normal((B, n * st)).astype(np.float32)
    out = np.full((B, (n // 2 + 1) * st), 7 + 7j, np.complex64)
    plan.forward_host(x, out=out, inc_in=st, inc_out=st)
    dense = plan.forward_host(np.ascontiguousarray(x[:, ::st]))
    assert np.array_equal(np.ascontiguousarray(out[:, ::st]).view(np.uint32), dense.view(np.uint32))
    assert np.all(out[:, 1::st] == 7 + 7j)
    yo = np.full((B, n * st), -3, np.float32)
    plan.inverse_host(np.ascontiguousarray(out[:, ::st]), out=yo, inc_out=st)
    assert np.array_equal(bits(yo[:, ::st]), bits(host(plan.inverse(dev(torch, dense)))))
    assert np.all(yo[:, 1::st] == -3)
    for nc in (128, 512, 2048, 100):
        cp = pkg.FftPlan(nc, domain=pkg.FFT_COMPLEX)
        z = (rng.standard_normal((3, nc)) + 1j * rng.standard_normal((3, nc))).astype(np.complex64)
        Z = cp.forward_complex_host(z)
        assert np.array_equal(Z.view(np.uint32), host(cp.forward_complex(dev(torch, z))).view(np.uint32)), nc
        zi = cp.inverse_complex_host(Z)
        assert np.array_equal(zi.view(np.uint32), host(cp.inverse_complex(dev(torch, Z))).view(np.uint32)), nc
        assert np.linalg.norm(zi - z) <= 1e-5 * np.linalg.norm(z), nc
    p960 = pkg.FftPlan(960)  # mixed radix: the any-size call server
    x = rng.standard_normal((2, 960)).astype(np.float32)
    X = p960.forward_host(x)
    assert np.array_equal(X.view(np.uint32), host(p960.forward(dev(torch, x))).view(np.uint32))
    assert np.array_equal(bits(p960.inverse_host(X)), bits(host(p960.inverse(dev(torch, X)))))
    with pytest.raises(RuntimeError):
        plan.forward_complex_host(np.zeros((1, n), np.complex64))


def test_ola_host_calls_speculated_produce(pkg, oracle, torch_cuda):
    """OLAAccumulator host calls on the call kernel: produce(H) after every push
    (served from the block speculated after the push), produce with other counts
    (real calls), host / device-form calls interleaved on one object -- all
    bit-identical to the oracle's OLAAccumulator restatement."""
    torch = torch_cuda
    n, h, C = 1024, 256, 2
    rng = np.random.default_rng(21)
    w = oracle.window(oracle.HANN, n)
    cfg = pkg.OLAConfig(sample_rate=48000, frame_size=n, hop_size=h, channels=C, eps=1e-8,
                        apply_window_inside=True)
    ola = pkg.OLAAccumulator(cfg)
    ola.set_window(w)
    ref = oracle.Ola(n, h, C, eps=1e-8, inside=True)
    ref.set_window(w)
    outs, refs = [], []
    for k in range(60):
        fr = rng.standard_normal((n, C)).astype(np.float32)
        if k % 7 == 3:  # a device-form push in between
            ola.push_frame_AoS_device(dev(torch, fr), None, k * h, 0, n, 1.0)
        else:
            ola.push_frame_AoS(fr, None, k * h, 0, n, 1.0)
        ref.push_frame_aos(fr, k * h, 0, n, 1.0)
        m = h if k % 5 else (h // 2 if k % 10 else 3 * h)
        got, chans = ola.produce(m)
        outs.append([c[:got] for c in chans])
        refs.append(ref.produce(m))
    for a, b in zip(outs, refs):
        assert len(a) == len(b)
        for ca, cb in zip(a, b):
            assert ca.shape == cb.shape and np.array_equal(bits(ca), bits(cb))
    assert ola.produced_samples() == ref.produced and ola.read_pos() == ref.read_pos


@pytest.mark.gpu
@pytest.mark.parametrize("n,h", [(1024, 256), (960, 240), (882, 441)])
def test_chained_speculation_hits_and_misses(pkg, oracle, torch_cuda, n, h):
    """The e2e loop's rhythm (forward -> inverse -> push_frame_AoS(inverse) ->
    produce(H)) on one FFT plan and one mono OLA object, with the rhythm broken
    on purpose: a pushed frame one bit off the speculated inverse, another gain,
    another produce count, an extra forward between inverse and push, a push at
    an unexpected position.  Every produce is bit-identical to the oracle's
    OLAAccumulator fed the frames actually pushed, whichever of the chained,
    speculated or computed paths served it.  960 and 882 run on the any-size
    call server (fft_any.h), which the OLA object shares with the FFT plan."""
    rng = np.random.default_rng(33)
    w = oracle.window(oracle.HANN, n)
    fft = pkg.FftPlan(n, pkg.FFT_REAL)
    cfg = pkg.OLAConfig(sample_rate=48000, frame_size=n, hop_size=h, channels=1, eps=1e-8,
                        apply_window_inside=True)
    ola = pkg.OLAAccumulator(cfg)
    ola.set_window(w)
    ref = oracle.Ola(n, h, 1, eps=1e-8, inside=True)
    ref.set_window(w)
    start = 0
    for k in range(96):
        x = (rng.standard_normal(n) * w).astype(np.float32)
        y = fft.inverse_host(fft.forward_host(x[None]))[0]
        case = k % 8
        gain, m = 1.0, h
        if case == 3:
            y = y.copy()
            y[k % n] = np.nextafter(y[k % n], np.float32(np.inf))  # one bit off
        elif case == 4:
            gain = 0.5
        elif case == 5:
            m = h // 2 if k % 16 == 5 else 2 * h
        elif case == 6:
            fft.forward_host(rng.standard_normal((1, n)).astype(np.float32))  # an unrelated call
        elif case == 7 and k % 16 == 7:
            start += 3  # a push off the rhythm
        ola.push_frame_AoS(y, None, start, 0, n, gain)
        ref.push_frame_aos(y, start, 0, n, gain)
        got, chans = ola.produce(m)
        want = ref.produce(m)
        assert got == len(want[0]), k
        assert np.array_equal(bits(chans[0][:got]), bits(want[0])), k
        start += h
    assert ola.produced_samples() == ref.produced and ola.read_pos() == ref.read_pos


@pytest.mark.gpu
def test_objects_constructed_in_a_loop_reuse_pooled_resources(pkg, oracle, torch_cuda):
    """performance_benchmark.cc:181-210 constructs FrameQueue, OLAAccumulator and
    an FFT plan per iteration: with the resource pools (streams, pinned blocks,
    stream-ordered device memory) every reconstructed object still starts clean
    -- a zeroed ring, its own frames -- and each iteration's output equals the
    oracle's OLA fed the same frames, bit for bit."""
    n, h, L = 1024, 512, 8192
    rng = np.random.default_rng(55)
    w = oracle.window(oracle.HANN, n)
    for it in range(24):
        x = rng.standard_normal(L).astype(np.float32)
        fq = pkg.FrameQueue(x, n, h, True, pkg.PAD_CONSTANT)
        fft = pkg.FftPlan(n, pkg.FFT_REAL)
        cfg = pkg.OLAConfig(sample_rate=48000, frame_size=n, hop_size=h, channels=1, eps=1e-8,
                            apply_window_inside=True)
        ola = pkg.OLAAccumulator(cfg)
        ola.set_window(w)
        ref = oracle.Ola(n, h, 1, eps=1e-8, inside=True)
        ref.set_window(w)
        for i in range(fq.getNumFrames()):
            y = fft.inverse_host(fft.forward_host(fq.getFrame(i)[None]))[0]
            ola.push_frame_AoS(y, None, i * h, 0, n, 1.0)
            ref.push_frame_aos(y, i * h, 0, n, 1.0)
            got, chans = ola.produce(h)
            want = ref.produce(h)
            assert got == len(want[0])
            assert np.array_equal(bits(chans[0][:got]), bits(want[0])), (it, i)
        ola.close()
        fft.close()
        fq.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n,h", [(1024, 256), (960, 240)])
def test_chained_push_survives_call_server_idle_exit(pkg, oracle, torch_cuda, n, h):
    """The chained push rides on the next request (the call kernel kept the frame
    in LDS).  The call kernel exits after 20 ms without a request; a real-time
    48 kHz stream waits a whole hop (21 ms at 1024) between frames, so the commit
    often runs in a relaunched kernel whose LDS no longer holds the frame.  It must
    then read the frame's copy from the speculation slot: with pauses longer than
    the idle timeout at every point of the rhythm, every produce is bit-identical
    to the oracle's OLAAccumulator."""
    import time
    rng = np.random.default_rng(77)
    w = oracle.window(oracle.HANN, n)
    fft = pkg.FftPlan(n, pkg.FFT_REAL)
    cfg = pkg.OLAConfig(sample_rate=48000, frame_size=n, hop_size=h, channels=1, eps=1e-8,
                        apply_window_inside=True)
    ola = pkg.OLAAccumulator(cfg)
    ola.set_window(w)
    ref = oracle.Ola(n, h, 1, eps=1e-8, inside=True)
    ref.set_window(w)
    for k in range(24):
        x = (rng.standard_normal(n) * w).astype(np.float32)
        spec = fft.forward_host(x[None])
        if k % 4 == 1:
            time.sleep(0.03)
        y = fft.inverse_host(spec)[0]
        if k % 4 == 2:
            time.sleep(0.03)
        ola.push_frame_AoS(y, None, k * h, 0, n, 1.0)
        ref.push_frame_aos(y, k * h, 0, n, 1.0)
        if k % 4 == 3:
            time.sleep(0.03)
        got, chans = ola.produce(h)
        want = ref.produce(h)
        assert got == len(want[0]), k
        assert np.array_equal(bits(chans[0][:got]), bits(want[0])), k
        if k % 2 == 0:
            time.sleep(0.03)  # the commit of this frame runs after an idle exit
    assert ola.produced_samples() == ref.produced


@pytest.mark.gpu
def test_speculation_dropped_when_shared_server_grows(pkg, oracle, torch_cuda):
    """A wide OLA object of the same frame size grows the shared call server
    (reallocating its arenas) between a forward and the push of its inverse: the
    speculation recorded before the growth points into freed memory and must not
    be used; the narrow object's output stays bit-identical to the oracle."""
    n, h = 1024, 256
    rng = np.random.default_rng(78)
    w = oracle.window(oracle.HANN, n)
    fft = pkg.FftPlan(n, pkg.FFT_REAL)
    mk = lambda c: pkg.OLAConfig(sample_rate=48000, frame_size=n, hop_size=h, channels=c, eps=1e-8,
                                 apply_window_inside=True)
    ola = pkg.OLAAccumulator(mk(1))
    ola.set_window(w)
    ref = oracle.Ola(n, h, 1, eps=1e-8, inside=True)
    ref.set_window(w)
    for k in range(12):
        x = (rng.standard_normal(n) * w).astype(np.float32)
        y = fft.inverse_host(fft.forward_host(x[None]))[0]
        if k in (3, 7):
            c = 24 + 8 * k  # wider than any object before: the server grows
            wide = pkg.OLAAccumulator(mk(c))
            wide.set_window(w)
            wide.push_frame_AoS(rng.standard_normal(n * c).astype(np.float32), None, 0, 0, n, 1.0)
            wide.produce(h)
            wide.close()
        ola.push_frame_AoS(y, None, k * h, 0, n, 1.0)
        ref.push_frame_aos(y, k * h, 0, n, 1.0)
        got, chans = ola.produce(h)
        want = ref.produce(h)
        assert np.array_equal(bits(chans[0][:got]), bits(want[0])), k


@pytest.mark.gpu
def test_device_kernels_bit_exact_vs_reference_build(pkg, torch_cuda, ref_tables):
    """The batched device forms and the host-pointer forms of dsp::axpy /
    axpy_windowed / normalize_and_clear against the outputs of the reference's
    own kernels.cc scalar kernels compiled here (ref_tables.npz k_* fixtures):
    bit for bit, where kernels_test.cc:214-429 allows the Highway versions 1 ULP."""
    import re
    torch = torch_cuda
    n_checked = 0
    for key in ref_tables.files:
        m = re.match(r"(k_n(\d+)_g\d)_dst$", key)
        if not m or int(m[2]) == 0:
            continue
        k = m[1]
        dst, src, win, norm = (ref_tables[f"{k}_{s}"] for s in ("dst", "src", "win", "norm"))
        g = float(ref_tables[f"{k}_gain"][0])
        eps = float(ref_tables[f"{k}_eps"][0])
        d = dev(torch, dst)
        pkg.axpy(d, dev(torch, src), g)
        assert np.array_equal(bits(host(d)), bits(ref_tables[f"{k}_axpy"])), k
        d = dev(torch, dst)
        pkg.axpy(d, dev(torch, src), g, dev(torch, win))
        assert np.array_equal(bits(host(d)), bits(ref_tables[f"{k}_axpyw"])), k
        acc, out = dev(torch, dst), torch.empty(dst.size, dtype=torch.float32, device="cuda")
        pkg.normalize_and_clear(out, acc, dev(torch, norm), eps)
        assert np.array_equal(bits(host(out)), bits(ref_tables[f"{k}_out"])), k
        assert np.array_equal(bits(host(acc)), bits(ref_tables[f"{k}_acc"])), k
        h = dst.copy()
        pkg.axpy_host(h, src, g, win)
        assert np.array_equal(bits(h), bits(ref_tables[f"{k}_axpyw"])), k
        ha, ho = dst.copy(), np.empty_like(dst)
        pkg.normalize_and_clear_host(ho, ha, norm, eps)
        assert np.array_equal(bits(ho), bits(ref_tables[f"{k}_out"])), k
        n_checked += 1
    assert n_checked == 24


def _e2e_loop(pkg, oracle, x, n, h, breaks=None, window=None):
    """bench/e2e_benchmark.cc:138-186 through the drop-in objects, streaming-
    interleaved; `breaks` maps a frame index to a deviation from the rhythm.
    Returns (spectra, inverse frames, produced blocks, pushed frames)."""
    breaks = breaks or {}
    w = pkg.window_table(pkg.HANN, n) if window is None else window
    fr = pkg.Framer()
    fr.set_params(n, h, 1, pkg.ZERO_PAD)
    fft = pkg.FftPlan(n, pkg.FFT_REAL)
    cfg = pkg.OLAConfig(sample_rate=48000, frame_size=n, hop_size=h, channels=1, eps=1e-8,
                        apply_window_inside=True)
    ola = pkg.OLAAccumulator(cfg)
    ola.set_window(w)
    fr.push(x)
    specs, invs, outs, pushed = [], [], [], []
    k = 0
    start = 0
    while True:
        f = fr.pop()
        if f is None:
            break
        p = (f * w).astype(np.float32)
        b = breaks.get(k)
        if b == "input":
            p = p.copy()
            p[k % n] = np.nextafter(p[k % n], np.float32(np.inf))
        X = fft.forward_host(p[None])
        if b == "extra_forward":
            fft.forward_host((p * np.float32(0.5))[None])
        y = fft.inverse_host(X)[0]
        gain = 0.5 if b == "gain" else 1.0
        if b == "device_push":
            import torch
            ola.push_frame_AoS_device(torch.from_numpy(y.copy()).cuda(), None, start, 0, n, gain)
            torch.cuda.synchronize()
        else:
            ola.push_frame_AoS(y, None, start, 0, n, gain)
        m = h // 2 if b == "short_produce" else h
        got, chans = ola.produce(m)
        specs.append(np.asarray(X).copy())
        invs.append(y.copy())
        outs.append(chans[0][:got].copy())
        pushed.append((y.copy(), start, gain, m))
        start += h
        k += 1
    ola.close()
    fft.close()
    fr.close()
    return specs, invs, outs, pushed


def _oracle_outputs(oracle, n, h, w, pushed):
    ref = oracle.Ola(n, h, 1, eps=1e-8, inside=True)
    ref.set_window(w)
    out = []
    for y, start, gain, m in pushed:
        ref.push_frame_aos(y, start, 0, n, gain)
        out.append(ref.produce(m)[0])
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("n,h", [(1024, 256), (1024, 512), (960, 240), (882, 441)])
def test_batched_loop_equals_per_call_path(pkg, oracle, torch_cuda, n, h):
    """The e2e loop served from the batched speculation gives, call by call, the
    bits the per-call path (crlot_set_call_speculation(1)) gives: spectra,
    inverse frames and every produced block; and the produced blocks are the
    oracle OLAAccumulator's fed the same frames, bit for bit.  The counters show
    the batch really served the loop."""
    x = oracle.synth(48_000, n + h)
    try:
        pkg.set_call_speculation(1)
        a = _e2e_loop(pkg, oracle, x, n, h)
        pkg.set_call_speculation(2)
        s0 = pkg.call_speculation_stats()
        b = _e2e_loop(pkg, oracle, x, n, h)
        s1 = pkg.call_speculation_stats()
    finally:
        pkg.set_call_speculation(2)
    F = len(a[0])
    assert len(b[0]) == F
    for k in range(F):
        assert np.array_equal(bits(a[0][k]), bits(b[0][k])), ("spectrum", k)
        assert np.array_equal(bits(a[1][k]), bits(b[1][k])), ("inverse", k)
        assert np.array_equal(bits(a[2][k]), bits(b[2][k])), ("produce", k)
    ref = _oracle_outputs(oracle, n, h, pkg.window_table(pkg.HANN, n), b[3])
    for k in range(F):
        assert np.array_equal(bits(b[2][k]), bits(ref[k])), ("oracle", k)
    served = {key: s1[key] - s0[key] for key in s1}
    assert served["batches"] == 1 and served["forwards"] == F and served["inverses"] == F, served
    assert served["pushes"] == F and served["produces"] == F and served["rebuilds"] == 0, served


def _pipeline_loop(pkg, x, n, h, interleaved=True, tamper=None, gain=1.0):
    """bench/performance_benchmark.cc:174-246 through the drop-in objects (the
    harness/pipeline_bench loop): FrameQueue(x, N, H, centre) -> per frame:
    getFrame -> forward -> inverse -> add_frame_SoA(window, i H) [-> produce(H)]
    -> produce(H) until the signal length.  `tamper` = frame index whose forward
    input is nudged by one ulp (the batch must not serve it)."""
    L = x.size
    q = pkg.FrameQueue(x, n, h, center=True)
    w = pkg.window_table(pkg.HANN, n)
    fft = pkg.FftPlan(n, pkg.FFT_REAL)
    cfg = pkg.OLAConfig(sample_rate=48000, frame_size=n, hop_size=h, channels=1, eps=1e-8,
                        apply_window_inside=True)
    ola = pkg.OLAAccumulator(cfg)
    ola.set_window(w)
    specs, invs, outs = [], [], []
    total = 0
    for i in range(q.getNumFrames()):
        f = q.getFrame(i)
        if i == tamper:
            f = f.copy()
            f[7] = np.nextafter(f[7], np.float32(np.inf))
        X = fft.forward_host(f[None])
        y = fft.inverse_host(X)[0]
        ola.add_frame_SoA([y], w, i * h, 0, n, gain)
        specs.append(np.asarray(X).copy())
        invs.append(y.copy())
        if interleaved and total < L:
            got, chans = ola.produce(h)
            outs.append(chans[0][:got].copy())
            total += got
    while total < L:
        got, chans = ola.produce(h)
        if got == 0:
            break
        outs.append(chans[0][:got].copy())
        total += got
    ola.close()
    q.close()
    return specs, invs, np.concatenate(outs) if outs else np.zeros(0, np.float32)


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,L", [(1024, 512, 16384), (1024, 256, 20_000), (960, 240, 9_600), (256, 64, 6_000),
                                   (512, 128, 8_000), (2048, 512, 30_000), (4096, 1024, 50_000)])
@pytest.mark.parametrize("interleaved", [True, False])
def test_batched_pipeline_loop_equals_per_call_path(pkg, oracle, torch_cuda, n, h, L, interleaved):
    """The reference's second pipeline (performance_benchmark.cc: FrameQueue frames,
    no analysis window, add_frame_SoA, the trailing produces) served from the
    batched speculation -- the FrameQueue read last is its source -- gives the
    per-call path's bits call by call (spectra, inverse frames, every produced
    sample, the tail included) and the oracle OLAAccumulator's; the counters show
    the batch served it (256-2048: the fused forward+inverse launch; 960 and
    4096: the two-launch chain).  In the harness's literal order (every push first) the
    ring wraps onto unread slots; the batch serves that order too (the wrapped
    slots, k_ola_gather_wrap): same bits."""
    x = oracle.synth(L, n + h)
    try:
        pkg.set_call_speculation(1)
        a = _pipeline_loop(pkg, x, n, h, interleaved)
        pkg.set_call_speculation(2)
        s0 = pkg.call_speculation_stats()
        b = _pipeline_loop(pkg, x, n, h, interleaved)
        s1 = pkg.call_speculation_stats()
        c = _pipeline_loop(pkg, x, n, h, interleaved, tamper=5)
        pkg.set_call_speculation(1)
        c1 = _pipeline_loop(pkg, x, n, h, interleaved, tamper=5)
    finally:
        pkg.set_call_speculation(2)
    F = len(a[0])
    assert len(b[0]) == F
    for k in range(F):
        assert np.array_equal(bits(a[0][k]), bits(b[0][k])), ("spectrum", k)
        assert np.array_equal(bits(a[1][k]), bits(b[1][k])), ("inverse", k)
    assert np.array_equal(bits(a[2]), bits(b[2]))
    assert np.array_equal(bits(c[2]), bits(c1[2]))  # a frame off the rhythm: the per-call bits again
    # the oracle OLAAccumulator fed the same inverse frames (add_frame_SoA == push_frame_AoS for mono)
    ref = oracle.Ola(n, h, 1, eps=1e-8, inside=True)
    ref.set_window(pkg.window_table(pkg.HANN, n))
    outs, total = [], 0
    for i, y in enumerate(b[1]):
        ref.push_frame_aos(y, i * h, 0, n, 1.0)
        if interleaved and total < L:
            o = ref.produce(h)[0]
            outs.append(o)
            total += o.size
    while total < L:
        o = ref.produce(h)[0]
        if o.size == 0:
            break
        outs.append(o)
        total += o.size
    assert np.array_equal(bits(b[2]), bits(np.concatenate(outs)))
    served = {key: s1[key] - s0[key] for key in s1}
    assert served["batches"] == 1 and served["forwards"] == F and served["inverses"] == F, served
    # every push and produce served, in either order: no ring was rebuilt
    assert served["pushes"] == F and served["rebuilds"] == 0 and served["produces"] > 0, served


@pytest.mark.gpu
@pytest.mark.parametrize("interleaved", [True, False])
def test_batched_pipeline_other_gain(pkg, oracle, torch_cuda, interleaved):
    """Pushes with gain 0.5: the overlap-add the batch computed with its chain
    (gain 1, for the OLA object whose window was set last) is not used; the
    attach computes it with the pushes' gain: the per-call path's bits."""
    n, h, L = 1024, 512, 16384
    x = oracle.synth(L, 13)
    try:
        pkg.set_call_speculation(1)
        a = _pipeline_loop(pkg, x, n, h, interleaved, gain=0.5)
        pkg.set_call_speculation(2)
        s0 = pkg.call_speculation_stats()
        b = _pipeline_loop(pkg, x, n, h, interleaved, gain=0.5)
        s1 = pkg.call_speculation_stats()
    finally:
        pkg.set_call_speculation(2)
    assert np.array_equal(bits(a[2]), bits(b[2]))
    served = {key: s1[key] - s0[key] for key in s1}
    assert served["pushes"] == len(a[0]) and served["rebuilds"] == 0 and served["produces"] > 0, served


@pytest.mark.gpu
@pytest.mark.parametrize("reads", [0, 3, 30])
def test_wrapped_batch_rebuilds_the_ring_mid_read(pkg, oracle, torch_cuda, reads):
    """The push-everything-first order, then `reads` produces of H, then a call
    the batch did not predict (one more push, past the signal): the ring is
    rebuilt from the wrapped slots with the ones already read cleared, and every
    later produce has the per-call path's bits (reads = 0: the rebuild happens
    before any wrapped produce, from the frames)."""
    n, h, L = 1024, 512, 16384
    x = oracle.synth(L, 11)
    extra = oracle.synth(n, 12)

    def run():
        q = pkg.FrameQueue(x, n, h, center=True)
        w = pkg.window_table(pkg.HANN, n)
        fft = pkg.FftPlan(n, pkg.FFT_REAL)
        cfg = pkg.OLAConfig(sample_rate=48000, frame_size=n, hop_size=h, channels=1, eps=1e-8,
                            apply_window_inside=True)
        ola = pkg.OLAAccumulator(cfg)
        ola.set_window(w)
        F = q.getNumFrames()
        for i in range(F):
            y = fft.inverse_host(fft.forward_host(q.getFrame(i)[None]))[0]
            ola.add_frame_SoA([y], w, i * h, 0, n, 1.0)
        outs = []
        for _ in range(reads):
            got, chans = ola.produce(h)
            outs.append(chans[0][:got].copy())
        ola.add_frame_SoA([extra], w, F * h, 0, n, 1.0)
        for _ in range(60):
            got, chans = ola.produce(h)
            if got == 0:
                break
            outs.append(chans[0][:got].copy())
        ola.close()
        q.close()
        return np.concatenate(outs)

    try:
        pkg.set_call_speculation(1)
        a = run()
        pkg.set_call_speculation(2)
        s0 = pkg.call_speculation_stats()
        b = run()
        s1 = pkg.call_speculation_stats()
    finally:
        pkg.set_call_speculation(2)
    assert a.size == b.size and np.array_equal(bits(a), bits(b))
    served = {key: s1[key] - s0[key] for key in s1}
    assert served["batches"] == 1 and served["rebuilds"] == 1 and served["produces"] == reads, served


@pytest.mark.gpu
@pytest.mark.parametrize("brk", ["input", "extra_forward", "gain", "short_produce", "device_push"])
def test_batched_loop_falls_back_on_a_broken_rhythm(pkg, oracle, torch_cuda, brk):
    """One call off the predicted rhythm mid-stream (a forward input one bit off,
    an unrelated forward, another gain, a shorter produce, a push through the
    device form): the batch ends there, the OLA ring is rebuilt from the frames
    it was served, and every later call (the per-call path, and a new batch
    where the rhythm resumes) still gives the per-call path's bits and the
    oracle's blocks."""
    n, h = 1024, 256
    x = oracle.synth(48_000, 7)
    breaks = {60: brk, 61: brk} if brk == "short_produce" else {60: brk}
    try:
        pkg.set_call_speculation(1)
        a = _e2e_loop(pkg, oracle, x, n, h, breaks)
        pkg.set_call_speculation(2)
        s0 = pkg.call_speculation_stats()
        b = _e2e_loop(pkg, oracle, x, n, h, breaks)
        s1 = pkg.call_speculation_stats()
    finally:
        pkg.set_call_speculation(2)
    F = len(a[0])
    for k in range(F):
        assert np.array_equal(bits(a[1][k]), bits(b[1][k])), ("inverse", k)
        assert np.array_equal(bits(a[2][k]), bits(b[2][k])), ("produce", k)
    ref = _oracle_outputs(oracle, n, h, pkg.window_table(pkg.HANN, n), b[3])
    for k in range(F):
        assert np.array_equal(bits(b[2][k]), bits(ref[k])), ("oracle", k)
    served = {key: s1[key] - s0[key] for key in s1}
    if brk == "short_produce":  # still inside the finalised blocks: served, nothing rebuilt
        assert served["rebuilds"] == 0 and served["produces"] == F, served
    else:
        assert served["rebuilds"] == 1 and served["forwards"] >= 60, served


@pytest.mark.gpu
def test_batched_loop_keeps_ring_aliasing_of_the_harness_order(pkg, oracle, torch_cuda):
    """bench/e2e_benchmark.cc's literal order pushes every frame before the
    produce loop, so the 6144-sample OLA ring wraps onto unread data,
    and its produce(T) reads past the ring's capacity (RingBuffer::split clamps
    it: R outputs, the rest of the caller's buffer untouched).  The batch serves
    both (the wrapped slots, k_ola_gather_wrap), keeping the reference's
    aliasing: the same bits as the per-call path -- the untouched tail included --
    and as the oracle OLAAccumulator fed the same calls."""
    n, h = 1024, 256
    x = oracle.synth(48_000, 11)
    w = pkg.window_table(pkg.HANN, n)

    def run():
        fr = pkg.Framer()
        fr.set_params(n, h, 1, pkg.ZERO_PAD)
        fft = pkg.FftPlan(n, pkg.FFT_REAL)
        ola = pkg.OLAAccumulator(pkg.OLAConfig(sample_rate=48000, frame_size=n, hop_size=h, channels=1,
                                               eps=1e-8, apply_window_inside=True))
        ola.set_window(w)
        fr.push(x)
        frames, k = [], 0
        while True:
            f = fr.pop()
            if f is None:
                break
            y = fft.inverse_host(fft.forward_host((f * w).astype(np.float32)[None]))[0]
            ola.push_frame_AoS(y, None, k * h, 0, n, 1.0)
            frames.append(y.copy())
            k += 1
        out = []
        while True:
            got, chans = ola.produce(48_000, [np.full(48_000, 7.0, np.float32)])
            if got == 0 or sum(len(o) for o in out) >= 48_000:
                break
            out.append(chans[0][:got].copy())
        ola.close()
        fft.close()
        fr.close()
        return frames, np.concatenate(out)

    try:
        pkg.set_call_speculation(1)
        fa, ya = run()
        pkg.set_call_speculation(2)
        s0 = pkg.call_speculation_stats()
        fb, yb = run()
        s1 = pkg.call_speculation_stats()
    finally:
        pkg.set_call_speculation(2)
    assert all(np.array_equal(bits(a), bits(b)) for a, b in zip(fa, fb))
    assert np.array_equal(bits(ya), bits(yb))
    assert np.all(yb[6144:48_000] == 7.0)  # the clamped read left the caller's tail alone
    served = {key: s1[key] - s0[key] for key in s1}
    assert served["pushes"] == len(fb) and served["produces"] == 2 and served["rebuilds"] == 0, served
    ref = oracle.Ola(n, h, 1, eps=1e-8, inside=True)
    ref.set_window(w)
    for k, y in enumerate(fb):
        ref.push_frame_aos(y, k * h, 0, n, 1.0)
    r = np.full(48_000, 7.0, np.float32)
    got = ref.produce_into(48_000, [r])
    assert np.array_equal(bits(yb[:got]), bits(r[:got]))


# ---- bounded batches: windows of at most kBatchWindow frames

def _e2e_digest(pkg, x, n, h, breaks=None, limit=None):
    """The e2e loop (streaming-interleaved) without keeping its outputs: a digest
    of every spectrum, inverse frame and produced block, and the frame count.
    `breaks`: frame -> "input" (forward input one ulp off); `limit`: frames run."""
    import hashlib
    breaks = breaks or {}
    w = pkg.window_table(pkg.HANN, n)
    fr = pkg.Framer()
    fr.set_params(n, h, 1, pkg.ZERO_PAD)
    fft = pkg.FftPlan(n, pkg.FFT_REAL)
    ola = pkg.OLAAccumulator(pkg.OLAConfig(sample_rate=48000, frame_size=n, hop_size=h, channels=1, eps=1e-8,
                                           apply_window_inside=True))
    ola.set_window(w)
    fr.push(x)
    dig = hashlib.sha256()
    k = 0
    while limit is None or k < limit:
        f = fr.pop()
        if f is None:
            break
        p = (f * w).astype(np.float32)
        if breaks.get(k) == "input":
            p[k % n] = np.nextafter(p[k % n], np.float32(np.inf))
        X = fft.forward_host(p[None])
        y = fft.inverse_host(X)[0]
        ola.push_frame_AoS(y, None, k * h, 0, n, 1.0)
        got, chans = ola.produce(h)
        for a in (np.asarray(X), y, chans[0][:got]):
            dig.update(np.ascontiguousarray(a).view(np.uint32).tobytes())
        k += 1
    ola.close()
    fft.close()
    fr.close()
    return dig.hexdigest(), k


def _spec_delta(pkg, run):
    s0 = pkg.call_speculation_stats_ex()
    out = run()
    s1 = pkg.call_speculation_stats_ex()
    return out, {key: s1[key] - s0[key] for key in s1}


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,T", [(1024, 256, 160_000), (960, 240, 130_000), (1024, 512, 300_000)])
def test_batched_loop_spans_windows(pkg, oracle, torch_cuda, n, h, T):
    """A signal longer than one batch window: the batch runs window after window
    (each continuation carries the last frames' inverse outputs over for the OLA
    object), and every call still gives the per-call path's bits and the oracle
    OLAAccumulator's blocks."""
    x = oracle.synth(T, n + 3 * h)
    try:
        pkg.set_call_speculation(1)
        a = _e2e_loop(pkg, oracle, x, n, h)
        pkg.set_call_speculation(2)
        b, served = _spec_delta(pkg, lambda: _e2e_loop(pkg, oracle, x, n, h))
    finally:
        pkg.set_call_speculation(2)
    F = len(a[0])
    K = pkg.call_batch_capacity()["window_frames"]
    assert F > K and len(b[0]) == F
    for k in range(F):
        assert np.array_equal(bits(a[0][k]), bits(b[0][k])), ("spectrum", k)
        assert np.array_equal(bits(a[1][k]), bits(b[1][k])), ("inverse", k)
        assert np.array_equal(bits(a[2][k]), bits(b[2][k])), ("produce", k)
    ref = _oracle_outputs(oracle, n, h, pkg.window_table(pkg.HANN, n), b[3])
    for k in range(F):
        assert np.array_equal(bits(b[2][k]), bits(ref[k])), ("oracle", k)
    assert served["batches"] == 1 and served["windows"] == (F - 1) // K, served
    assert served["forwards"] == F and served["inverses"] == F and served["pushes"] == F, served
    assert served["produces"] == F and served["rebuilds"] == 0 and served["frames"] == F, served


@pytest.mark.gpu
def test_batched_loop_ten_minutes_bounded_memory(pkg, oracle, torch_cuda):
    """bench/e2e_benchmark.cc:144 pushes one second of audio whole into the
    Framer; here ten minutes (28.8 M samples, 112 500 frames at 1024/256).  The
    batch works window by window: the pinned and device memory it holds stay at
    one window's worth (an unbounded batch would pin ~0.9 GB here), and every
    spectrum, inverse frame and produced block equals the per-call path's."""
    n, h, T = 1024, 256, 48_000 * 600
    rng = np.random.default_rng(600)
    x = (rng.standard_normal(T) * 0.1).astype(np.float32)
    try:
        pkg.set_call_speculation(1)
        a = _e2e_digest(pkg, x, n, h)
        pkg.set_call_speculation(2)
        b, served = _spec_delta(pkg, lambda: _e2e_digest(pkg, x, n, h))
    finally:
        pkg.set_call_speculation(2)
    assert a == b, (a, b)
    F = a[1]
    cap = pkg.call_batch_capacity()
    K = cap["window_frames"]
    assert served["frames"] == F and served["windows"] == (F - 1) // K and served["rebuilds"] == 0, served
    whole = F * (2 * n + 2) * 4  # spectra + inverse frames of the whole signal
    assert cap["pinned_peak"] <= 128 << 20 < whole, cap
    assert cap["pinned_bytes"] <= 40 << 20 and cap["device_bytes"] <= 64 << 20, cap
    print(f"\n10-minute loop: {F} frames, {served['windows']} window continuations, batch memory {cap}")


@pytest.mark.gpu
def test_batched_loop_broken_at_frame_2_does_bounded_work(pkg, oracle, torch_cuda):
    """A caller that breaks the rhythm at frame 2 of a long signal pays for at most
    one window per batch start, not for the whole signal."""
    n, h = 1024, 256
    x = oracle.synth(48_000 * 60, 5)
    (dig, k), served = _spec_delta(pkg, lambda: _e2e_digest(pkg, x, n, h, breaks={2: "input"}, limit=12))
    K = pkg.call_batch_capacity()["window_frames"]
    assert k == 12 and served["batches"] == 2 and served["rebuilds"] == 1, served
    assert served["frames"] <= 2 * K < (x.size // h), served
    try:
        pkg.set_call_speculation(1)
        ref = _e2e_digest(pkg, x, n, h, breaks={2: "input"}, limit=12)
    finally:
        pkg.set_call_speculation(2)
    assert ref == (dig, k)


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,count", [(2000, 500, 1), (2200, 550, 1000)])
def test_batched_loop_declines_when_allocation_fails(pkg, oracle, torch_cuda, n, h, count):
    """An allocation failure inside the speculation (injected: the next `count`
    batch buffer allocations fail) is not the caller's error: the forward takes
    the ordinary path and returns the right spectrum.  Frame sizes no other test
    batches, so their buffers are allocated here."""
    x = oracle.synth(40_000, 13)
    try:
        pkg.set_call_speculation(1)
        a = _e2e_digest(pkg, x, n, h)
        pkg.set_call_speculation(2)
        pkg.test_inject(pkg.INJECT_BATCH_ALLOC, count)
        b, served = _spec_delta(pkg, lambda: _e2e_digest(pkg, x, n, h))
    finally:
        pkg.test_inject(pkg.INJECT_BATCH_ALLOC, 0)
        pkg.set_call_speculation(2)
    assert a == b
    assert served["declined"] >= 1, served
    if count == 1:  # the next frame's forward starts the batch
        assert served["batches"] == 1 and served["forwards"] == a[1] - 1, served
    else:
        assert served["batches"] == 0 and served["forwards"] == 0, served


@pytest.mark.gpu
def test_call_server_recovers_after_a_timed_out_request(pkg, oracle, torch_cuda):
    """a request that times out used to disable its (device, size)
    server for the rest of the process.  The timeout path (injected: the wait
    gives up at once while the request completes normally) fails that call
    loudly; once every request submitted before has completed, the server serves
    again, with the right bits."""
    import time
    n = 1024
    rng = np.random.default_rng(77)
    x = rng.standard_normal((1, n)).astype(np.float32)
    fft = pkg.FftPlan(n, pkg.FFT_REAL)
    try:
        pkg.set_call_speculation(1)
        ref = np.asarray(fft.forward_host(x)).copy()
        pkg.test_inject(pkg.INJECT_CALL_TIMEOUT, 1)
        with pytest.raises(Exception):
            fft.forward_host(x)
        time.sleep(0.05)  # the timed-out request finishes on the device
        again = np.asarray(fft.forward_host(x)).copy()
        inv = fft.inverse_host(again)[0]
    finally:
        pkg.test_inject(pkg.INJECT_CALL_TIMEOUT, 0)
        pkg.set_call_speculation(2)
        fft.close()
    assert np.array_equal(bits(again), bits(ref))
    assert np.allclose(inv, x[0], atol=1e-4)


def _e2e_gain_loop(pkg, x, n, h, g):
    """The e2e loop with a spectral step on the host: every bin of each spectrum
    scaled by g[k] between forward and inverse (e2e_benchmark.cc:161-162)."""
    w = pkg.window_table(pkg.HANN, n)
    fr = pkg.Framer()
    fr.set_params(n, h, 1, pkg.ZERO_PAD)
    fft = pkg.FftPlan(n, pkg.FFT_REAL)
    ola = pkg.OLAAccumulator(pkg.OLAConfig(sample_rate=48000, frame_size=n, hop_size=h, channels=1, eps=1e-8,
                                           apply_window_inside=True))
    ola.set_window(w)
    fr.push(x)
    outs, k = [], 0
    while True:
        f = fr.pop()
        if f is None:
            break
        X = np.asarray(fft.forward_host((f * w).astype(np.float32)[None])).copy()
        X[0].real *= g
        X[0].imag *= g
        y = fft.inverse_host(X)[0]
        ola.push_frame_AoS(y, None, k * h, 0, n, 1.0)
        got, chans = ola.produce(h)
        outs.append(chans[0][:got].copy())
        k += 1
    ola.close()
    fft.close()
    fr.close()
    return np.concatenate(outs)


@pytest.mark.gpu
@pytest.mark.parametrize("n,h", [(1024, 256), (960, 240)])
def test_e2e_loop_with_host_spectral_gain(pkg, oracle, torch_cuda, n, h):
    """A real spectral step in the per-frame loop (bench --suite e2e's
    spectral_gain row): the caller scales every bin on the host between forward
    and inverse.  The batch learns the fixed per-bin gain from the first edited
    inverse input (bit for bit: input == spectrum * g), redoes its inverses with
    it, and serves every call; the result is the per-call path's bits, and both
    match the oracle's loop with the same gain within the FFT tolerance."""
    x = oracle.synth(48_000, 21)
    g = (0.5 + 0.5 * np.cos(np.pi * np.arange(n // 2 + 1) / (n // 2))).astype(np.float32)
    try:
        pkg.set_call_speculation(1)
        a = _e2e_gain_loop(pkg, x, n, h, g)
        pkg.set_call_speculation(2)
        b, served = _spec_delta(pkg, lambda: _e2e_gain_loop(pkg, x, n, h, g))
    finally:
        pkg.set_call_speculation(2)
    assert np.array_equal(bits(a), bits(b))
    ref = oracle.roundtrip_gain(x, n, h, g)
    assert a.shape == ref.shape
    d = (a.astype(np.float64) - ref)
    assert np.linalg.norm(d) <= 1e-6 * max(np.linalg.norm(ref), np.linalg.norm(x))  # the parity bar
    assert np.abs(d).max() <= 4e-6 * np.abs(x).max()
    F = a.size // h
    # one frame's products need not pin every bin's gain (a neighbouring float can
    # reproduce them): a few relearns while the ambiguous bins settle, not one a frame
    assert 1 <= served["gains"] <= 8 and served["batches"] == 1 and served["rebuilds"] == 0, served
    assert served["inverses"] == F and served["pushes"] == F and served["produces"] == F, served


@pytest.mark.gpu
def test_e2e_loop_gain_changes_midstream(pkg, oracle, torch_cuda):
    """The spectral gain changes half-way (another fixed gain) and, in a second
    run, turns into an edit that is no per-bin real gain (one bin rotated): the
    batch relearns or falls back, and every call keeps the per-call path's bits."""
    n, h = 1024, 256
    x = oracle.synth(48_000 * 3, 23)
    g1 = (0.5 + 0.5 * np.cos(np.pi * np.arange(n // 2 + 1) / (n // 2))).astype(np.float32)
    g2 = np.linspace(1.5, 0.25, n // 2 + 1).astype(np.float32)

    def run(kind):
        w = pkg.window_table(pkg.HANN, n)
        fr = pkg.Framer()
        fr.set_params(n, h, 1, pkg.ZERO_PAD)
        fft = pkg.FftPlan(n, pkg.FFT_REAL)
        ola = pkg.OLAAccumulator(pkg.OLAConfig(sample_rate=48000, frame_size=n, hop_size=h, channels=1, eps=1e-8,
                                               apply_window_inside=True))
        ola.set_window(w)
        fr.push(x)
        outs, k = [], 0
        while True:
            f = fr.pop()
            if f is None:
                break
            X = np.asarray(fft.forward_host((f * w).astype(np.float32)[None])).copy()
            g = g1 if k < 300 else g2
            X[0].real *= g
            X[0].imag *= g
            if kind == "rotate" and k >= 300:
                X[0][5] = X[0][5] * np.complex64(1j)
            y = fft.inverse_host(X)[0]
            ola.push_frame_AoS(y, None, k * h, 0, n, 1.0)
            got, chans = ola.produce(h)
            outs.append(chans[0][:got].copy())
            k += 1
        ola.close()
        fft.close()
        fr.close()
        return np.concatenate(outs)

    for kind in ("regain", "rotate"):
        try:
            pkg.set_call_speculation(1)
            a = run(kind)
            pkg.set_call_speculation(2)
            b, served = _spec_delta(pkg, lambda: run(kind))
        finally:
            pkg.set_call_speculation(2)
        assert np.array_equal(bits(a), bits(b)), kind
        if kind == "regain":
            assert 2 <= served["gains"] <= 16, served


def _framer_forward_loop(pkg, x, n, h, chunks):
    """Push x into a Framer in `chunks` pieces, popping after each push, and take
    every popped frame (times the Hann table) through IFftPlan::forward: the
    per-frame loop whose pops the batched speculation watches."""
    w = pkg.window_table(pkg.HANN, n)
    fr = pkg.Framer()
    fr.set_params(n, h, 1, pkg.ZERO_PAD)
    fft = pkg.FftPlan(n, pkg.FFT_REAL)
    specs = []
    for piece in np.array_split(x, chunks):
        fr.push(np.ascontiguousarray(piece))
        while True:
            f = fr.pop()
            if f is None:
                break
            specs.append(np.asarray(fft.forward_host((f * w).astype(np.float32)[None])).copy())
    fft.close()
    fr.close()
    return specs


@pytest.mark.gpu
def test_framers_on_two_threads_while_forwards_speculate(pkg, oracle, torch_cuda):
    """the speculation reads the process-wide last-popped
    Framer from any thread's forward while its owner pushes (reallocating the
    buffer), pops (compacting it) or resets it.  Every Framer mutation now holds
    the last-pop lock.  Two threads, each with its own Framer and FFT plan of the
    same size, run the push/pop/forward loop at once; each thread's spectra are the
    bits the same loop gives alone."""
    import threading
    n, h = 1024, 256
    xs = [oracle.synth(48_000, 31 + t) for t in range(2)]
    alone = [_framer_forward_loop(pkg, xs[t], n, h, 24) for t in range(2)]
    for rep in range(3):
        got = [None, None]
        errs = []

        def run(t):
            try:
                got[t] = _framer_forward_loop(pkg, xs[t], n, h, 24)
            except Exception as e:  # reported below: a thread's exception would be lost
                errs.append(e)

        th = [threading.Thread(target=run, args=(t,)) for t in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        assert not errs, errs
        for t in range(2):
            assert len(got[t]) == len(alone[t]), (rep, t)
            for k, (a, b) in enumerate(zip(alone[t], got[t])):
                assert np.array_equal(bits(a), bits(b)), (rep, t, k)


def _random_rhythm_loop(pkg, x, n, h, seed, frames_max=None):
    """The e2e loop with random deviations from the harness rhythm, drawn from
    `seed` (the same script in every mode): a fixed per-bin gain from some frame
    on, one-off spectrum edits (a bin rotated, a bin scaled), a forward asked
    twice, a frame whose push is skipped, produce sizes other than H.  Returns
    every array a call handed back, in call order."""
    rng = np.random.default_rng(seed)
    w = pkg.window_table(pkg.HANN, n)
    fr = pkg.Framer()
    fr.set_params(n, h, 1, pkg.ZERO_PAD)
    fft = pkg.FftPlan(n, pkg.FFT_REAL)
    ola = pkg.OLAAccumulator(pkg.OLAConfig(sample_rate=48000, frame_size=n, hop_size=h, channels=1, eps=1e-8,
                                           apply_window_inside=True))
    ola.set_window(w)
    fr.push(x)
    g = (0.5 + 0.5 * np.cos(np.pi * np.arange(n // 2 + 1) / (n // 2))).astype(np.float32)
    gain_from = int(rng.integers(20, 200)) if rng.random() < 0.5 else None
    got, k = [], 0
    while frames_max is None or k < frames_max:
        f = fr.pop()
        if f is None:
            break
        p = (f * w).astype(np.float32)[None]
        X = np.asarray(fft.forward_host(p)).copy()
        r = rng.random()
        if r < 0.03:  # the same forward again
            X = np.asarray(fft.forward_host(p)).copy()
        got.append(X.copy())
        if gain_from is not None and k >= gain_from:
            X[0].real *= g
            X[0].imag *= g
        r = rng.random()
        if r < 0.03:
            X[0][int(rng.integers(1, n // 2))] *= np.complex64(1j)
        elif r < 0.05:
            X[0][int(rng.integers(0, n // 2 + 1))] *= np.float32(1.5)
        y = np.asarray(fft.inverse_host(X))[0].copy()
        got.append(y)
        if rng.random() >= 0.02:  # (else the frame's push is skipped)
            ola.push_frame_AoS(y, None, k * h, 0, n, 1.0)
        r = rng.random()
        m = h if r < 0.9 else (h // 2 if r < 0.95 else 2 * h)
        cnt, chans = ola.produce(m)
        got.append(chans[0][:cnt].copy())
        k += 1
    ola.close()
    fft.close()
    fr.close()
    return got


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5, 6, 7, 8])
def test_random_rhythm_loop_batch_equals_per_call(pkg, oracle, torch_cuda, seed):
    """Property test of the batched speculation as a state machine: the e2e loop
    with random deviations from the harness rhythm gives, call for call, the bits
    the per-call path gives with the batch off (crlot_set_call_speculation(1)).
    Signals of 1.5 windows and more, so deviations land inside windows and on
    their seams."""
    n, h = (1024, 256) if seed % 2 else (960, 240)
    x = oracle.synth(int(48_000 * 3.2), 40 + seed)
    try:
        pkg.set_call_speculation(1)
        a = _random_rhythm_loop(pkg, x, n, h, seed)
        pkg.set_call_speculation(2)
        b, served = _spec_delta(pkg, lambda: _random_rhythm_loop(pkg, x, n, h, seed))
    finally:
        pkg.set_call_speculation(2)
    assert len(a) == len(b)
    for i, (u, v) in enumerate(zip(a, b)):
        assert u.shape == v.shape and np.array_equal(bits(u), bits(v)), (seed, i // 3, i % 3)
    assert served["forwards"] > len(a) // 6, served  # the batch served a good part of the loop


def _random_pipeline_loop(pkg, x, n, h, seed):
    """performance_benchmark.cc's loop (FrameQueue frames, add_frame_SoA) with
    random deviations drawn from `seed`: a frame read twice, a frame read out of
    order, a forward input nudged by one ulp, a spectrum edit, produce sizes
    other than H.  Returns every array a call handed back, in call order."""
    rng = np.random.default_rng(seed)
    q = pkg.FrameQueue(x, n, h, center=True)
    w = pkg.window_table(pkg.HANN, n)
    fft = pkg.FftPlan(n, pkg.FFT_REAL)
    ola = pkg.OLAAccumulator(pkg.OLAConfig(sample_rate=48000, frame_size=n, hop_size=h, channels=1, eps=1e-8,
                                           apply_window_inside=True))
    ola.set_window(w)
    got = []
    F = q.getNumFrames()
    for i in range(F):
        r = rng.random()
        if r < 0.02 and i + 3 < F:
            q.getFrame(i + 3)  # a read ahead, then the frame itself
        f = q.getFrame(i)
        if rng.random() < 0.02:
            f = q.getFrame(i)  # read twice
        if rng.random() < 0.02:
            f = f.copy()
            f[int(rng.integers(0, n))] = np.nextafter(f[0], np.float32(np.inf))
        X = np.asarray(fft.forward_host(f[None])).copy()
        got.append(X.copy())
        if rng.random() < 0.03:
            X[0][int(rng.integers(1, n // 2))] *= np.complex64(1j)
        y = np.asarray(fft.inverse_host(X))[0].copy()
        got.append(y)
        ola.add_frame_SoA([y], w, i * h, 0, n, 1.0)
        r = rng.random()
        m = h if r < 0.9 else (h // 2 if r < 0.95 else 3 * h)
        cnt, chans = ola.produce(m)
        got.append(chans[0][:cnt].copy())
    ola.close()
    fft.close()
    q.close()
    return got


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [11, 12, 13, 14])
def test_random_pipeline_loop_batch_equals_per_call(pkg, oracle, torch_cuda, seed):
    """The FrameQueue source of the batched speculation under random deviations
    from performance_benchmark.cc's rhythm: every call gives the per-call path's
    bits with the batch on."""
    n, h = (1024, 256) if seed % 2 else (2048, 512)
    x = oracle.synth(int(48_000 * 3.2), 60 + seed)
    try:
        pkg.set_call_speculation(1)
        a = _random_pipeline_loop(pkg, x, n, h, seed)
        pkg.set_call_speculation(2)
        b, served = _spec_delta(pkg, lambda: _random_pipeline_loop(pkg, x, n, h, seed))
    finally:
        pkg.set_call_speculation(2)
    assert len(a) == len(b)
    for i, (u, v) in enumerate(zip(a, b)):
        assert u.shape == v.shape and np.array_equal(bits(u), bits(v)), (seed, i // 3, i % 3)
    assert served["forwards"] > len(a) // 6, served


def _e2e_mask_loop(pkg, x, n, h, masks, pushed=None):
    """The e2e loop with a time-varying spectral step: frame k's bins scaled by
    masks[k % len(masks)] on the host between forward and inverse."""
    w = pkg.window_table(pkg.HANN, n)
    fr = pkg.Framer()
    fr.set_params(n, h, 1, pkg.ZERO_PAD)
    fft = pkg.FftPlan(n, pkg.FFT_REAL)
    ola = pkg.OLAAccumulator(pkg.OLAConfig(sample_rate=48000, frame_size=n, hop_size=h, channels=1, eps=1e-8,
                                           apply_window_inside=True))
    ola.set_window(w)
    fr.push(x)
    outs, k = [], 0
    while True:
        f = fr.pop()
        if f is None:
            break
        X = np.asarray(fft.forward_host((f * w).astype(np.float32)[None])).copy()
        g = masks[k % len(masks)]
        X[0].real *= g
        X[0].imag *= g
        y = fft.inverse_host(X)[0]
        ola.push_frame_AoS(y, None, k * h, 0, n, 1.0)
        got, chans = ola.produce(h)
        outs.append(chans[0][:got].copy())
        if pushed is not None:
            pushed.append((np.array(y, copy=True), k * h, 1.0, h))
        k += 1
    ola.close()
    fft.close()
    fr.close()
    return (np.concatenate(outs), outs) if pushed is not None else np.concatenate(outs)


@pytest.mark.gpu
@pytest.mark.parametrize("n,h", [(1024, 256), (960, 240), (2048, 512), (3840, 960), (4000, 1000)])
def test_e2e_loop_with_time_varying_mask_backs_off(pkg, oracle, torch_cuda, n, h):
    """A per-frame mask (a noise suppressor's shape: eight masks in turn) is no
    fixed gain: after the first learned gain is replaced within a few frames by a
    very different one, the batch stops redoing its window's inverses (each would
    be a chain per frame) and backs off; the inverses take the per-call path, the
    forwards are still served, and every bit equals the per-call path's.
    (3840: the any-size server keeps two chained frames and runs its ring commits
    late; 4000: its LDS keeps one, the commits run before the transform.)"""
    x = oracle.synth(48_000 * 2, 29)
    masks = [(0.5 + 0.5 * np.cos(np.pi * np.arange(n // 2 + 1) / (n // 2) + 0.7 * j)).astype(np.float32)
             for j in range(8)]
    try:
        pkg.set_call_speculation(1)
        a = _e2e_mask_loop(pkg, x, n, h, masks)
        pkg.set_call_speculation(2)
        b, served = _spec_delta(pkg, lambda: _e2e_mask_loop(pkg, x, n, h, masks))
    finally:
        pkg.set_call_speculation(2)
    assert np.array_equal(bits(a), bits(b))
    F = a.size // h
    assert served["gains"] <= 2 and served["gain_backoffs"] >= 1, served
    assert served["forwards"] == F, served
    # the produce blocks (served from the chained inverse's speculation once the OLA
    # object is off the batch) are the oracle OLAAccumulator's fed the same frames
    pushed = []
    _, blocks = _e2e_mask_loop(pkg, x, n, h, masks, pushed)
    ref = _oracle_outputs(oracle, n, h, pkg.window_table(pkg.HANN, n), pushed)
    for k in range(len(blocks)):
        assert np.array_equal(bits(blocks[k]), bits(ref[k])), ("oracle", k)


@pytest.mark.gpu
@pytest.mark.parametrize("gain_from", [0, 5, 40])
def test_harness_order_with_a_gain_learned_late(pkg, oracle, torch_cuda, gain_from):
    """the harness's literal order (push every frame, then
    produce) with a spectral gain that starts at frame `gain_from`.  The batch
    learns the gain there and redoes the window's later inverses; the object's
    wrapped ring (precomputed with the chain from the ungained inverses) must be
    rebuilt from the redone rows.  Bits equal the per-call path's."""
    n, h = 1024, 256
    x = oracle.synth(48_000, 31)
    w = pkg.window_table(pkg.HANN, n)
    # (a gain no other test uses: the speculation keeps a learned gain across batches,
    # and one already known is served without being learned again)
    g = (0.25 + 0.75 * np.cos(np.pi * np.arange(n // 2 + 1) / (n // 2) + 0.1 + 0.01 * gain_from) ** 2
         ).astype(np.float32)

    def run():
        fr = pkg.Framer()
        fr.set_params(n, h, 1, pkg.ZERO_PAD)
        fft = pkg.FftPlan(n, pkg.FFT_REAL)
        ola = pkg.OLAAccumulator(pkg.OLAConfig(sample_rate=48000, frame_size=n, hop_size=h, channels=1,
                                               eps=1e-8, apply_window_inside=True))
        ola.set_window(w)
        fr.push(x)
        k = 0
        while True:
            f = fr.pop()
            if f is None:
                break
            X = np.asarray(fft.forward_host((f * w).astype(np.float32)[None])).copy()
            if k >= gain_from:
                X[0].real *= g
                X[0].imag *= g
            ola.push_frame_AoS(fft.inverse_host(X)[0], None, k * h, 0, n, 1.0)
            k += 1
        got, chans = ola.produce(48_000, [np.full(48_000, 7.0, np.float32)])
        out = chans[0].copy()
        ola.close()
        fft.close()
        fr.close()
        return got, out

    try:
        pkg.set_call_speculation(1)
        ga, ya = run()
        pkg.set_call_speculation(2)
        s0 = pkg.call_speculation_stats_ex()
        gb, yb = run()
        s1 = pkg.call_speculation_stats_ex()
    finally:
        pkg.set_call_speculation(2)
    assert ga == gb
    assert np.array_equal(bits(ya), bits(yb))
    assert s1["gains"] - s0["gains"] >= 1, (s0, s1)


@pytest.mark.gpu
def test_timed_out_ola_request_poisons_its_object(pkg, torch_cuda):
    """a timed-out request that changes an OLA ring (a push
    or produce) has side effects the host never recorded.  The object's ring is
    poisoned: every later call on it fails loudly until reset(), which zeroes the
    ring; after that its calls give the bits of a fresh object.  Stateless FFT
    calls on the same server resume (test_call_server_recovers_...)."""
    import time
    n, h = 1024, 256
    cfg = pkg.OLAConfig(sample_rate=48000, frame_size=n, hop_size=h, channels=1, eps=1e-8, apply_window_inside=False)
    fr = np.random.default_rng(5).standard_normal(n).astype(np.float32)

    def fresh_run(ola):
        ola.push_frame_AoS(fr, None, 0, 0, n, 1.0)
        got, ch = ola.produce(h)
        return ch[0][:got].copy()

    ref_ola = pkg.OLAAccumulator(cfg)
    ref = fresh_run(ref_ola)
    ref_ola.close()
    for op in ("push", "produce"):
        ola = pkg.OLAAccumulator(cfg)
        try:
            fresh_run(ola)
            pkg.test_inject(pkg.INJECT_CALL_TIMEOUT, 1)
            with pytest.raises(Exception):  # (a push may ride on the next request: the produce waits)
                if op == "push":
                    ola.push_frame_AoS(fr, None, h, 0, n, 1.0)
                ola.produce(h)
            pkg.test_inject(pkg.INJECT_CALL_TIMEOUT, 0)
            time.sleep(0.05)  # the timed-out request completes on the device
            with pytest.raises(Exception, match="reset"):
                ola.push_frame_AoS(fr, None, 2 * h, 0, n, 1.0)
                ola.produce(h)
            ola.reset()
            assert np.array_equal(bits(fresh_run(ola)), bits(ref))
        finally:
            pkg.test_inject(pkg.INJECT_CALL_TIMEOUT, 0)
            ola.close()
