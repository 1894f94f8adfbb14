"""One plan, several HIP streams (and host threads) at once.

A plan keeps its launch scratch per stream handle (include/crlot_dsp.h,
"Streams and threads"): K_pair's per-walker regime flags, which the paired-only
hot walker writes and the fix-up walker reads, the staged path's frame
workspace and the interleaved path's channel planes.  These tests interleave
round trips of one plan on two torch streams -- inputs carrying NaN and 1e25
bursts so the hot walker really flags chunks for the fix-up walker -- and
require every output to equal the serial run bit for bit and the oracle within
the parity tolerance (tests/test_gpu_parity.py).
"""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REL_L2 = 1e-6


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    return t.detach().cpu().numpy()


def bursty(oracle, S, T, h, config_id):
    """Streams with a 2e25-scaled hop and a NaN in different chunks per stream:
    the pairs holding them leave the paired regime, so the hot walker flags
    their chunks and only the fix-up walker produces those outputs."""
    x = oracle.synth_streams(S, T, config_id=config_id)
    hops = T // h - 4
    for s in range(S):
        b = (s * 37 + 5) % hops
        x[s, b * h:(b + 1) * h] *= np.float32(2e25)
        x[s, ((b + hops // 2) % hops) * h + 3] = np.nan
    return x


def check_vs_oracle(oracle, x, y, n, h, streams):
    for s in streams:
        ref = oracle.roundtrip(x[s], n, h)
        assert y[s].shape == ref.shape and np.all(np.isfinite(y[s]))
        d = np.linalg.norm(y[s].astype(np.float64) - ref)
        assert d <= REL_L2 * np.linalg.norm(ref), (s, d / np.linalg.norm(ref))


@pytest.mark.parametrize("n,h", [(1024, 256), (4096, 1024), (512, 128), (2048, 512), (960, 240)])
def test_two_streams_one_plan_flagged_chunks(pkg, oracle, torch_cuda, n, h):
    torch = torch_cuda
    S, T = 192, 96_000
    xa = bursty(oracle, S, T, h, 601)
    xb = oracle.synth_streams(S, T, config_id=602)  # clean: its hot walker flags nothing
    plan = pkg.Plan(frame_size=n, hop_size=h)
    xad, xbd = dev(torch, xa), dev(torch, xb)
    ya_ser, yb_ser = host(plan.roundtrip(xad)), host(plan.roundtrip(xbd))
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    outs = []
    for it in range(6):
        # alternate which stream issues first, so hot_B lands between hot_A and fix_A
        first, second = ((sa, xad), (sb, xbd)) if it % 2 == 0 else ((sb, xbd), (sa, xad))
        with torch.cuda.stream(first[0]):
            y1 = plan.roundtrip(first[1])
        with torch.cuda.stream(second[0]):
            y2 = plan.roundtrip(second[1])
        outs.append((y1, y2) if it % 2 == 0 else (y2, y1))
    torch.cuda.synchronize()
    for it, (ya, yb) in enumerate(outs):
        assert np.array_equal(bits(host(ya)), bits(ya_ser)), (n, h, it, "bursty stream")
        assert np.array_equal(bits(host(yb)), bits(yb_ser)), (n, h, it, "clean stream")
    check_vs_oracle(oracle, xa, ya_ser, n, h, (0, 1, S - 1))


def test_two_streams_staged_and_interleaved_paths(pkg, oracle, torch_cuda):
    """The staged path (unaligned rows: synth -> frame workspace -> gather) and the
    three-pass interleaved path (channel planes) on two streams at once."""
    torch = torch_cuda
    n, h, S, T = 1024, 256, 24, 40_000
    plan = pkg.Plan(frame_size=n, hop_size=h)
    xa = oracle.synth_streams(S, T, config_id=611)
    xb = oracle.synth_streams(S, T, config_id=612)
    big_a = torch.zeros((S, T + 1), dtype=torch.float32, device="cuda")
    big_b = torch.zeros((S, T + 1), dtype=torch.float32, device="cuda")
    big_a[:, 1:] = dev(torch, xa)
    big_b[:, 1:] = dev(torch, xb)
    ua, ub = big_a[:, 1:], big_b[:, 1:]  # 4-byte offset: forces the staged path
    g, c = 4, 8
    ia = dev(torch, oracle.synth_streams(g * c, T, config_id=613).reshape(g, c, T).transpose(0, 2, 1))
    ib = dev(torch, oracle.synth_streams(g * c, T, config_id=614).reshape(g, c, T).transpose(0, 2, 1))
    ser = [host(plan.roundtrip(ua)), host(plan.roundtrip(ub)),
           host(plan.roundtrip_interleaved(ia)), host(plan.roundtrip_interleaved(ib))]
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    got = []
    for _ in range(3):
        with torch.cuda.stream(sa):
            r0 = plan.roundtrip(ua)
            r2 = plan.roundtrip_interleaved(ia)
        with torch.cuda.stream(sb):
            r1 = plan.roundtrip(ub)
            r3 = plan.roundtrip_interleaved(ib)
        got.append((r0, r1, r2, r3))
    torch.cuda.synchronize()
    for rs in got:
        for k, r in enumerate(rs):
            assert np.array_equal(bits(host(r)), bits(ser[k])), k
    check_vs_oracle(oracle, xa, ser[0], n, h, (0, S - 1))


def test_two_host_threads_one_plan(pkg, oracle, torch_cuda):
    """Two host threads, each with its own stream, share one plan."""
    torch = torch_cuda
    n, h, S, T = 1024, 256, 64, 48_000
    plan = pkg.Plan(frame_size=n, hop_size=h)
    xs = [bursty(oracle, S, T, h, 621), bursty(oracle, S, T, h, 622)]
    xds = [dev(torch, x) for x in xs]
    ser = [host(plan.roundtrip(xd)) for xd in xds]
    torch.cuda.synchronize()
    results, errors = [[], []], []

    def worker(k):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                for _ in range(8):
                    results[k].append(plan.roundtrip(xds[k]))
            s.synchronize()
        except Exception as e:  # surfaced below
            errors.append(e)

    th = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    for k in range(2):
        assert len(results[k]) == 8
        for r in results[k]:
            assert np.array_equal(bits(host(r)), bits(ser[k])), k


def test_reserve_stream_then_graph_capture(pkg, oracle, torch_cuda):
    """reserve_stream grows the stream's slot up front; the round trip then
    allocates nothing and can be captured into a HIP graph and replayed."""
    torch = torch_cuda
    n, h, S, T = 1024, 256, 16, 30_000
    plan = pkg.Plan(frame_size=n, hop_size=h)
    x = dev(torch, bursty(oracle, S, T, h, 631))
    y_ref = host(plan.roundtrip(x))
    s = torch.cuda.Stream()
    y = torch.empty((S, plan.output_length(T)), dtype=torch.float32, device="cuda")
    with torch.cuda.stream(s):
        plan.reserve_stream(S, T)
        plan.roundtrip(x, y)  # warm: the slot exists and is large enough
    s.synchronize()
    y.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        plan.roundtrip(x, y)
    for _ in range(2):
        y.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(bits(host(y)), bits(y_ref))


def test_stream_rt_gain_update_behind_queued_work(pkg, oracle, torch_cuda):
    """A spectral-gain update queued on the torch stream behind a long kernel,
    immediately followed by a resident-kernel hop: that hop must see the new gain
    (the relaunch waits for the staged copy), and the hops before it the old one;
    the per-launch Stream fed the same hops and updates is the reference."""
    torch = torch_cuda
    n, h, C_, hops = 512, 128, 8, 24
    x = oracle.synth_streams(C_, hops * h, config_id=641)
    xd = dev(torch, x)
    g2 = np.linspace(1.5, 0.25, n // 2 + 1).astype(np.float32)

    def run(kind):
        plan = pkg.Plan(frame_size=n, hop_size=h, boundary_mode=pkg.DROP, frame_pairing=False)
        st = pkg.StreamRT(plan, C_) if kind == "rt" else pkg.Stream(plan, C_)
        ys = []
        for q in range(hops):
            if q == 10:
                if kind == "rt":
                    torch.cuda._sleep(100_000_000)  # ~50 ms of device time on the torch stream
                plan.set_spectral_gain(g2)  # stream-ordered on the torch stream
            if kind == "rt":
                out, em = st.push_hop(x[:, q * h:(q + 1) * h])
            else:
                out, em = st.push_hop(xd[:, q * h:(q + 1) * h].contiguous())
                out = host(out)
            ys.append(out.copy() if em else None)
        torch.cuda.synchronize()
        st.close()
        return ys

    a, b = run("rt"), run("ref")
    for q, (ya, yb) in enumerate(zip(a, b)):
        assert (ya is None) == (yb is None), q
        if ya is not None:
            assert np.array_equal(bits(ya), bits(yb)), q


def test_stream_rt_idle_exit_is_grid_wide(pkg, oracle, torch_cuda):
    """Doorbells that arrive right at the idle timeout, on a 256-workgroup resident
    kernel (1024 channels): the first workgroup whose timer expires makes the
    whole grid leave (stop = 2), so a hop never waits for straggler workgroups
    to time out on their own clocks; every hop keeps the per-launch Stream's bits.
    One slow hop is tolerated: a single host-side stall of a few ms (the GPU box
    shares its CPUs) was seen once in five runs; a grid that is not leaving as a
    whole stalls every doorbell that lands in the exit window."""
    import time
    torch = torch_cuda
    n, h, C_, hops, idle = 512, 128, 1024, 48, 0.004
    x = oracle.synth_streams(C_, hops * h, config_id=651)
    xd = dev(torch, x)
    plan = pkg.Plan(frame_size=n, hop_size=h, boundary_mode=pkg.DROP, frame_pairing=False)
    ref = pkg.Stream(plan, C_)
    want = []
    for q in range(hops):
        out, em = ref.push_hop(xd[:, q * h:(q + 1) * h].contiguous())
        want.append(host(out).copy() if em else None)
    ref.close()
    st = pkg.StreamRT(plan, C_)
    st.set_idle_timeout(idle)
    rng = np.random.default_rng(7)
    slow = []
    for q in range(hops):
        if q >= 2:
            time.sleep(idle + float(rng.uniform(-2e-4, 2e-4)))
        t0 = time.perf_counter()
        out, em = st.push_hop(x[:, q * h:(q + 1) * h])
        dt = time.perf_counter() - t0
        if dt > 0.75 * idle:
            slow.append((q, dt))
        assert (em != 0) == (want[q] is not None), q
        if em:
            assert np.array_equal(bits(out), bits(want[q])), q
    st.close()
    assert len(slow) <= 1, slow


@pytest.mark.parametrize("pairing", [True, False])
def test_two_streams_spectral_entries(pkg, oracle, torch_cuda, pairing):
    """crlot_stft / crlot_istft_ola and the masked round trip of one plan on two
    streams at once (the staged fallbacks take per-stream scratch: unaligned
    output rows force them for half the calls): bits equal the serial runs."""
    torch = torch_cuda
    n, h, S, T = 1024, 256, 3, 20_000
    plan = pkg.Plan(frame_size=n, hop_size=h)
    plan.set_frame_pairing(pairing)
    F = plan.frame_count(T)
    xa = dev(torch, bursty(oracle, S, T, h, 91))
    xb = dev(torch, oracle.synth_streams(S, T, config_id=92))
    m = torch.from_numpy(np.random.default_rng(5).uniform(0, 1, (F, n // 2 + 1)).astype(np.float32)).cuda()

    def work(x, yo):
        spec = plan.stft(x)
        y1 = plan.istft_ola(spec)
        plan.roundtrip(x, yo[:, :F * h])  # (odd row stride: per frame the staged path)
        return spec, y1

    serial = []
    plan.set_spectral_mask(m)
    for x in (xa, xb):
        yo = torch.zeros((S, F * h + 1), device="cuda")
        spec, y1 = work(x, yo)
        serial.append((host(spec), host(y1), host(yo[:, :F * h])))
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    for it in range(3):
        outs = []
        yoa = torch.zeros((S, F * h + 1), device="cuda")
        yob = torch.zeros((S, F * h + 1), device="cuda")
        with torch.cuda.stream(sa):
            ra = work(xa, yoa)
        with torch.cuda.stream(sb):
            rb = work(xb, yob)
        torch.cuda.synchronize()
        outs = [(host(ra[0]), host(ra[1]), host(yoa[:, :F * h])), (host(rb[0]), host(rb[1]), host(yob[:, :F * h]))]
        for got, want in zip(outs, serial):
            for g_, w_ in zip(got, want):
                assert np.array_equal(bits(g_.view(np.float32) if g_.dtype == np.complex64 else g_),
                                      bits(w_.view(np.float32) if w_.dtype == np.complex64 else w_)), (pairing, it)
    plan.set_spectral_mask(None)
