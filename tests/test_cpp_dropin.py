"""The reference harness loop (bench/e2e_benchmark.cc:42-76, 138-186) rebuilt
against the C++ drop-in classes (include/crlot_dsp.hpp: Framer, WindowLUT cache,
MakeFftPlan, OLAAccumulator), run as tests/cpp/e2e_loop on the device, and
checked two ways:

  * end to end against the committed golden vectors tests/golden/e2e_oracle.npz
    (the oracle's streaming-interleaved round trip) within the FFT tolerance
    (rel-L2 <= 1e-6, max-abs <= 4e-6 max|x|);
  * bit-exact: the frames the loop pushed, fed to the oracle's OLAAccumulator
    with the same push/produce sequence, give the loop's output bit for bit.

C = 2 interleaved channels run the same streams through Framer(N, H, 2), strided
FFT plans and a 2-channel OLAAccumulator; every channel equals its mono run.
"""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "e2e_loop")

CASES = [("c2_1024_256", 1024, 256, "zpad"), ("c3_4096_1024", 4096, 1024, "zpad"),
         ("c4_512_128_drop", 512, 128, "drop"), ("c_1024_512", 1024, 512, "zpad"),
         ("c_2048_384", 2048, 384, "zpad"), ("sanit", 1024, 256, "zpad")]


def run_loop(tmp_path, x_interleaved, T, C, n, h, mode):
    xp, yp, fp = tmp_path / "x.f32", tmp_path / "y.f32", tmp_path / "frames.f32"
    np.ascontiguousarray(x_interleaved, np.float32).tofile(xp)
    if not os.path.exists(EXE):
        subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "cpp")], check=True)
    r = subprocess.run([EXE, str(xp), str(T), str(C), str(n), str(h), mode, str(yp), str(fp)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    y = np.fromfile(yp, np.float32).reshape(C, -1)
    frames = np.fromfile(fp, np.float32).reshape(-1, n * C)
    return y, frames


def oracle_ola(oracle, frames, n, h, C):
    """The loop's push/produce sequence on the oracle's OLAAccumulator."""
    o = oracle.Ola(n, h, C)
    o.set_window(oracle.window(oracle.HANN, n))
    out = [[] for _ in range(C)]
    for k, fr in enumerate(frames):
        o.push_frame_aos(fr, k * h, 0, n, 1.0)
        for c, v in enumerate(o.produce(h)):
            out[c].append(v)
    return np.stack([np.concatenate(v) for v in out])


@pytest.mark.gpu
@pytest.mark.parametrize("key,n,h,mode", CASES)
def test_e2e_loop_mono_vs_golden(tmp_path, torch_cuda, oracle, e2e_gold, key, n, h, mode):
    xs, ys = e2e_gold[f"{key}/x"], e2e_gold[f"{key}/y"]
    for s in range(xs.shape[0]):
        x = xs[s]
        y, frames = run_loop(tmp_path, x, x.size, 1, n, h, mode)
        ref = ys[s]
        assert y.shape[1] == ref.size  # frame count / produced length exact
        xmax = float(np.max(np.abs(x[np.isfinite(x)]))) if np.isfinite(x).any() else 1.0
        assert np.linalg.norm(y[0] - ref) <= 1e-6 * max(np.linalg.norm(ref), np.linalg.norm(
            np.nan_to_num(x, nan=0, posinf=0, neginf=0)))
        assert np.max(np.abs(y[0] - ref)) <= 4e-6 * max(xmax, 1e-30)
        assert np.array_equal(y, oracle_ola(oracle, frames, n, h, 1))


@pytest.mark.gpu
@pytest.mark.parametrize("key,n,h,mode", [CASES[0], CASES[2], CASES[4]])
def test_e2e_loop_two_channels_interleaved(tmp_path, torch_cuda, oracle, e2e_gold, key, n, h, mode):
    xs, ys = e2e_gold[f"{key}/x"], e2e_gold[f"{key}/y"]
    if xs.shape[0] < 2:
        xs = np.stack([xs[0], xs[0][::-1].copy()])
    x2 = np.stack([xs[0], xs[1]], 1).reshape(-1)
    y2, frames2 = run_loop(tmp_path, x2, xs.shape[1], 2, n, h, mode)
    assert np.array_equal(y2, oracle_ola(oracle, frames2, n, h, 2))
    for c in range(2):
        y1, _ = run_loop(tmp_path, xs[c], xs.shape[1], 1, n, h, mode)
        assert np.array_equal(y2[c], y1[0])
        if c < ys.shape[0]:
            ref = ys[c]
            assert np.linalg.norm(y2[c] - ref) <= 1e-6 * max(np.linalg.norm(ref), np.linalg.norm(xs[c]))


@pytest.mark.gpu
@pytest.mark.parametrize("n,h", [(960, 240), (882, 441), (1920, 480)])
def test_e2e_loop_any_size_vs_oracle(tmp_path, torch_cuda, oracle, n, h):
    """The e2e loop at 20 / 40 ms frames (48 and 44.1 kHz): the FFT plan and the
    OLA object share the any-size call server (fft_any.h passes, chained
    speculation); the output is the oracle's round trip within the parity
    tolerance and the oracle's OLAAccumulator fed the loop's frames bit for bit."""
    x = oracle.synth_streams(1, 30_000, config_id=91)[0]
    y, frames = run_loop(tmp_path, x, x.size, 1, n, h, "zpad")
    ref = oracle.roundtrip(x, n, h)
    assert y.shape[1] == ref.size
    assert np.linalg.norm(y[0] - ref) <= 1e-6 * max(np.linalg.norm(ref), np.linalg.norm(x))
    assert np.max(np.abs(y[0] - ref)) <= 4e-6 * float(np.max(np.abs(x)))
    assert np.array_equal(y, oracle_ola(oracle, frames, n, h, 1))


@pytest.mark.gpu
def test_kernels_loop_reference_header(torch_cuda):
    """tests/cpp/kernels_loop: kernels_benchmark.cc's scalar / "Highway" / default
    triple and kernels_test.cc's 1-ULP bar, compiled against the reference's own
    "dsp/ola/kernels.h" path (include/ref): the device kernels behind axpy_hwy and
    axpy agree with the scalar kernels within 1 ULP (in fact bit for bit)."""
    exe = os.path.join(ROOT, "tests", "cpp", "kernels_loop")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "cpp")], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "target gfx950" in r.stdout and r.stdout.strip().endswith("OK"), r.stdout
    assert all(" ulp axpy 0 windowed 0 normalize 0 " in ln for ln in r.stdout.splitlines() if ln.startswith("n ")), \
        r.stdout
