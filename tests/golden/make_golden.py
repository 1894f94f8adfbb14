"""Regenerate the golden fixtures in tests/golden/ (run in the build container only).

    python tests/golden/make_golden.py

Writes three fixture files (data only: inputs and expected outputs):

ref_tables.npz   produced by oracle/_ref/ref_dump, i.e. by the REFERENCE's own
                 dsp/window/WindowLUT.cc, dsp/ola/norm_builder.cc and
                 dsp/frame/framer.cc compiled unchanged from /root/reference
                 (oracle/Makefile target `ref`).  Window tables, COLA norm
                 tables, Framer pop sequences + available_frames traces.
kiss_gst.npz     kissfft float32 real transforms computed by the kissfft build
                 bundled in this image's GStreamer 1.14 (libgstfft-1.0.so,
                 gst_fft_f32_*), an independent build of the third-party
                 algorithm the reference calls (kissfft 131.1.0 is absent:
                 empty submodule).  Pins oracle/crlot_oracle.c's kissfft
                 restatement bit for bit.  Skipped if the library is absent.
fq_oracle.npz    FrameQueue-framed round trips (performance_benchmark.cc:174-246
                 pipeline: centre padding, no analysis window) from the oracle,
                 whose FrameQueue restatement ref_tables.npz pins (fq_* arrays,
                 dumped from the reference's own FrameQueue.cc).
e2e_oracle.npz   round-trip vectors (input, per-stage frames/spectra, output)
                 from the pinned oracle for the BASELINE configs at small T,
                 plus sanitizer cases (NaN / Inf / 1e-40 inputs).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
GOLD = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402


def ref_tables():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    out = {}
    with tempfile.TemporaryDirectory() as d:
        subprocess.run([os.path.join(ROOT, "oracle", "_ref", "ref_dump"), d], check=True)
        for line in open(os.path.join(d, "manifest.txt")):
            name, kind, _ = line.split()
            dt = np.float32 if kind == "f32" else np.uint64
            out[name] = np.fromfile(os.path.join(d, f"{name}.{kind}"), dtype=dt)
    np.savez_compressed(os.path.join(GOLD, "ref_tables.npz"), **out)
    print("ref_tables.npz:", len(out), "arrays")


def kiss_gst():
    path = "/opt/conda/lib/libgstfft-1.0.so.0"
    if not os.path.exists(path):
        print("libgstfft not found; kiss_gst.npz not regenerated")
        return
    g = C.CDLL(path)
    g.gst_fft_f32_new.restype = C.c_void_p
    g.gst_fft_f32_new.argtypes = [C.c_int, C.c_int]
    g.gst_fft_f32_fft.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    g.gst_fft_f32_inverse_fft.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    g.gst_fft_f32_free.argtypes = [C.c_void_p]
    rng = np.random.default_rng(20250905)
    out = {}
    for n in [8, 30, 64, 96, 256, 512, 1000, 1024, 2048, 4096]:
        x = rng.standard_normal(n).astype(np.float32)
        fwd = g.gst_fft_f32_new(n, 0)
        inv = g.gst_fft_f32_new(n, 1)
        X = np.zeros(n + 2, np.float32)
        g.gst_fft_f32_fft(fwd, x.ctypes.data, X.ctypes.data)
        # inverse of an independent random spectrum (imag of DC/Nyquist ignored by kiss)
        Y = rng.standard_normal(n + 2).astype(np.float32)
        y = np.zeros(n, np.float32)
        g.gst_fft_f32_inverse_fft(inv, Y.ctypes.data, y.ctypes.data)
        g.gst_fft_f32_free(fwd)
        g.gst_fft_f32_free(inv)
        out[f"x_{n}"], out[f"X_{n}"], out[f"Y_{n}"], out[f"y_{n}"] = x, X, Y, y
    np.savez_compressed(os.path.join(GOLD, "kiss_gst.npz"), **out)
    print("kiss_gst.npz:", len(out), "arrays")


# (name, N, H, mode, n_streams, T)
E2E_CASES = [
    ("c2_1024_256", 1024, 256, O.ZERO_PAD, 2, 4096 + 100),
    ("c3_4096_1024", 4096, 1024, O.ZERO_PAD, 2, 3 * 4096 + 7),
    ("c4_512_128_drop", 512, 128, O.DROP, 2, 4096),
    ("c_1024_512", 1024, 512, O.ZERO_PAD, 1, 3000),
    ("c_2048_384", 2048, 384, O.ZERO_PAD, 1, 5000),
]


def e2e_oracle():
    out = {}
    for cid, (name, n, h, mode, S, T) in enumerate(E2E_CASES):
        x = O.synth_streams(S, T, config_id=100 + cid)
        out[f"{name}/x"] = x
        ys, frs, sps = [], [], []
        for s in range(S):
            y, fr, sp = O.roundtrip(x[s], n, h, mode=mode, want_frames=True, want_spec=True)
            ys.append(y)
            frs.append(fr)
            sps.append(sp)
        out[f"{name}/y"] = np.stack(ys)
        out[f"{name}/frames"] = np.stack(frs)
        out[f"{name}/spec"] = np.stack(sps)
        out[f"{name}/meta"] = np.array([n, h, mode, S, T], np.int64)
    # sanitizer cases (fft_test.cc:199-221 style): NaN, +-Inf, denormal, tiny
    n, h, T = 1024, 256, 3000
    x = O.synth(T, 7).copy()
    x[[0, 5, 700, 1500, 2999]] = [np.nan, np.inf, -np.inf, 1e-40, np.nan]
    x[100:110] = 1e-31
    y, fr, sp = O.roundtrip(x, n, h, want_frames=True, want_spec=True)
    out["sanit/x"], out["sanit/y"], out["sanit/frames"], out["sanit/spec"] = x[None], y[None], fr[None], sp[None]
    out["sanit/meta"] = np.array([n, h, O.ZERO_PAD, 1, T], np.int64)
    np.savez_compressed(os.path.join(GOLD, "e2e_oracle.npz"), **out)
    print("e2e_oracle.npz:", len(out), "arrays")


# (name, N, H, center, pad_mode, analysis_window, n_streams, T)
FQ_CASES = [
    ("perf_1024_512_const", 1024, 512, 1, O.PAD_CONSTANT, 0, 1, 9000),
    ("c_1024_256_reflect", 1024, 256, 1, O.PAD_REFLECT, 0, 2, 5000),
    ("c_512_128_edge_win", 512, 128, 1, O.PAD_EDGE, 1, 2, 3001),
    ("c_4096_1024_reflect", 4096, 1024, 1, O.PAD_REFLECT, 0, 1, 9000),
    ("c_1024_300_edge", 1024, 300, 1, O.PAD_EDGE, 0, 1, 4000),
    ("nc_1024_256", 1024, 256, 0, O.PAD_CONSTANT, 0, 1, 5000),
    ("short_reflect", 1024, 256, 1, O.PAD_REFLECT, 0, 1, 7),
]


def fq_oracle():
    out = {}
    for cid, (name, n, h, center, pm, aw, S, T) in enumerate(FQ_CASES):
        x = O.synth_streams(S, T, config_id=200 + cid)
        ys, frs = [], []
        for s in range(S):
            y, fr = O.roundtrip_ex(x[s], n, h, mode=O.FRAMEQUEUE, center=bool(center), pad_mode=pm,
                                   analysis_window=bool(aw), want_frames=True)
            ys.append(y)
            frs.append(fr)
        out[f"{name}/x"] = x
        out[f"{name}/y"] = np.stack(ys)
        out[f"{name}/frames"] = np.stack(frs)
        out[f"{name}/meta"] = np.array([n, h, center, pm, aw, S, T], np.int64)
    np.savez_compressed(os.path.join(GOLD, "fq_oracle.npz"), **out)
    print("fq_oracle.npz:", len(out), "arrays")


if __name__ == "__main__":
    O.build()
    ref_tables()
    kiss_gst()
    e2e_oracle()
    fq_oracle()
