"""CPU tests of the product's host side: the C ABI library loads, exports every
symbol include/crlot_dsp.h declares, validates plans like the reference
constructors do, and builds its tables bit-exactly like the reference's own
compiled sources (tests/golden/ref_tables.npz).  No GPU compute here."""
import ctypes as C
import re
import subprocess

import numpy as np
import pytest

TYPES = {"hann": 0, "hamming": 1, "blackman": 2, "rect": 3}


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def test_library_exports_every_header_symbol(pkg):
    L = pkg.lib()
    syms = pkg.header_symbols()
    assert len(syms) >= 23
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", pkg.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\b(crlot_[a-z0-9_]+)\b", out))
    assert set(syms) <= exported
    assert L.crlot_abi_version() == 2


def test_library_built_from_this_tree(pkg):
    """crlot_build_info: the source hash baked in at build time equals the tree's
    (tools/src_hash.py lib_hash), so the library a run loads is the sources' build."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import src_hash
    info = pkg.build_info()
    assert info["arch"] == "gfx950"
    assert info["src"] == src_hash.lib_hash(), info


def test_library_has_gfx950_code_object(pkg):
    data = open(pkg.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_window_tables_bit_exact_vs_reference(pkg, ref_tables):
    n = 0
    for key in ref_tables.files:
        m = re.match(r"window_(\w+?)_p(\d)_n(\d+)_norm(\d)$", key)
        if not m:
            continue
        w = pkg.window_table(TYPES[m[1]], int(m[3]), bool(int(m[2])), int(m[4]))
        assert np.array_equal(bits(w), bits(ref_tables[key])), key
        n += 1
    assert n >= 100


def test_norm_tables_bit_exact_vs_reference(pkg, ref_tables):
    n = 0
    for key in ref_tables.files:
        m = re.match(r"norm_hann_p(\d)_n(\d+)_h(\d+)_r(\d+)$", key)
        if not m:
            continue
        per, fn, h, r = (int(v) for v in m.groups())
        assert pkg.ring_len(fn, h) == r
        if h == fn:
            continue  # the OLA special-cases H == N (checked below against the oracle)
        w = pkg.window_table(0, fn, bool(per))
        got = pkg.norm_table(w, fn, h, r)
        assert np.array_equal(bits(got), bits(ref_tables[key])), key
        n += 1
    assert n >= 14


def test_norm_special_cases_match_oracle(pkg, oracle):
    """initialize_normalization special cases (OLAAccumulator.cc:260-288)."""
    w = pkg.window_table(1, 512)
    for h, inside, win in ((512, True, w), (128, False, w), (128, True, None), (100, True, w)):
        got = pkg.norm_table(win, 512, h, None, inside)
        exp = oracle.norm_table(win, 512, h, inside)
        assert np.array_equal(bits(got), bits(exp)), (h, inside, win is None)


def test_window_rejects_like_reference(pkg):
    with pytest.raises(ValueError):
        pkg.window_table(pkg.HANN, 0)
    with pytest.raises(ValueError):
        pkg.window_table(pkg.BLACKMAN_HARRIS, 64)


@pytest.mark.parametrize("kw,exc", [
    (dict(frame_size=0), ValueError),            # Framer::set_params / OLAConfig::isValid
    (dict(hop_size=0), ValueError),
    (dict(eps=-1.0), ValueError),
    (dict(frame_size=513), RuntimeError),        # MakeFftPlan: odd N (kissfft_adapter.cc:44-46)
    (dict(frame_size=20000, hop_size=5000), NotImplementedError),  # beyond the device path
    (dict(window_type=4), ValueError),           # BLACKMAN_HARRIS
    (dict(boundary_mode=2, pad_mode=7), ValueError),  # unknown dsp::PadMode
    (dict(boundary_mode=3), ValueError),
])
def test_plan_validation_before_device(pkg, kw, exc):
    cfg = dict(frame_size=1024, hop_size=256)
    cfg.update(kw)
    with pytest.raises(exc):
        pkg.Plan(**cfg)


@pytest.mark.parametrize("domain,nfft,exc", [
    (2, 512, RuntimeError),            # "Unsupported FFT domain" (kissfft_adapter.cc:15-17)
    (0, 513, RuntimeError),            # odd real size (kissfft_adapter.cc:36-40)
    (0, 20000, NotImplementedError),   # valid for kissfft, beyond the device path
    (0, 0, NotImplementedError),
    (1, 10000, NotImplementedError),
])
def test_fft_plan_validation_before_device(pkg, domain, nfft, exc):
    with pytest.raises(exc):
        pkg.FftPlan(nfft, domain)


def test_struct_layout_matches_header(pkg):
    assert C.sizeof(pkg.FftDesc) == 3 * 4
    assert C.sizeof(pkg.PlanDesc) == 14 * 4


def test_build_norm_linear_bit_exact_vs_reference(pkg, ref_tables):
    """crlot_build_norm_linear (dsp::ola::build_norm_linear of include/ref) is the
    reference's norm_builder.cc:8-52 on every fixture, H == N included (there the
    OLA object special-cases the table, the builder does not)."""
    L = pkg.lib()
    L.crlot_build_norm_linear.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_int64]
    n = 0
    for key in ref_tables.files:
        m = re.match(r"norm_hann_p(\d)_n(\d+)_h(\d+)_r(\d+)$", key)
        if not m:
            continue
        per, fn, h, r = (int(v) for v in m.groups())
        w = pkg.window_table(0, fn, bool(per))
        got = np.zeros(r, np.float32)
        assert L.crlot_build_norm_linear(got.ctypes.data, w.ctypes.data, r, fn, h) == 0
        assert np.array_equal(bits(got), bits(ref_tables[key])), key
        n += 1
    assert n == 16


REF_TU = r'''
// every header the reference's bench/ and tests/ include for the hot path,
// by the reference's own paths, with its using-directives
#include "dsp/frame/framer.h"
#include "dsp/frame/FrameQueue.h"
#include "dsp/window/WindowLUT.h"
#include "dsp/ola/OLAAccumulator.h"
#include "dsp/ola/kernels.h"
#include "dsp/ola/norm_builder.h"
#include "dsp/fft/api/fft_api.h"
#include "io/wav.h"
using namespace dsp;
using namespace dsp::fft;
int probe() {
    Framer f;
    f.set_params(1024, 256, 1, BoundaryMode::ZERO_PAD);
    OLAConfig c;
    c.frame_size = 1024; c.hop_size = 256; c.channels = 1;
    WindowLUT& lut = WindowLUT::getInstance();
    auto w = lut.GetWindowSafe(WindowType::HANN, 1024);
    FftPlanDesc d{FftDomain::Real, 1024, false, 1, 1, 1};
    std::unique_ptr<IFftPlan> p;
    (void)d; (void)w; (void)p;
    float a[4] = {0}, b[4] = {0}, nrm[8] = {0}, win[4] = {1, 1, 1, 1};
    axpy_scalar(a, b, 1.0f, 4);
    if (false) axpy_hwy(a, b, 1.0f, 4);
    ola::build_norm_linear(nrm, win, 8, 4, 2);
    PadMode pm = PadMode::REFLECT;
    (void)pm;
    WavReader* r = nullptr;
    (void)r;
    return int(kMaxFrameSize) + int(get_simd_lanes());
}
'''


def test_reference_include_paths_compile(tmp_path):
    """The drop-in headers under include/ref answer the reference's own include
    paths and names (bench/e2e_benchmark.cc:8-15: #include "dsp/...", using
    namespace dsp / dsp::fft): a translation unit written as the reference writes
    it compiles with only -I include/ref."""
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = tmp_path / "ref_tu.cpp"
    src.write_text(REF_TU)
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-D__HIP_PLATFORM_AMD__",
                        "-I/opt/rocm/include", "-I" + os.path.join(root, "include", "ref"), str(src)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
