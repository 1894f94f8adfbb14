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
