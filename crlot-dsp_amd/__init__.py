"""crlot-dsp_amd -- MI355X-native batched STFT -> iSTFT -> OLA engine (Python host binding).

Thin ctypes layer over the C ABI in include/crlot_dsp.h (libcrlot_dsp.so, built
in-tree by __graft_entry__.build()).  PyTorch is used only for device memory and
the current HIP stream.  Names and argument meanings follow the reference's
C++ API (dsp::Framer / WindowLUT / fft::IFftPlan / OLAAccumulator); error codes
map to the reference's exception types: CRLOT_EINVAL -> ValueError
(std::invalid_argument), CRLOT_ERUNTIME / CRLOT_EHIP -> RuntimeError
(std::runtime_error), CRLOT_ENOMEM -> MemoryError (std::bad_alloc),
CRLOT_EUNSUPPORTED -> NotImplementedError.

There is no CPU fallback: if the library cannot be loaded, every entry raises.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CRLOT_LIB") or os.path.join(HERE, "libcrlot_dsp.so")
HEADER_PATH = os.path.join(os.path.dirname(HERE), "include", "crlot_dsp.h")

# dsp::WindowType / NormalizationType / BoundaryMode ordinals
HANN, HAMMING, BLACKMAN, RECT, BLACKMAN_HARRIS = range(5)
NORM_NONE, NORM_SUM_TO_ONE, NORM_L2, NORM_OLA_UNITY_GAIN, NORM_OLA_SUM_WSQ = range(5)
ZERO_PAD, DROP, FRAMEQUEUE = 0, 1, 2
# dsp::PadMode (FrameQueue.h:8-12)
PAD_CONSTANT, PAD_REFLECT, PAD_EDGE = 0, 1, 2
# dsp::fft::FftDomain
FFT_REAL, FFT_COMPLEX = 0, 1

OK, EINVAL, EUNSUPPORTED, EHIP, ENOMEM, ERUNTIME, ERANGE = 0, -1, -2, -3, -4, -5, -6


class PlanDesc(C.Structure):
    """crlot_plan_desc (include/crlot_dsp.h)."""
    _fields_ = [
        ("frame_size", C.c_int32),
        ("hop_size", C.c_int32),
        ("window_type", C.c_int32),
        ("periodic", C.c_int32),
        ("window_norm", C.c_int32),
        ("boundary_mode", C.c_int32),
        ("analysis_window", C.c_int32),
        ("apply_window_inside", C.c_int32),
        ("eps", C.c_float),
        ("ola_gain", C.c_float),
        ("ring_len", C.c_int32),
        ("device", C.c_int32),
        ("center", C.c_int32),
        ("pad_mode", C.c_int32),
    ]


class LaunchInfo(C.Structure):
    """crlot_launch_info (include/crlot_dsp.h): what a plan's last call on a stream launched."""
    _fields_ = [
        ("n_kernels", C.c_int32),
        ("kernels", C.c_int32 * 8),
        ("grid", C.c_int64 * 8),
        ("n_chunks", C.c_int32),
        ("reserved", C.c_int32),
    ]


class OlaConfigC(C.Structure):
    """crlot_ola_config (include/crlot_dsp.h) = dsp::OLAConfig + device."""
    _fields_ = [
        ("sample_rate", C.c_int32),
        ("frame_size", C.c_int64),
        ("hop_size", C.c_int64),
        ("channels", C.c_int64),
        ("eps", C.c_float),
        ("apply_window_inside", C.c_int32),
        ("shadow_ring", C.c_int32),
        ("device", C.c_int32),
    ]


class FftDesc(C.Structure):
    """crlot_fft_desc (include/crlot_dsp.h)."""
    _fields_ = [("domain", C.c_int32), ("nfft", C.c_int32), ("device", C.c_int32)]


_lib = None


def lib():
    """Load libcrlot_dsp.so (raises if it is missing: no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built; run __graft_entry__.build()")
    # torch ships its own libamdhip64.so.7 and loads it by path; if this library
    # bound /opt/rocm's copy first, the process would hold two HIP runtimes
    # that do not share devices, streams or allocations.  Load torch's first.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    vp, i32, i64, f32 = C.c_void_p, C.c_int32, C.c_int64, C.c_float
    fp = C.POINTER(C.c_float)
    sig = {
        "crlot_last_error": ([], C.c_char_p),
        "crlot_abi_version": ([], C.c_int),
        "crlot_build_info": ([], C.c_char_p),
        "crlot_plan_create": ([C.POINTER(PlanDesc), C.POINTER(vp)], C.c_int),
        "crlot_plan_destroy": ([vp], None),
        "crlot_plan_upload_tables": ([vp, vp, vp], C.c_int),
        "crlot_plan_set_spectral_gain": ([vp, vp], C.c_int),
        "crlot_plan_upload_tables_async": ([vp, vp, vp, vp], C.c_int),
        "crlot_plan_set_spectral_gain_async": ([vp, vp, vp], C.c_int),
        "crlot_plan_set_frame_pairing": ([vp, i32], C.c_int),
        "crlot_plan_set_chunks": ([vp, i32], C.c_int),
        "crlot_set_call_speculation": ([i32], C.c_int),
        "crlot_call_speculation_stats": ([C.POINTER(i64)], C.c_int),
        "crlot_call_speculation_stats_ex": ([C.POINTER(i64), i32], C.c_int),
        "crlot_call_batch_capacity": ([C.POINTER(i64), C.POINTER(i64), C.POINTER(i64), C.POINTER(i64)], C.c_int),
        "crlot_test_inject": ([i32, i32], C.c_int),
        "crlot_plan_last_launch": ([vp, vp, C.POINTER(LaunchInfo)], C.c_int),
        "crlot_kernel_name": ([i32], C.c_char_p),
        "crlot_plan_info": ([vp, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32)], C.c_int),
        "crlot_frame_count": ([vp, i64], i64),
        "crlot_output_length": ([vp, i64], i64),
        "crlot_workspace_bytes": ([vp, i32, i64], i64),
        "crlot_plan_reserve": ([vp, i64], C.c_int),
        "crlot_roundtrip": ([vp, vp, vp, i32, i64, i64, i64, vp], C.c_int),
        "crlot_roundtrip_stages": ([vp, vp, i32, i64, i64, vp, vp, vp], C.c_int),
        "crlot_ola_gather": ([vp, vp, vp, i32, i64, i64, i64, vp], C.c_int),
        "crlot_rfft_batched": ([vp, vp, vp, i32, i64, i64, i64, i64, vp], C.c_int),
        "crlot_irfft_batched": ([vp, vp, vp, i32, i64, i64, i64, i64, vp], C.c_int),
        "crlot_plan_set_spectral_mask": ([vp, vp, i64, i64], C.c_int),
        "crlot_stft": ([vp, vp, vp, i32, i64, i64, i64, i64, vp], C.c_int),
        "crlot_istft_ola": ([vp, vp, vp, i32, i64, i64, i64, i64, vp], C.c_int),
        "crlot_fft_plan_create": ([C.POINTER(FftDesc), C.POINTER(vp)], C.c_int),
        "crlot_fft_plan_destroy": ([vp], None),
        "crlot_fft_plan_info": ([vp, C.POINTER(i32), C.POINTER(i32)], C.c_int),
        "crlot_fft_forward": ([vp, vp, vp, i32, i64, i64, i64, i64, vp], C.c_int),
        "crlot_fft_inverse": ([vp, vp, vp, i32, i64, i64, i64, i64, vp], C.c_int),
        "crlot_fft_forward_complex": ([vp, vp, vp, i32, i64, i64, i64, i64, vp], C.c_int),
        "crlot_fft_inverse_complex": ([vp, vp, vp, i32, i64, i64, i64, i64, vp], C.c_int),
        "crlot_roundtrip_interleaved": ([vp, vp, vp, i32, i32, i64, i64, i64, vp], C.c_int),
        "crlot_stream_create": ([vp, i32, C.POINTER(vp)], C.c_int),
        "crlot_stream_destroy": ([vp], None),
        "crlot_stream_reset": ([vp], C.c_int),
        "crlot_stream_push_hop": ([vp, vp, vp, C.POINTER(i32), vp], C.c_int),
        "crlot_stream_set_layout": ([vp, i32], C.c_int),
        "crlot_stream_rt_create": ([vp, i32, i32, i32, C.POINTER(vp)], C.c_int),
        "crlot_stream_rt_destroy": ([vp], None),
        "crlot_stream_rt_reset": ([vp], C.c_int),
        "crlot_stream_rt_push_hop": ([vp, vp, vp, C.POINTER(i32)], C.c_int),
        "crlot_stream_rt_input_slot": ([vp], vp),
        "crlot_stream_rt_submit": ([vp, C.POINTER(i64)], C.c_int),
        "crlot_stream_rt_wait": ([vp, i64, C.POINTER(vp), C.POINTER(i32)], C.c_int),
        "crlot_stream_rt_info": ([vp, C.POINTER(i64), C.POINTER(C.c_double), C.POINTER(i32)], C.c_int),
        "crlot_stream_rt_set_idle_timeout": ([vp, C.c_double, C.c_double], C.c_int),
        "crlot_wav_reader_open": ([C.c_char_p, C.POINTER(vp)], C.c_int),
        "crlot_wav_reader_close": ([vp], None),
        "crlot_wav_reader_info": ([vp, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                   C.POINTER(C.c_uint64), C.POINTER(C.c_uint32), C.POINTER(i32)],
                                  C.c_int),
        "crlot_wav_reader_read": ([vp, fp, C.c_uint64, C.POINTER(C.c_uint64)], C.c_int),
        "crlot_wav_writer_open": ([C.c_char_p, C.c_uint32, C.c_uint32, C.c_uint32, i32,
                                   C.POINTER(vp)], C.c_int),
        "crlot_wav_writer_write": ([vp, fp, C.c_uint64, C.POINTER(C.c_uint64)], C.c_int),
        "crlot_wav_writer_close": ([vp], C.c_int),
        "crlot_framer_create": ([C.POINTER(vp)], C.c_int),
        "crlot_framer_destroy": ([vp], None),
        "crlot_framer_set_params": ([vp, i64, i64, i64, i32], C.c_int),
        "crlot_framer_push": ([vp, vp, i64], C.c_int),
        "crlot_framer_pop": ([vp, vp], C.c_int),
        "crlot_framer_available": ([vp], i64),
        "crlot_framer_reset": ([vp], C.c_int),
        "crlot_framer_info": ([vp, C.POINTER(i64), C.POINTER(i64), C.POINTER(i64), C.POINTER(i32),
                               C.POINTER(i64)], C.c_int),
        "crlot_ola_create": ([C.POINTER(OlaConfigC), C.POINTER(vp)], C.c_int),
        "crlot_ola_destroy": ([vp], None),
        "crlot_ola_set_window": ([vp, vp, i32], C.c_int),
        "crlot_ola_add_frame_soa": ([vp, vp, vp, i64, i64, i64, f32], C.c_int),
        "crlot_ola_push_frame_aos": ([vp, vp, vp, i64, i64, i64, f32], C.c_int),
        "crlot_ola_produce": ([vp, vp, i64, C.POINTER(i64)], C.c_int),
        "crlot_ola_add_frame_soa_device": ([vp, vp, i64, vp, i64, i64, i64, f32, vp], C.c_int),
        "crlot_ola_push_frame_aos_device": ([vp, vp, vp, i64, i64, i64, f32, vp], C.c_int),
        "crlot_ola_produce_device": ([vp, vp, i64, i64, C.POINTER(i64), vp], C.c_int),
        "crlot_ola_flush": ([vp], C.c_int),
        "crlot_ola_reset": ([vp], C.c_int),
        "crlot_ola_info": ([vp, C.POINTER(i64), C.POINTER(i64), C.POINTER(i64), C.POINTER(i32)],
                           C.c_int),
        "crlot_ola_meter_peak": ([vp, C.POINTER(f32)], C.c_int),
        "crlot_ola_norm_table": ([vp, fp], C.c_int),
        "crlot_ola_synchronize": ([vp], C.c_int),
        "crlot_fft_forward_host": ([vp, vp, vp, i32, i64, i64, i64, i64], C.c_int),
        "crlot_fft_inverse_host": ([vp, vp, vp, i32, i64, i64, i64, i64], C.c_int),
        "crlot_fft_forward_complex_host": ([vp, vp, vp, i32, i64, i64, i64, i64], C.c_int),
        "crlot_fft_inverse_complex_host": ([vp, vp, vp, i32, i64, i64, i64, i64], C.c_int),
        "crlot_axpy": ([vp, vp, f32, i64, i64, i64, i64, vp], C.c_int),
        "crlot_axpy_windowed": ([vp, vp, vp, f32, i64, i64, i64, i64, vp], C.c_int),
        "crlot_normalize_and_clear": ([vp, vp, vp, f32, i64, i64, i64, i64, vp], C.c_int),
        "crlot_call_axpy": ([vp, vp, f32, i64], C.c_int),
        "crlot_call_axpy_windowed": ([vp, vp, vp, f32, i64], C.c_int),
        "crlot_call_normalize_and_clear": ([vp, vp, vp, f32, i64], C.c_int),
        "crlot_framequeue_count": ([i64, i64, i64, i32], i64),
        "crlot_framequeue_frames": ([vp, i32, i64, i64, i64, i64, i32, i32, vp, vp], C.c_int),
        "crlot_framequeue_create": ([vp, i64, i64, i64, i32, i32, i32, C.POINTER(vp)], C.c_int),
        "crlot_framequeue_destroy": ([vp], None),
        "crlot_framequeue_info": ([vp, C.POINTER(i64), C.POINTER(i64), C.POINTER(i64)], C.c_int),
        "crlot_framequeue_frame": ([vp, i64], vp),
        "crlot_framequeue_copy_frame": ([vp, i64, vp], C.c_int),
        "crlot_framequeue_all_frames": ([vp], vp),
        "crlot_framequeue_device_frames": ([vp], vp),
        "crlot_plan_reserve_stream": ([vp, i32, i64, i32, vp], C.c_int),
        "crlot_window_table": ([i32, i64, i32, i32, fp], C.c_int),
        "crlot_ring_len": ([i64, i64], i64),
        "crlot_norm_table": ([fp, i64, i64, i64, i32, f32, fp], C.c_int),
    }
    for name, (argt, rest) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = argt
        fn.restype = rest
    _lib = L
    return L


def build_info() -> dict:
    """What the loaded library was built from (crlot_build_info): {"src": the
    source hash baked in at build time, "arch": ...}."""
    parts = dict(p.split(":", 1) for p in lib().crlot_build_info().decode().split())
    return {"src": parts.get("src"), "arch": parts.get("arch"), "path": LIB_PATH}


def set_call_speculation(mode: int):
    """1: per-call speculation of the call kernel only; 2 (default): the whole
    per-frame drop-in loop batched on the device as well (crlot_set_call_speculation)."""
    _check(lib().crlot_set_call_speculation(int(mode)), "crlot_set_call_speculation")


def call_speculation_stats() -> dict:
    """Process-wide counters of the batched speculation (crlot_call_speculation_stats)."""
    v = (C.c_int64 * 6)()
    _check(lib().crlot_call_speculation_stats(v), "crlot_call_speculation_stats")
    return dict(zip(("batches", "forwards", "inverses", "pushes", "produces", "rebuilds"), list(v)))


SPEC_STATS = ("batches", "forwards", "inverses", "pushes", "produces", "rebuilds", "frames", "windows", "declined",
              "gains", "gain_backoffs")


def call_speculation_stats_ex() -> dict:
    """All counters of the batched speculation (crlot_call_speculation_stats_ex):
    the six above plus frames transformed by batch chains, window continuations and
    declined speculations."""
    v = (C.c_int64 * len(SPEC_STATS))()
    _check(lib().crlot_call_speculation_stats_ex(v, len(SPEC_STATS)), "crlot_call_speculation_stats_ex")
    return dict(zip(SPEC_STATS, list(v)))


def call_batch_capacity() -> dict:
    """Bounds of the batched speculation (crlot_call_batch_capacity): frames per
    window, device / pinned bytes held now, pinned peak since load."""
    v = [C.c_int64() for _ in range(4)]
    _check(lib().crlot_call_batch_capacity(*[C.byref(x) for x in v]), "crlot_call_batch_capacity")
    return dict(zip(("window_frames", "device_bytes", "pinned_bytes", "pinned_peak"), [x.value for x in v]))


INJECT_BATCH_ALLOC = 1
INJECT_CALL_TIMEOUT = 2


def test_inject(what: int, count: int):
    """Test-only fault injection (crlot_test_inject): INJECT_BATCH_ALLOC fails the
    next `count` buffer allocations of the batched speculation."""
    _check(lib().crlot_test_inject(int(what), int(count)), "crlot_test_inject")


def kernel_name(kernel_id: int) -> str:
    """Name of a CRLOT_K_* launch-record id (crlot_kernel_name)."""
    return lib().crlot_kernel_name(int(kernel_id)).decode()


def _check(rc: int, what: str = "") -> int:
    if rc >= 0:
        return rc
    msg = lib().crlot_last_error().decode(errors="replace")
    msg = f"{what}: {msg}" if what else msg
    if rc == EINVAL:
        raise ValueError(msg)
    if rc == EUNSUPPORTED:
        raise NotImplementedError(msg)
    if rc == ENOMEM:
        raise MemoryError(msg)
    if rc == ERANGE:
        raise IndexError(msg)
    raise RuntimeError(msg)


def _fptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


# ----------------------------------------------------------------- host tables
def window_table(wtype: int, n: int, periodic: bool = False, norm: int = NORM_NONE) -> np.ndarray:
    """WindowLUT(n, type, periodic, norm).data() (WindowLUT.cc:215-388)."""
    out = np.zeros(max(n, 1), np.float32)
    _check(lib().crlot_window_table(wtype, n, int(periodic), norm, _fptr(out)), "window")
    return out[:n]


def ring_len(frame_size: int, hop: int) -> int:
    return _check(int(lib().crlot_ring_len(frame_size, hop)), "ring_len")


def norm_table(window, frame_size: int, hop: int, ring: int | None = None,
               apply_window_inside: bool = True, eps: float = 1e-8) -> np.ndarray:
    ring = ring_len(frame_size, hop) if ring is None else ring
    out = np.zeros(ring, np.float32)
    w = None if window is None else np.ascontiguousarray(window, np.float32)
    _check(lib().crlot_norm_table(None if w is None else _fptr(w), frame_size, hop, ring,
                                  int(apply_window_inside), eps, _fptr(out)), "norm")
    return out


def header_symbols() -> list[str]:
    """Every function the C header declares (for the ABI-surface test)."""
    import re
    txt = open(HEADER_PATH).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(crlot_[a-z0-9_]+)\s*\(", txt)))


# ----------------------------------------------------------------- device plan
def _torch():
    import torch
    return torch


def _ld(t, dim: int, minimum: int) -> int:
    """Leading dimension of `t` along `dim`; a size-1 dim's stride is meaningless
    (numpy/torch may report 0), so use the dense value there."""
    return int(t.stride(dim)) if t.shape[dim] > 1 else int(minimum)


def _stream_handle(tensor) -> int:
    torch = _torch()
    return int(torch.cuda.current_stream(tensor.device).cuda_stream)


@dataclass
class PlanConfig:
    frame_size: int = 1024
    hop_size: int = 256
    window_type: int = HANN
    periodic: bool = False
    window_norm: int = NORM_NONE
    boundary_mode: int = ZERO_PAD
    analysis_window: bool = True
    apply_window_inside: bool = True
    eps: float = 1e-8
    ola_gain: float = 1.0
    ring_len: int = 0
    device: int = -1
    center: bool = True          # boundary_mode == FRAMEQUEUE only (FrameQueue default)
    pad_mode: int = PAD_CONSTANT
    frame_pairing: bool = True   # crlot_plan_set_frame_pairing (N = 1024 fused path)


class Plan:
    """A device plan: tables resident in HBM, kernels dispatched per call.

    The default configuration is the reference harness's round trip
    (bench/e2e_benchmark.cc:42-76): symmetric Hann analysis window applied by the
    caller, window applied again inside the OLA, ZERO_PAD whole-stream framing.
    """

    def __init__(self, cfg: PlanConfig | None = None, **kw):
        cfg = cfg or PlanConfig(**kw)
        self.cfg = cfg
        d = PlanDesc(cfg.frame_size, cfg.hop_size, cfg.window_type, int(cfg.periodic),
                     cfg.window_norm, cfg.boundary_mode, int(cfg.analysis_window),
                     int(cfg.apply_window_inside), cfg.eps, cfg.ola_gain, cfg.ring_len,
                     cfg.device, int(cfg.center), cfg.pad_mode)
        h = C.c_void_p()
        _check(lib().crlot_plan_create(C.byref(d), C.byref(h)), "crlot_plan_create")
        self._h = h
        n, hop, ring = C.c_int32(), C.c_int32(), C.c_int32()
        _check(lib().crlot_plan_info(self._h, C.byref(n), C.byref(hop), C.byref(ring)))
        self.frame_size, self.hop_size, self.ring_len = n.value, hop.value, ring.value
        self.set_frame_pairing(cfg.frame_pairing)

    def close(self):
        if getattr(self, "_h", None):
            lib().crlot_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass

    # -- sizes
    def frame_count(self, T: int) -> int:
        return _check(int(lib().crlot_frame_count(self._h, T)))

    def output_length(self, T: int) -> int:
        return _check(int(lib().crlot_output_length(self._h, T)))

    def workspace_bytes(self, n_streams: int, T: int) -> int:
        return _check(int(lib().crlot_workspace_bytes(self._h, n_streams, T)))

    def reserve(self, nbytes: int):
        _check(lib().crlot_plan_reserve(self._h, nbytes))

    def reserve_stream(self, n_streams: int, T: int, channels: int = 1, stream: int | None = None):
        """Grow `stream`'s scratch slot (default: the current torch stream) for
        round trips of this shape, so those launches never allocate."""
        s = self._cur_stream() if stream is None else stream
        _check(lib().crlot_plan_reserve_stream(self._h, n_streams, T, channels, s), "reserve_stream")

    def _cur_stream(self) -> int:
        torch = _torch()
        dev = self.cfg.device if self.cfg.device >= 0 else torch.cuda.current_device()
        return int(torch.cuda.current_stream(dev).cuda_stream)

    def upload_tables(self, window=None, norm=None):
        """Replace window / norm, ordered on the current torch stream."""
        w = None if window is None else np.ascontiguousarray(window, np.float32)
        nm = None if norm is None else np.ascontiguousarray(norm, np.float32)
        _check(lib().crlot_plan_upload_tables_async(self._h, None if w is None else w.ctypes.data,
                                                    None if nm is None else nm.ctypes.data,
                                                    self._cur_stream()))

    def set_frame_pairing(self, enable: bool = True):
        """Two frames per complex transform on the fused round trip (default);
        False selects the per-frame kernels, bit-identical to stages + ola_gather;
        2 pairs through the two-regime walkers only (hot walkers off, same bits)."""
        _check(lib().crlot_plan_set_frame_pairing(self._h, 2 if enable == 2 else int(bool(enable))))

    def set_chunks(self, chunks_per_stream: int = 0):
        """Force the chunked walkers to split every stream into this many chunks
        (min(n, F); 0 restores the library's choice).  Output bits never depend
        on it; parity tests use it to move the chunk seams (crlot_plan_set_chunks)."""
        _check(lib().crlot_plan_set_chunks(self._h, int(chunks_per_stream)), "crlot_plan_set_chunks")

    def last_launch(self, stream: int | None = None) -> dict:
        """What the last call on `stream` (default: the current torch stream)
        launched: {"kernels": [names in launch order], "grid": [...],
        "n_chunks": chunks per stream, "n_kernels": count} (crlot_plan_last_launch)."""
        s = self._cur_stream() if stream is None else stream
        info = LaunchInfo()
        _check(lib().crlot_plan_last_launch(self._h, s, C.byref(info)), "crlot_plan_last_launch")
        k = min(info.n_kernels, 8)
        return {"n_kernels": info.n_kernels,
                "kernels": [kernel_name(info.kernels[i]) for i in range(k)],
                "grid": [int(info.grid[i]) for i in range(k)],
                "n_chunks": info.n_chunks}

    def set_spectral_gain(self, gain=None):
        g = None if gain is None else np.ascontiguousarray(gain, np.float32)
        if g is not None and g.size != self.frame_size // 2 + 1:
            raise ValueError("gain needs N/2+1 bins")
        _check(lib().crlot_plan_set_spectral_gain_async(self._h, None if g is None else g.ctypes.data,
                                                        self._cur_stream()))

    def set_spectral_mask(self, mask=None):
        """Time-varying spectral step (crlot_plan_set_spectral_mask): mask is a
        float32 device tensor (S, F, N/2+1) -- one real row per stream and frame --
        or (F, N/2+1), one row per frame shared by every stream; None clears it.
        The plan keeps a reference to the tensor until it is replaced."""
        if mask is None:
            self._mask = None
            _check(lib().crlot_plan_set_spectral_mask(self._h, None, 0, 0), "crlot_plan_set_spectral_mask")
            return
        bins = self.frame_size // 2 + 1
        if not mask.is_cuda or mask.shape[-1] != bins or mask.stride(-1) != 1 or mask.dim() not in (2, 3):
            raise ValueError("mask must be a (S, F, N/2+1) or (F, N/2+1) device tensor with contiguous rows")
        ld_frame = _ld(mask, -2, bins)
        ld_stream = 0 if mask.dim() == 2 else _ld(mask, 0, mask.shape[1] * ld_frame)
        self._mask = mask
        _check(lib().crlot_plan_set_spectral_mask(self._h, mask.data_ptr(), ld_frame, ld_stream),
               "crlot_plan_set_spectral_mask")

    def stft(self, x, spec=None, stream: int | None = None):
        """x: (S, T) float32 device tensor -> spec: (S, F, N/2+1) complex64, frame *
        analysis window then IFftPlan::forward per frame (crlot_stft)."""
        torch = _torch()
        if x.dim() == 1:
            return self.stft(x[None], None if spec is None else spec[None], stream)[0]
        S, T = x.shape
        if x.dtype != torch.float32 or not x.is_cuda or x.stride(1) != 1:
            raise ValueError("x must be a float32 device tensor with contiguous rows")
        F, bins = self.frame_count(T), self.frame_size // 2 + 1
        if spec is None:
            spec = torch.empty((S, F, bins), dtype=torch.complex64, device=x.device)
        if spec.dtype != torch.complex64 or spec.shape != (S, F, bins) or spec.stride(2) != 1:
            raise ValueError("spec must be (S, F, N/2+1) complex64 with contiguous rows")
        s = _stream_handle(x) if stream is None else stream
        _check(lib().crlot_stft(self._h, x.data_ptr(), spec.data_ptr(), S, T, _ld(x, 0, T),
                                2 * _ld(spec, 0, F * bins), 2 * _ld(spec, 1, bins), s), "crlot_stft")
        return spec

    def istft_ola(self, spec, y=None, stream: int | None = None):
        """spec: (S, F, N/2+1) complex64 device tensor -> y: (S, F*H): the spectral
        step, IFftPlan::inverse, overlap-add and produce (crlot_istft_ola)."""
        torch = _torch()
        if spec.dim() == 2:
            return self.istft_ola(spec[None], None if y is None else y[None], stream)[0]
        S, F, bins = spec.shape
        if spec.dtype != torch.complex64 or not spec.is_cuda or bins != self.frame_size // 2 + 1 or \
                spec.stride(2) != 1:
            raise ValueError("spec must be (S, F, N/2+1) complex64 with contiguous rows")
        L = F * self.hop_size
        if y is None:
            y = torch.empty((S, L), dtype=torch.float32, device=spec.device)
        if y.shape[0] != S or y.shape[1] < L or y.stride(1) != 1:
            raise ValueError("bad y shape")
        s = _stream_handle(spec) if stream is None else stream
        _check(lib().crlot_istft_ola(self._h, spec.data_ptr(), y.data_ptr(), S, F, 2 * _ld(spec, 0, F * bins),
                                     2 * _ld(spec, 1, bins), _ld(y, 0, L), s), "crlot_istft_ola")
        return y

    # -- hot path
    def roundtrip(self, x, y=None, stream: int | None = None):
        """x: (S, T) float32 CUDA tensor -> y: (S, F*H)."""
        torch = _torch()
        if x.dim() == 1:
            return self.roundtrip(x[None], None if y is None else y[None], stream)[0]
        if x.dtype != torch.float32 or not x.is_cuda:
            raise ValueError("x must be a float32 device tensor")
        S, T = x.shape
        if x.stride(1) != 1:
            raise ValueError("x rows must be contiguous")
        L = self.output_length(T)
        if y is None:
            y = torch.empty((S, L), dtype=torch.float32, device=x.device)
        if y.shape[0] != S or y.shape[1] < L or y.stride(1) != 1:
            raise ValueError("bad y shape")
        s = _stream_handle(x) if stream is None else stream
        _check(lib().crlot_roundtrip(self._h, x.data_ptr(), y.data_ptr(), S, T, _ld(x, 0, T),
                                     _ld(y, 0, L), s), "crlot_roundtrip")
        return y

    def roundtrip_interleaved(self, x, y=None, stream: int | None = None):
        """x: (G, T, C) float32 CUDA tensor of G groups of C interleaved channels ->
        y: (G, F*H, C), each channel an independent stream (crlot_roundtrip_interleaved)."""
        torch = _torch()
        G, T, Cc = x.shape
        if x.stride(2) != 1 or x.stride(1) != Cc:
            raise ValueError("x must be (G, T, C) with contiguous rows of C samples")
        L = self.output_length(T)
        if y is None:
            y = torch.empty((G, L, Cc), dtype=torch.float32, device=x.device)
        s = _stream_handle(x) if stream is None else stream
        ldx = x.stride(0) if G > 1 else T * Cc
        ldy = y.stride(0) if G > 1 else L * Cc
        _check(lib().crlot_roundtrip_interleaved(self._h, x.data_ptr(), y.data_ptr(), G, Cc, T, ldx, ldy, s),
               "crlot_roundtrip_interleaved")
        return y

    def stages(self, x, want_spec=True):
        """Per-stage outputs: frames (S, F, N) push_frame_AoS inputs, spec (S, F, N/2+1)."""
        torch = _torch()
        S, T = x.shape
        F = self.frame_count(T)
        n = self.frame_size
        frames = torch.empty((S, F, n), dtype=torch.float32, device=x.device)
        spec = (torch.empty((S, F, n // 2 + 1), dtype=torch.complex64, device=x.device)
                if want_spec else None)
        _check(lib().crlot_roundtrip_stages(self._h, x.data_ptr(), S, T, _ld(x, 0, T),
                                            frames.data_ptr(),
                                            None if spec is None else spec.data_ptr(),
                                            _stream_handle(x)), "crlot_roundtrip_stages")
        return frames, spec

    def ola_gather(self, frames, y=None):
        """frames (S, F, N) -> y (S, F*H) through the bit-exact OLA kernel."""
        torch = _torch()
        S, F, n = frames.shape
        if n != self.frame_size or frames.stride(2) != 1 or (
                S > 1 and frames.stride(0) != F * _ld(frames, 1, n)):
            raise ValueError("frames must be (S, F, N) with contiguous (F, N) blocks")
        L = F * self.hop_size
        if y is None:
            y = torch.empty((S, L), dtype=torch.float32, device=frames.device)
        _check(lib().crlot_ola_gather(self._h, frames.data_ptr(), y.data_ptr(), S, F,
                                      _ld(frames, 1, n), _ld(y, 0, L), _stream_handle(frames)),
               "crlot_ola_gather")
        return y

    def rfft(self, x):
        """(B, N) real -> (B, N/2+1) complex, KissFftPlan::forward semantics."""
        torch = _torch()
        B, n = x.shape
        out = torch.empty((B, n // 2 + 1), dtype=torch.complex64, device=x.device)
        _check(lib().crlot_rfft_batched(self._h, x.data_ptr(), out.data_ptr(), B, _ld(x, 0, n),
                                        x.stride(1), 2 * (n // 2 + 1), 1, _stream_handle(x)),
               "crlot_rfft_batched")
        return out

    def irfft(self, X):
        """(B, N/2+1) complex -> (B, N) real, KissFftPlan::inverse semantics."""
        torch = _torch()
        B, bins = X.shape
        n = self.frame_size
        X = X.contiguous()
        out = torch.empty((B, n), dtype=torch.float32, device=X.device)
        _check(lib().crlot_irfft_batched(self._h, X.data_ptr(), out.data_ptr(), B, 2 * bins,
                                         1, n, 1, _stream_handle(X)),
               "crlot_irfft_batched")
        return out


class FftPlan:
    """dsp::fft::IFftPlan on the device (fft_api.h:26-48), both domains.

    Batched over the leading dim of torch CUDA tensors; `forward`/`inverse` for a
    Real plan, `forward_complex`/`inverse_complex` for a Complex plan (the other
    domain's calls raise RuntimeError with the reference's message)."""

    def __init__(self, nfft: int, domain: int = FFT_REAL, device: int = -1):
        self.nfft, self.domain = nfft, domain
        self._h = None
        h = C.c_void_p()
        _check(lib().crlot_fft_plan_create(C.byref(FftDesc(domain, nfft, device)), C.byref(h)),
               "crlot_fft_plan_create")
        self._h = h

    def close(self):
        if self._h:
            lib().crlot_fft_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def size(self) -> int:
        return self.nfft

    def forward(self, x):
        """(B, nfft) real -> (B, nfft/2+1) complex (sanitized input)."""
        torch = _torch()
        B, n = x.shape
        bins = n // 2 + 1
        out = torch.empty((B, bins), dtype=torch.complex64, device=x.device)
        _check(lib().crlot_fft_forward(self._h, x.data_ptr(), out.data_ptr(), B, _ld(x, 0, n),
                                       x.stride(1), 2 * bins, 1, _stream_handle(x)),
               "forward")
        return out

    def inverse(self, X):
        """(B, nfft/2+1) complex -> (B, nfft) real (*1/nfft, sanitize)."""
        torch = _torch()
        X = X.contiguous()
        B, bins = X.shape
        out = torch.empty((B, self.nfft), dtype=torch.float32, device=X.device)
        _check(lib().crlot_fft_inverse(self._h, X.data_ptr(), out.data_ptr(), B, 2 * bins, 1,
                                       self.nfft, 1, _stream_handle(X)),
               "inverse")
        return out

    def _cplx(self, fn, name, Z):
        torch = _torch()
        B, n = Z.shape
        out = torch.empty((B, n), dtype=torch.complex64, device=Z.device)
        ld = 2 * Z.stride(0) if B > 1 else 2 * n
        _check(fn(self._h, Z.data_ptr(), out.data_ptr(), B, ld, Z.stride(1), 2 * n, 1,
                  _stream_handle(Z)), name)
        return out

    def forward_complex(self, Z):
        """(B, nfft) complex64 -> (B, nfft) complex64, unnormalised."""
        return self._cplx(lib().crlot_fft_forward_complex, "forward_complex", Z)

    def inverse_complex(self, Z):
        """(B, nfft) complex64 -> (B, nfft) complex64, *1/nfft, sanitize."""
        return self._cplx(lib().crlot_fft_inverse_complex, "inverse_complex", Z)

    # -- host-pointer forms (numpy in/out; the reference's calling convention,
    #    served by the plan's resident call kernel)
    def forward_host(self, x, out=None, inc_in: int = 1, inc_out: int = 1):
        """x: (B, nfft*inc_in) float32 numpy -> (B, (nfft/2+1)*inc_out) complex64."""
        x = np.ascontiguousarray(x, np.float32)
        x2 = x.reshape(-1, x.shape[-1])
        B = x2.shape[0]
        bins = self.nfft // 2 + 1
        if out is None:
            out = np.zeros((B, bins * inc_out), np.complex64)
        _check(lib().crlot_fft_forward_host(self._h, x2.ctypes.data, out.ctypes.data, B, x2.shape[1], inc_in,
                                            2 * out.shape[1], inc_out), "forward_host")
        return out

    def inverse_host(self, X, out=None, inc_in: int = 1, inc_out: int = 1):
        """X: (B, (nfft/2+1)*inc_in) complex64 numpy -> (B, nfft*inc_out) float32."""
        X = np.ascontiguousarray(X, np.complex64)
        X2 = X.reshape(-1, X.shape[-1])
        B = X2.shape[0]
        if out is None:
            out = np.zeros((B, self.nfft * inc_out), np.float32)
        _check(lib().crlot_fft_inverse_host(self._h, X2.ctypes.data, out.ctypes.data, B, 2 * X2.shape[1], inc_in,
                                            out.shape[1], inc_out), "inverse_host")
        return out

    def _cplx_host(self, fn, name, Z):
        Z = np.ascontiguousarray(Z, np.complex64)
        Z2 = Z.reshape(-1, Z.shape[-1])
        out = np.zeros_like(Z2)
        _check(fn(self._h, Z2.ctypes.data, out.ctypes.data, Z2.shape[0], 2 * Z2.shape[1], 1, 2 * Z2.shape[1], 1),
               name)
        return out

    def forward_complex_host(self, Z):
        return self._cplx_host(lib().crlot_fft_forward_complex_host, "forward_complex_host", Z)

    def inverse_complex_host(self, Z):
        return self._cplx_host(lib().crlot_fft_inverse_complex_host, "inverse_complex_host", Z)


# ----------------------------------------------------------------- OLA kernels (free functions)
def axpy(dst, src, g: float, win=None, stream: int | None = None):
    """dsp::axpy / axpy_windowed on device tensors: dst (B, n) += (src (B, n) [* win (n)]) * g,
    per element fma(src, g, dst) / fma(fma(src, win, 0), g, dst) (kernels.cc:18-28)."""
    d2 = dst if dst.dim() == 2 else dst[None]
    s2 = src if src.dim() == 2 else src[None]
    B, n = d2.shape
    if d2.stride(1) != 1 or s2.stride(1) != 1 or s2.shape != d2.shape:
        raise ValueError("dst / src must be (B, n) with contiguous rows")
    s = _stream_handle(dst) if stream is None else stream
    if win is None:
        _check(lib().crlot_axpy(d2.data_ptr(), s2.data_ptr(), g, n, B, _ld(d2, 0, n), _ld(s2, 0, n), s), "axpy")
    else:
        _check(lib().crlot_axpy_windowed(d2.data_ptr(), s2.data_ptr(), win.data_ptr(), g, n, B, _ld(d2, 0, n),
                                         _ld(s2, 0, n), s), "axpy_windowed")
    return dst


def normalize_and_clear(out, acc, norm, eps: float, stream: int | None = None):
    """dsp::normalize_and_clear on device tensors: out (B, n) = acc / max(norm, eps), acc = 0."""
    o2 = out if out.dim() == 2 else out[None]
    a2 = acc if acc.dim() == 2 else acc[None]
    B, n = a2.shape
    s = _stream_handle(acc) if stream is None else stream
    _check(lib().crlot_normalize_and_clear(o2.data_ptr(), a2.data_ptr(), norm.data_ptr(), eps, n, B,
                                           _ld(o2, 0, n), _ld(a2, 0, n), s), "normalize_and_clear")
    return out


def axpy_host(dst: np.ndarray, src: np.ndarray, g: float, win: np.ndarray | None = None):
    """The reference's host-pointer dsp::axpy / axpy_windowed (in place on dst, numpy float32)."""
    assert dst.dtype == np.float32 and dst.flags.c_contiguous
    src = np.ascontiguousarray(src, np.float32)
    if win is None:
        _check(lib().crlot_call_axpy(dst.ctypes.data, src.ctypes.data, g, dst.size), "axpy")
    else:
        win = np.ascontiguousarray(win, np.float32)
        _check(lib().crlot_call_axpy_windowed(dst.ctypes.data, src.ctypes.data, win.ctypes.data, g, dst.size),
               "axpy_windowed")
    return dst


def normalize_and_clear_host(out: np.ndarray, acc: np.ndarray, norm: np.ndarray, eps: float):
    """The reference's host-pointer dsp::normalize_and_clear (numpy float32, acc zeroed)."""
    assert out.dtype == np.float32 and acc.dtype == np.float32 and acc.flags.c_contiguous
    norm = np.ascontiguousarray(norm, np.float32)
    _check(lib().crlot_call_normalize_and_clear(out.ctypes.data, acc.ctypes.data, norm.ctypes.data, eps, acc.size),
           "normalize_and_clear")
    return out


# ----------------------------------------------------------------- FrameQueue
def framequeue_count(T: int, frame_size: int, hop_size: int, center: bool = True) -> int:
    return _check(int(lib().crlot_framequeue_count(T, frame_size, hop_size, int(center))), "framequeue_count")


def framequeue_frames(x, frame_size: int, hop_size: int, center: bool = True, pad_mode: int = PAD_CONSTANT,
                      stream: int | None = None):
    """Batched device form: x (S, T) CUDA tensor -> frames (S, F, N) (crlot_framequeue_frames)."""
    torch = _torch()
    x2 = x if x.dim() == 2 else x[None]
    S, T = x2.shape
    F = framequeue_count(T, frame_size, hop_size, center)
    fr = torch.empty((S, F, frame_size), dtype=torch.float32, device=x.device)
    s = _stream_handle(x) if stream is None else stream
    _check(lib().crlot_framequeue_frames(x2.data_ptr() if T else None, S, T, _ld(x2, 0, T), frame_size, hop_size,
                                         int(center), pad_mode, fr.data_ptr(), s), "framequeue_frames")
    return fr if x.dim() == 2 else fr[0]


class FrameQueue:
    """dsp::FrameQueue (FrameQueue.h:35-59): frames built on the device at construction."""

    def __init__(self, x, frame_size: int, hop_size: int, center: bool = True, pad_mode: int = PAD_CONSTANT,
                 device: int = -1):
        self._h = None
        a = None if x is None else np.ascontiguousarray(x, np.float32).reshape(-1)
        n = 0 if a is None else a.size
        h = C.c_void_p()
        _check(lib().crlot_framequeue_create(None if a is None or n == 0 else a.ctypes.data, n, frame_size,
                                             hop_size, int(center), pad_mode, device, C.byref(h)), "FrameQueue")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().crlot_framequeue_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _info(self):
        f, n, h = C.c_int64(), C.c_int64(), C.c_int64()
        _check(lib().crlot_framequeue_info(self._h, C.byref(f), C.byref(n), C.byref(h)))
        return f.value, n.value, h.value

    def getNumFrames(self) -> int:
        return self._info()[0]

    def getFrameSize(self) -> int:
        return self._info()[1]

    def getHopSize(self) -> int:
        return self._info()[2]

    def getFrame(self, idx: int) -> np.ndarray:
        p = lib().crlot_framequeue_frame(self._h, idx)
        if not p:
            _check(ERANGE if idx < 0 or idx >= self.getNumFrames() else EINVAL, "getFrame")
        n = self.getFrameSize()
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_float)), (n,)).copy()

    def copyFrame(self, idx: int, out: np.ndarray):
        _check(lib().crlot_framequeue_copy_frame(self._h, idx, None if out is None else out.ctypes.data),
               "copyFrame")

    def getAllFrames(self) -> np.ndarray:
        f, n, _ = self._info()
        if f == 0:
            return np.zeros(0, np.float32)
        p = lib().crlot_framequeue_all_frames(self._h)
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_float)), (f * n,)).copy()


class Stream:
    """Low-latency per-hop path (config 4): DROP-mode framing of `channels`
    channels fed one hop at a time; device state persists across calls."""

    def __init__(self, plan: Plan, channels: int, interleaved: bool = False):
        self.plan = plan
        self.channels = channels
        self.interleaved = interleaved
        h = C.c_void_p()
        _check(lib().crlot_stream_create(plan._h, channels, C.byref(h)), "crlot_stream_create")
        self._h = h
        _check(lib().crlot_stream_set_layout(self._h, int(interleaved)))

    def close(self):
        if getattr(self, "_h", None):
            lib().crlot_stream_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass

    def reset(self):
        _check(lib().crlot_stream_reset(self._h))

    def push_hop(self, hop, out=None, stream: int | None = None) -> tuple:
        """hop: (channels, H) float32 CUDA tensor ((H, channels) if interleaved).
        Returns (out, emitted) where emitted is 0 or H."""
        torch = _torch()
        if not hop.is_contiguous():
            raise ValueError("hop must be contiguous")
        if out is None:
            out = torch.empty_like(hop)
        em = C.c_int32()
        s = _stream_handle(hop) if stream is None else stream
        _check(lib().crlot_stream_push_hop(self._h, hop.data_ptr(), out.data_ptr(), C.byref(em), s),
               "crlot_stream_push_hop")
        return out, em.value


class StreamRT:
    """Resident low-latency per-hop path (config 4) for hops in host memory: the
    crlot_stream_rt_* entries.  Same contract and bits as Stream; hops are numpy
    float32 arrays (channels, H), or (H, channels) if interleaved."""

    def __init__(self, plan: Plan, channels: int, interleaved: bool = False, depth: int = 4):
        self.plan = plan
        self.channels = channels
        self.interleaved = interleaved
        self.depth = depth
        h = C.c_void_p()
        _check(lib().crlot_stream_rt_create(plan._h, channels, int(interleaved), depth, C.byref(h)),
               "crlot_stream_rt_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().crlot_stream_rt_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass

    def reset(self):
        _check(lib().crlot_stream_rt_reset(self._h))

    def set_idle_timeout(self, idle_seconds: float, hop_timeout_seconds: float = 2.0):
        _check(lib().crlot_stream_rt_set_idle_timeout(self._h, idle_seconds, hop_timeout_seconds))

    def push_hop(self, hop, out=None) -> tuple:
        """Returns (out, emitted) where emitted is 0 or H (out untouched when 0)."""
        import numpy as np
        hop = np.ascontiguousarray(hop, dtype=np.float32)
        if out is None:
            out = np.zeros_like(hop)
        em = C.c_int32()
        _check(lib().crlot_stream_rt_push_hop(self._h, hop.ctypes.data, out.ctypes.data, C.byref(em)),
               "crlot_stream_rt_push_hop")
        return out, em.value

    def info(self) -> dict:
        hops, ns, run = C.c_int64(), C.c_double(), C.c_int32()
        _check(lib().crlot_stream_rt_info(self._h, C.byref(hops), C.byref(ns), C.byref(run)))
        return {"hops": hops.value, "last_device_ns": ns.value, "running": bool(run.value)}


# ----------------------------------------------------------------- Framer / OLAAccumulator
class Framer:
    """dsp::Framer (framer.h:26-127): host object, interleaved PCM in, frames out.
    set_params raises ValueError (std::invalid_argument) on zero sizes; push/pop
    return the reference's bools."""

    def __init__(self):
        h = C.c_void_p()
        _check(lib().crlot_framer_create(C.byref(h)), "crlot_framer_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().crlot_framer_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass

    def set_params(self, frame_size: int, hop_size: int, channels: int = 1,
                   boundary_mode: int = ZERO_PAD):
        _check(lib().crlot_framer_set_params(self._h, frame_size, hop_size, channels,
                                             boundary_mode), "set_params")

    def push(self, interleaved, frames: int | None = None) -> bool:
        if interleaved is None:
            return bool(_check(lib().crlot_framer_push(self._h, None, frames or 0)))
        a = np.ascontiguousarray(interleaved, np.float32).reshape(-1)
        ch = self.channels()
        frames = a.size // ch if frames is None else frames
        if frames * ch > a.size:
            raise ValueError("push: fewer samples than frames * channels")
        return bool(_check(lib().crlot_framer_push(self._h, a.ctypes.data if a.size else None,
                                                   frames)))

    def pop(self, out: np.ndarray | None = None):
        """Next frame (frame_size*channels floats) or None when none is available."""
        n, ch = self.frame_size(), self.channels()
        buf = np.empty(max(1, n * ch), np.float32) if out is None else out
        ok = _check(lib().crlot_framer_pop(self._h, buf.ctypes.data))
        return buf[:n * ch] if ok else None

    def available_frames(self) -> int:
        return _check(int(lib().crlot_framer_available(self._h)))

    def reset(self):
        _check(lib().crlot_framer_reset(self._h))

    def _info(self):
        n, h, c, b = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
        m = C.c_int32()
        _check(lib().crlot_framer_info(self._h, C.byref(n), C.byref(h), C.byref(c), C.byref(m),
                                       C.byref(b)))
        return n.value, h.value, c.value, m.value, b.value

    def frame_size(self) -> int:
        return self._info()[0]

    def hop_size(self) -> int:
        return self._info()[1]

    def channels(self) -> int:
        return self._info()[2]

    def boundary_mode(self) -> int:
        return self._info()[3]

    def buffer_size(self) -> int:
        return self._info()[4]


@dataclass
class OLAConfig:
    """dsp::OLAConfig (OLAAccumulator.h:15-29)."""
    sample_rate: int = 48000
    frame_size: int = 1024
    hop_size: int = 256
    channels: int = 1
    eps: float = 1e-8
    apply_window_inside: bool = True
    shadow_ring: bool = False
    device: int = -1

    def isValid(self) -> bool:  # noqa: N802 (reference name)
        return (self.sample_rate > 0 and self.frame_size > 0 and self.hop_size > 0
                and self.channels > 0 and self.eps > 0.0)


class OLAAccumulator:
    """dsp::OLAAccumulator (OLAAccumulator.h:63-217) with its rings on the device.

    Host forms take numpy arrays (the reference's pointers); *_device forms take
    float32 CUDA tensors and run on the current torch stream."""

    def __init__(self, cfg: OLAConfig):
        self.cfg = cfg
        self._h = None
        c = OlaConfigC(cfg.sample_rate, cfg.frame_size, cfg.hop_size, cfg.channels, cfg.eps,
                       int(cfg.apply_window_inside), int(cfg.shadow_ring), cfg.device)
        h = C.c_void_p()
        _check(lib().crlot_ola_create(C.byref(c), C.byref(h)), "OLAAccumulator")
        self._h = h
        self._keep = None

    def close(self):
        if getattr(self, "_h", None):
            lib().crlot_ola_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass

    def config(self) -> OLAConfig:
        return self.cfg

    def set_window(self, w, wlen: int | None = None):
        if w is None:
            _check(lib().crlot_ola_set_window(self._h, None, wlen or 0), "set_window")
            return
        a = np.ascontiguousarray(w, np.float32)
        _check(lib().crlot_ola_set_window(self._h, a.ctypes.data, a.size if wlen is None else wlen),
               "set_window")

    @staticmethod
    def _win(window):
        if window is None:
            return None, None
        a = np.ascontiguousarray(window, np.float32)
        return a, a.ctypes.data

    def add_frame_SoA(self, ch_frames, window, start_sample: int, start_off: int, size: int,  # noqa: N802
                      gain: float = 1.0):
        """ch_frames: sequence of per-channel arrays (None entries allowed, as null pointers)."""
        if ch_frames is None:
            _check(lib().crlot_ola_add_frame_soa(self._h, None, None, start_sample, start_off,
                                                 size, gain), "add_frame_SoA")
            return
        arrs = [None if f is None else np.ascontiguousarray(f, np.float32) for f in ch_frames]
        ptrs = (C.c_void_p * max(1, len(arrs)))(*[None if a is None else a.ctypes.data for a in arrs])
        wa, wp = self._win(window)
        _check(lib().crlot_ola_add_frame_soa(self._h, ptrs, wp, start_sample, start_off, size, gain),
               "add_frame_SoA")

    def push_frame_AoS(self, interleaved, window, start_sample: int, start_off: int, size: int,  # noqa: N802
                       gain: float = 1.0):
        a = None if interleaved is None else np.ascontiguousarray(interleaved, np.float32)
        wa, wp = self._win(window)
        _check(lib().crlot_ola_push_frame_aos(self._h, None if a is None else a.ctypes.data, wp,
                                              start_sample, start_off, size, gain),
               "push_frame_AoS")

    def produce(self, n: int, out=None):
        """Returns (count, [per-channel arrays of n floats]); out may be given
        as a list of float32 arrays (their tails beyond count stay untouched)."""
        ch = self.cfg.channels
        if out is None:
            out = [np.zeros(max(n, 1), np.float32) for _ in range(ch)]
        ptrs = (C.c_void_p * max(1, ch))(*[None if o is None else o.ctypes.data for o in out])
        got = C.c_int64()
        _check(lib().crlot_ola_produce(self._h, ptrs, n, C.byref(got)), "produce")
        return got.value, out

    # -- device forms (float32 CUDA tensors, current torch stream)
    def add_frame_SoA_device(self, frames, window, start_sample: int, start_off: int, size: int,  # noqa: N802
                             gain: float = 1.0):
        """frames: (channels, >= frame_size) tensor, rows contiguous."""
        ld = _ld(frames, 0, frames.shape[-1]) if frames.dim() == 2 else frames.shape[-1]
        _check(lib().crlot_ola_add_frame_soa_device(
            self._h, frames.data_ptr(), ld, None if window is None else window.data_ptr(),
            start_sample, start_off, size, gain, _stream_handle(frames)), "add_frame_SoA_device")

    def push_frame_AoS_device(self, interleaved, window, start_sample: int, start_off: int,  # noqa: N802
                              size: int, gain: float = 1.0):
        _check(lib().crlot_ola_push_frame_aos_device(
            self._h, interleaved.data_ptr(), None if window is None else window.data_ptr(),
            start_sample, start_off, size, gain, _stream_handle(interleaved)),
            "push_frame_AoS_device")

    def produce_device(self, out, n: int) -> int:
        """out: (channels, >= n) tensor; returns the samples provided."""
        got = C.c_int64()
        ld = _ld(out, 0, out.shape[-1]) if out.dim() == 2 else out.shape[-1]
        _check(lib().crlot_ola_produce_device(self._h, out.data_ptr(), ld, n, C.byref(got),
                                              _stream_handle(out)), "produce_device")
        return got.value

    def flush(self):
        _check(lib().crlot_ola_flush(self._h))

    def reset(self):
        _check(lib().crlot_ola_reset(self._h))

    def synchronize(self):
        _check(lib().crlot_ola_synchronize(self._h))

    def _info(self):
        p, r, rs = C.c_int64(), C.c_int64(), C.c_int64()
        hw = C.c_int32()
        _check(lib().crlot_ola_info(self._h, C.byref(p), C.byref(r), C.byref(rs), C.byref(hw)))
        return p.value, r.value, rs.value, bool(hw.value)

    def produced_samples(self) -> int:
        return self._info()[0]

    def read_pos(self) -> int:
        return self._info()[1]

    def ring_size(self) -> int:
        return self._info()[2]

    def has_window(self) -> bool:
        return self._info()[3]

    def meter_peak(self) -> float:
        v = C.c_float()
        _check(lib().crlot_ola_meter_peak(self._h, C.byref(v)))
        return v.value

    def norm(self) -> np.ndarray:
        out = np.zeros(self.ring_size(), np.float32)
        _check(lib().crlot_ola_norm_table(self._h, _fptr(out)))
        return out


# ----------------------------------------------------------------- WAV I/O
class WavReader:
    """io/wav.h WavReader (host): open() -> bool, read_all() -> interleaved float32."""

    def __init__(self):
        self._h = None
        self.last_error = ""

    def open(self, filename) -> bool:
        self.close()
        h = C.c_void_p()
        rc = lib().crlot_wav_reader_open(os.fsencode(filename), C.byref(h))
        if rc == ERUNTIME:
            self.last_error = lib().crlot_last_error().decode(errors="replace")
            return False
        _check(rc, "crlot_wav_reader_open")
        self._h = h
        ch, sr, bps = C.c_uint32(), C.c_uint32(), C.c_uint32()
        tf, fl = C.c_uint64(), C.c_int32()
        _check(lib().crlot_wav_reader_info(h, C.byref(ch), C.byref(sr), C.byref(tf), C.byref(bps),
                                           C.byref(fl)))
        self._info = (ch.value, sr.value, tf.value, bps.value, bool(fl.value))
        return True

    def close(self):
        if self._h:
            lib().crlot_wav_reader_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass

    def is_open(self) -> bool:
        return bool(self._h)

    def get_channels(self) -> int:
        return self._info[0] if self._h else 0

    def get_sample_rate(self) -> int:
        return self._info[1] if self._h else 0

    def get_total_frames(self) -> int:
        return self._info[2] if self._h else 0

    def get_bits_per_sample(self) -> int:
        return self._info[3] if self._h else 0

    def read(self, frames: int) -> np.ndarray:
        """Next `frames` frames (fewer at the end), interleaved float32."""
        if not self._h:
            return np.zeros(0, np.float32)
        out = np.zeros(max(frames, 0) * self.get_channels(), np.float32)
        got = C.c_uint64()
        _check(lib().crlot_wav_reader_read(self._h, _fptr(out) if out.size else None, frames,
                                           C.byref(got)), "crlot_wav_reader_read")
        return out[:got.value * self.get_channels()]

    def read_all(self) -> np.ndarray:
        return self.read(self.get_total_frames())


class WavWriter:
    """io/wav.h WavWriter (host): open(path, channels, sample_rate, bits=16, float_format=False)."""

    def __init__(self):
        self._h = None
        self.last_error = ""

    def open(self, filename, channels: int, sample_rate: int, bits_per_sample: int = 16,
             float_format: bool = False) -> bool:
        self.close()
        h = C.c_void_p()
        rc = lib().crlot_wav_writer_open(os.fsencode(filename), channels, sample_rate,
                                         bits_per_sample, int(float_format), C.byref(h))
        if rc == ERUNTIME:
            self.last_error = lib().crlot_last_error().decode(errors="replace")
            return False
        _check(rc, "crlot_wav_writer_open")
        self._h = h
        self.channels = channels
        return True

    def write(self, data) -> int:
        """Interleaved float32 frames; returns the frames written."""
        if not self._h:
            return 0
        a = np.ascontiguousarray(data, np.float32).reshape(-1)
        frames = a.size // self.channels
        put = C.c_uint64()
        _check(lib().crlot_wav_writer_write(self._h, _fptr(a) if a.size else None, frames,
                                            C.byref(put)), "crlot_wav_writer_write")
        return put.value

    def close(self):
        if self._h:
            h, self._h = self._h, None
            _check(lib().crlot_wav_writer_close(h), "crlot_wav_writer_close")

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass

    def is_open(self) -> bool:
        return bool(self._h)


def load_wav_mono(filename) -> tuple[np.ndarray, int]:
    """WavReader.read_all() mixed down to mono the way main/main.cc:155-160 does
    (sum the channels in float, divide by the channel count); returns (x, rate)."""
    r = WavReader()
    if not r.open(filename):
        raise RuntimeError(r.last_error)
    ch, sr = r.get_channels(), r.get_sample_rate()
    pcm = r.read_all().reshape(-1, ch)
    r.close()
    acc = np.zeros(pcm.shape[0], np.float32)
    for c in range(ch):
        acc = (acc + pcm[:, c]).astype(np.float32)
    return (acc / np.float32(ch)).astype(np.float32), sr
