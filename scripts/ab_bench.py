"""A/B timing of library variants (crlot-dsp_amd/variants/*.so) in ONE process,
interleaved rounds (cdna_hip_programming.md 5.4 rule 24), the
order rotated every round so that no library always holds the first slot.  Each variant is
loaded through its own ctypes handle; the workload is the headline one.  AB_OP=stft /
istft times crlot_stft / crlot_istft_ola instead of crlot_roundtrip (spectra in one
shared buffer; the istft input is the base library's stft of the signal)."""
import ctypes as C
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

S, T, N, H = int(os.environ.get("AB_S", 1024)), 480000, int(os.environ.get("AB_N", 1024)), int(os.environ.get("AB_H", 256))
libs = sorted(glob.glob(os.environ.get("AB_GLOB") or os.path.join(ROOT, "crlot-dsp_amd", "variants", "*.so")))
base = os.path.join(ROOT, "crlot-dsp_amd", "libcrlot_dsp.so")
libs = [base] + libs


class Desc(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("frame_size", "hop_size", "window_type", "periodic",
                                         "window_norm", "boundary_mode", "analysis_window",
                                         "apply_window_inside")] + [
        ("eps", C.c_float), ("ola_gain", C.c_float), ("ring_len", C.c_int32), ("device", C.c_int32),
        ("center", C.c_int32), ("pad_mode", C.c_int32)]


g = torch.Generator(device="cuda").manual_seed(3)
x = (torch.rand((S, T), generator=g, device="cuda") * 2 - 1) * 0.5
F = (T + H - 1) // H
ys = {}
plans = {}
handles = {}
for path in libs:
    L = C.CDLL(path, mode=os.RTLD_LOCAL)
    L.crlot_plan_create.argtypes = [C.POINTER(Desc), C.POINTER(C.c_void_p)]
    L.crlot_roundtrip.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_int64,
                                  C.c_int64, C.c_int64, C.c_void_p]
    d = Desc(N, H, 0, 0, 0, 0, 1, 1, 1e-8, 1.0, 0, -1)
    h = C.c_void_p()
    assert L.crlot_plan_create(C.byref(d), C.byref(h)) == 0
    if os.environ.get("AB_GAIN") == "1":  # a smooth per-bin gain (the spectral hook)
        gain = (0.5 + 0.5 * torch.cos(torch.linspace(0, 3.14159, N // 2 + 1))).float().numpy()
        L.crlot_plan_set_spectral_gain.argtypes = [C.c_void_p, C.c_void_p]
        assert L.crlot_plan_set_spectral_gain(h, gain.ctypes.data) == 0
    if os.environ.get("AB_MASK") in ("1", "2"):  # a per-frame spectral mask: 1 shared, 2 per stream
        shape = (F, N // 2 + 1) if os.environ["AB_MASK"] == "1" else (S, F, N // 2 + 1)
        mk = torch.rand(shape, generator=torch.Generator(device="cuda").manual_seed(4), device="cuda")
        L.crlot_plan_set_spectral_mask.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64]
        assert L.crlot_plan_set_spectral_mask(h, mk.data_ptr(), N // 2 + 1,
                                              0 if mk.dim() == 2 else F * (N // 2 + 1)) == 0
        ys[path + "#mask"] = mk  # (kept alive)
    handles[path], plans[path] = L, h
    ys[path] = torch.empty((S, F * H), device="cuda")

stream = torch.cuda.current_stream()
OP = os.environ.get("AB_OP", "roundtrip")
R = N + 2  # floats per spectrum row
if OP in ("stft", "istft"):
    spec = torch.empty((S, F, R), device="cuda")
    for p in libs:
        L = handles[p]
        L.crlot_stft.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_int64, C.c_int64, C.c_int64,
                                 C.c_int64, C.c_void_p]
        L.crlot_istft_ola.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_int64, C.c_int64,
                                      C.c_int64, C.c_int64, C.c_void_p]
    assert handles[base].crlot_stft(plans[base], x.data_ptr(), spec.data_ptr(), S, T, T, F * R, R,
                                    stream.cuda_stream) == 0


def call(L, h, y):
    if OP == "stft":
        return L.crlot_stft(h, x.data_ptr(), spec.data_ptr(), S, T, T, F * R, R, stream.cuda_stream)
    if OP == "istft":
        return L.crlot_istft_ola(h, spec.data_ptr(), y.data_ptr(), S, F, F * R, R, F * H, stream.cuda_stream)
    return L.crlot_roundtrip(h, x.data_ptr(), y.data_ptr(), S, T, T, F * H, stream.cuda_stream)


times = {p: [] for p in libs}
for rnd in range(int(os.environ.get("AB_ROUNDS", len(libs) * 2))):
    # rotate the order each round: the first slot of a round can run 2-4 % slow
    for p in libs[rnd % len(libs):] + libs[:rnd % len(libs)]:
        L, h, y = handles[p], plans[p], ys[p]
        for _ in range(2):
            call(L, h, y)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            call(L, h, y)
        e1.record()
        torch.cuda.synchronize()
        times[p].append(e0.elapsed_time(e1) / 5)
ref = ys[base]
for p in libs:
    t = sorted(times[p])
    same = bool(torch.equal(ys[p], ref))
    maxd = float((ys[p] - ref).abs().max())
    print(json.dumps({"lib": os.path.relpath(p, ROOT), "op": OP, "ms_median": round(t[len(t) // 2], 4),
                      "ms_min": round(t[0], 4), "Msamples_s": round(S * T / t[len(t) // 2] / 1e3, 1),
                      "bitexact_vs_base": same, "maxdiff": maxd}))
