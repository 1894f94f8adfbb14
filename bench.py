"""bench.py -- headline benchmark (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Metric: Msamples/s of the batched STFT -> iSTFT -> OLA round trip at
frame=1024 hop=256 batch=1024 (1024 synthetic mono streams x 480 000 samples
of 48 kHz audio = 10 s each, per GPU), inputs and outputs resident in HBM.
A "step" is one crlot_roundtrip over the whole batch.

Multi-GPU: one process per GPU.  `--gpus N` without an external
launcher starts the N ranks itself (dist.launch: fresh child processes, the
parent never touches the GPU).  Streams are independent, so there is no
data-path collective; the control plane (start/stop barrier, max-over-ranks
time) runs over RCCL when every rank owns a GPU, over gloo when ranks share one.
Two phases are timed:
  weak    (the headline `value`)  every rank runs its own 1024 streams;
  strong  (BASELINE config 5)     8192 streams in total, rank r takes
                                  dist.stream_range(8192, N, r).
`value` = samples all ranks processed / the slowest rank's wall time.

Besides the contract fields the JSON line carries
  roofline      the round-trip kernel's algorithmic HBM bytes (8 B per sample:
                4 in, 4 out) per launch / its average launch time, measured with
                HIP events on the launch stream inside the timed region; the
                same launches priced in FP32 VALU flops (what bounds the kernel,
                DESIGN.md section 5); traffic = PMC HBM bytes per launch from
                profiles/*pmc_summary.json when that profile was taken of the
                same kernel sources (src_hash), else null and flagged stale
  cpu_baseline  the oracle's C restatement of the reference CPU path (kissfft
                algorithm + scalar-FMA OLA, "kind": "port") timed on this host,
                rank 0 at N=1 only, on a bounded sample of streams, at the
                host's CPU share and single-threaded.
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Msamples/s STFT->OLA round-trip, frame=1024 hop=256 batch=1024; HBM roofline %"
N_FFT, HOP, STREAMS, T_LEN = 1024, 256, 1024, 480_000
STRONG_STREAMS = 8192          # BASELINE config 5
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
VALU_PEAK_TFLOPS = 157.3       # MI355X_MICROARCH.md: FP32 vector peak (spec)
BYTES_PER_SAMPLE = 8           # 4 B read + 4 B written


def flop_per_sample(n: int, h: int) -> float:
    """2 x 2.5 N log2 N per frame (rfft + irfft) / H, + ~6 elementwise."""
    import math
    return 2 * 2.5 * n * math.log2(n) / h + 6


def src_hash() -> str:
    """Hash of the kernel sources and their build flags (Makefile); a PMC profile
    applies only to the same hash."""
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "crlot-dsp_amd", "csrc")
    for f in sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.h")) +
                    [os.path.join(csrc, "Makefile")]):
        h.update(os.path.basename(f).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def build_check(pkg) -> dict:
    """The loaded library's baked-in source hash against the tree's
    (tools/src_hash.py lib_hash): a stale prebuilt .so fails the run."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import src_hash as SH
    info = pkg.build_info()
    tree = SH.lib_hash()
    if info["src"] != tree:
        raise SystemExit(f"stale library: {info['path']} was built from sources {info['src']}, the tree is {tree} "
                         "(run __graft_entry__.build())")
    return {"lib_src_hash": info["src"], "tree_src_hash": tree, "kernel_src_hash": src_hash(), "match": True}


def cpu_share() -> int:
    """Threads this process may use: the pool's per-GPU share (OMP_NUM_THREADS on
    the GPU box) or the affinity mask, never the whole machine's os.cpu_count()."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(aff, int(omp))) if omp and omp.isdigit() else aff


CPU_REPS = 5  # timed repetitions after one warm-up, median reported (BASELINE.md:51)


def cpu_baseline(n_streams: int = 1024, reps: int = CPU_REPS):
    """Oracle restatement of the reference CPU path on this host (kind "port"):
    one untimed warm-up pass, then `reps` timed passes, median (BASELINE.md:51)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    native = False
    try:
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "native"], check=True,
                       capture_output=True, timeout=120)
        native = True
    except Exception:
        pass
    threads = cpu_share()
    x = O.synth_streams(n_streams, T_LEN, config_id=2)

    def median_time(xs, nthreads):
        O.roundtrip_batch(xs, N_FFT, HOP, nthreads=nthreads, native=native)  # warm-up
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            O.roundtrip_batch(xs, N_FFT, HOP, nthreads=nthreads, native=native)
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)), ts

    dt, ts = median_time(x, threads)
    dt1, ts1 = median_time(x[:4], 1)
    single = 4 * T_LEN / dt1 / 1e6
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    ncpu = os.cpu_count() or 1
    return {
        "value": round(n_streams * T_LEN / dt / 1e6, 3),
        "unit": "Msamples/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{n_streams} of the 1024 streams x {T_LEN} samples (the N=1 workload) on "
                  f"{threads} pthreads (this host's CPU share: OMP_NUM_THREADS / affinity), "
                  f"oracle/crlot_oracle.c -O3{' -march=native' if native else ''} "
                  f"(kissfft-algorithm + scalar-FMA OLA restatement), 1 warm-up + {reps} timed "
                  f"passes, median {dt:.2f} s; single thread on 4 streams, median {dt1:.3f} s",
        "reps": reps,
        "rep_seconds": [round(t, 4) for t in ts],
        "single_thread_rep_seconds": [round(t, 4) for t in ts1],
        "single_thread_value": round(single, 3),
        "host_cpus": ncpu,
        "all_cpus_linear_bound": round(single * ncpu, 1),
        "all_cpus_note": "single_thread_value x host_cpus: an upper bound assuming perfect "
                         "scaling over every CPU of the machine (not measured: the pool "
                         "grants one GPU a share of the host)",
        "cpu_model": cpu_model,
    }


def load_pmc_traffic(workload_key: str):
    """HBM bytes per launch from the profiles/*pmc_summary.json of this workload
    taken of the same kernel sources (else the last by name, reported stale:
    null)."""
    pdir = os.path.join(ROOT, "profiles")
    cur = src_hash()
    best, best_f, match = None, None, False
    for f in sorted(glob.glob(os.path.join(pdir, "*pmc_summary.json"))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("workload_key") == workload_key:
            same = d.get("src_hash") == cur
            if same or not match:
                best, best_f, match = d, f, same
    if best is None:
        return None, {"file": None, "stale": True, "note": "no PMC profile of this workload"}
    stale = best.get("src_hash") != cur
    meta = {"file": os.path.relpath(best_f, ROOT), "kernel": best.get("kernel"),
            "profile_src_hash": best.get("src_hash"), "src_hash": cur, "stale": stale,
            "hbm_over_algorithmic": best.get("hbm_over_algorithmic"),
            "valu_issue": None if stale else best.get("valu_issue")}
    return (None if stale else best.get("hbm_bytes_per_launch")), meta


ISSUE_CYCLES = {"packed": 4, "permlane": 8, "other": 2}  # per wave64 instruction


def isa_issue_model(pairs_per_simd, kernel_cycles):
    """The main loop's VALU issue cost from its instruction classes (the newest
    profiles/*_isa_hist.json of these kernel sources): cycles per frame pair per
    wave = 4 x packed + 8 x permlane + 2 x other VALU; times the pairs a SIMD
    runs per launch, over the kernel's cycles (PMC GRBM_GUI_ACTIVE / 8)."""
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_isa_hist.json"))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("src_hash") == src_hash():
            best = (f, d)
    if best is None:
        return None
    f, d = best
    k = next((k for k in d["kernels"] if k.get("label", "").startswith("K_pair 1024/256")), None)
    if not k or not k.get("pairs_per_iteration"):
        return None
    ppi = k["pairs_per_iteration"]
    packed, perm = k["loop_packed"] / ppi, k["loop_permlane"] / ppi
    other = k["loop_valu"] / ppi - packed - perm
    cyc = ISSUE_CYCLES["packed"] * packed + ISSUE_CYCLES["permlane"] * perm + ISSUE_CYCLES["other"] * other
    out = {"file": os.path.relpath(f, ROOT), "valu_per_pair": round(k["loop_valu"] / ppi, 1),
           "packed_per_pair": round(packed, 1), "permlane_per_pair": round(perm, 1), "other_per_pair": round(other, 1),
           "issue_cycles_per_pair": round(cyc, 1), "cycles_per_instruction": ISSUE_CYCLES}
    if kernel_cycles:
        out["issue_frac"] = round(cyc * pairs_per_simd / kernel_cycles, 4)
    return out


def valu_block(fps, achieved_tf, issue, kern_ms, pairs_per_simd=None):
    """roofline.valu: the launches priced in SURVEY 8d flops against the FP32
    vector peak, plus -- from the same kernel sources' PMC profile -- the cycles
    the SIMDs had a VALU instruction active (SQ_ACTIVE_INST_VALU-based: issue
    plus the dependency latency it waits out, not issue alone) over the kernel's
    cycles, the issue cost from the loop's instruction classes, and the FP32
    flops the hardware counted (SQ_INSTS_VALU_FLOPS_FP32) at this run's time."""
    v = {"flop_per_sample": round(fps, 1), "achieved_tflops": round(achieved_tf, 2),
         "peak_tflops": VALU_PEAK_TFLOPS, "frac": round(achieved_tf / VALU_PEAK_TFLOPS, 4)}
    if pairs_per_simd:
        v["issue_model"] = isa_issue_model(pairs_per_simd, (issue or {}).get("kernel_cycles"))
    if issue:
        v["active_inst_frac_pmc"] = None if issue.get("busy_frac") is None else round(issue["busy_frac"], 4)
        if issue.get("kernel_cycles"):
            # GRBM_GUI_ACTIVE / 8 over the profile's average kernel duration, and the same
            # cycles over this run's kernel time (cycles, not time, are what the
            # instruction trims move; the clock is power-capped)
            v["clock_ghz"] = None if issue.get("clock_ghz") is None else round(issue["clock_ghz"], 3)
            v["clock_ghz_this_run"] = round(issue["kernel_cycles"] / (kern_ms * 1e6), 3)
            v["kernel_cycles_pmc"] = round(issue["kernel_cycles"])
        if issue.get("fp32_flops_per_launch"):
            tf = issue["fp32_flops_per_launch"] / (kern_ms * 1e-3) / 1e12
            v["counted_fp32_tflops"] = round(tf, 2)
            v["counted_frac"] = round(tf / VALU_PEAK_TFLOPS, 4)
    return v


SIMDS = 1024  # 256 CUs x 4 SIMDs
RAMP_S = 0.25  # untimed clock ramp before the warm-up steps (reported as clock_ramp_steps)


def timed_phase(plan, x, y, steps: int, warmup: int, D, dev, torch, ramp: dict = None, timings: dict = None):
    """Clock ramp (untimed round trips for RAMP_S seconds: an idle MI355X takes
    ~100-200 ms to reach its loaded clock, longer than a few warm-up steps), then
    `warmup` untimed steps, then `steps` round trips bracketed by barrier +
    synchronize; returns (wall seconds max over ranks, mean kernel ms on the
    launch stream)."""
    stream = torch.cuda.current_stream(dev)
    slow = float(os.environ.get("CRLOT_BENCH_SLOW_RANK_FACTOR", "0") or 0) if D.env_rank_world()[0] == int(
        os.environ.get("CRLOT_BENCH_SLOW_RANK", "-1")) else 0.0  # (rehearsal of a straggler: tests only)
    n_ramp, t_end = 0, time.perf_counter() + RAMP_S
    while time.perf_counter() < t_end:
        plan.roundtrip(x, y)
        torch.cuda.synchronize(dev)
        n_ramp += 1
    if ramp is not None:
        ramp["clock_ramp_steps"] = n_ramp
    for _ in range(warmup):
        plan.roundtrip(x, y)
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    D.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(steps):
        ev[i][0].record(stream)
        plan.roundtrip(x, y)
        ev[i][1].record(stream)
    torch.cuda.synchronize(dev)
    own = time.perf_counter() - t0  # this rank's own time, before the closing barrier
    if slow > 1.0:
        time.sleep(own * (slow - 1.0))
        own *= slow
    D.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / steps
    if timings is not None:
        timings["own_ms"] = own * 1e3 / steps
    return D.max_over_ranks(elapsed, dev), kern_ms


def synth_device(torch, S: int, T: int, dev, seed: int):
    g = torch.Generator(device=dev).manual_seed(seed)
    x = torch.empty((S, T), dtype=torch.float32, device=dev)
    x.uniform_(-0.5, 0.5, generator=g)
    return x



# --------------------------------------------------------------------------- suites
# `bench.py --suite NAME` runs one of the reference's other bench/ programs
# against the product (one JSON line each, never the headline contract line);
# their CPU legs are this file's cpu_baseline legs (the oracle's C restatement
# timed on this host, single thread, as the reference's benchmarks run).
def _oracle(native_try=True):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    native = False
    if native_try:
        try:
            subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "native"], check=True,
                           capture_output=True, timeout=120)
            native = True
        except Exception:
            pass
    return O, native


def _ev_time(torch, fn, reps, stream=None):
    """Mean ms per call of fn() by HIP events on the current stream (after one warm-up)."""
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def _sync_latency_us(torch, fn, reps):
    """p50 wall us of fn() + synchronize (the per-call latency a host caller sees)."""
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e6)
    ts.sort()
    return round(ts[len(ts) // 2], 2)


def suite_ola(pkg, torch, dev):
    """bench/ola_benchmark.cc counterparts.  GPU-native form: the OLA-only stage
    batched (crlot_ola_gather: frames already in HBM -> produced samples), over the
    reference's parameter grid N x H (ParamAddFrameSoA/ParamProduce, :465-485),
    priced against HBM (4 B read per frame sample + 4 B written per output
    sample).  Per-call form: the device-backed dsp::OLAAccumulator object driven
    call by call as the fixture does (AddFrameSoA / Produce / AddFrameAoS /
    Multichannel / FullPipeline, :120-240), launch-bound by construction."""
    O, native = _oracle()
    res = {"suite": "ola", "reference": "bench/ola_benchmark.cc", "grid": [], "per_call": {}}
    g = torch.Generator(device=dev).manual_seed(11)
    for n in (1024, 2048, 4096):
        for h in (n // 4, n // 2):
            S, F = 256, (480_000 // h)
            plan = pkg.Plan(frame_size=n, hop_size=h, device=dev.index)
            frames = torch.rand((S, F, n), generator=g, device=dev) - 0.5
            y = torch.empty((S, F * h), device=dev)
            ms = _ev_time(torch, lambda: plan.ola_gather(frames, y), 10)
            gbs = (S * F * n * 4 + S * F * h * 4) / (ms * 1e-3) / 1e9
            # CPU: the reference's streaming add_frame_SoA + produce(H), one stream, one thread
            Fc = min(F, 600)
            fr = frames[0, :Fc].cpu().numpy()[:, None, :]
            w = O.window(O.HANN, n)
            O.bench_ola_stream(fr[:8], n, h, w, native=native)
            t0 = time.perf_counter()
            O.bench_ola_stream(fr, n, h, w, native=native)
            cpu_s = time.perf_counter() - t0
            res["grid"].append({
                "frame": n, "hop": h, "streams": S, "frames_per_stream": F,
                "gpu_ms": round(ms, 4), "gpu_msamples_s": round(S * F * h / (ms * 1e-3) / 1e6, 1),
                "gpu_gbs": round(gbs, 1), "hbm_frac": round(gbs / HBM_PEAK_GBS, 4),
                "cpu_msamples_s_1thread": round(Fc * h / cpu_s / 1e6, 2),
                "cpu_us_per_frame": round(cpu_s / Fc * 1e6, 3)})
            del frames, y
    # per-call object API, N=1024 H=256 (the fixture's OLAConfig)
    n, h = 1024, 256
    cfg = pkg.OLAConfig(sample_rate=48000, frame_size=n, hop_size=h, channels=1, eps=1e-8,
                        apply_window_inside=False)
    w = pkg.window_table(pkg.HANN, n)
    wd = torch.from_numpy(w).to(dev)
    fr = (torch.rand((2, n), generator=g, device=dev) - 0.5).contiguous()
    out = torch.empty((2, h), device=dev)
    ola = pkg.OLAAccumulator(cfg)
    ola.set_window(w)
    k = [0]

    def add():
        ola.add_frame_SoA_device(fr[:1], wd, k[0] * h, 0, n, 1.0)

    def add_produce():
        ola.add_frame_SoA_device(fr[:1], wd, k[0] * h, 0, n, 1.0)
        ola.produce_device(out[:1], h)
        k[0] += 1

    res["per_call"]["AddFrameSoA_us_p50_synced"] = _sync_latency_us(torch, add, 200)
    res["per_call"]["AddFrameSoA_produce_us_p50_synced"] = _sync_latency_us(torch, add_produce, 200)
    t0 = time.perf_counter()
    for _ in range(2000):
        add_produce()
    torch.cuda.synchronize()
    res["per_call"]["AddFrameSoA_produce_us_async_issue"] = round((time.perf_counter() - t0) / 2000 * 1e6, 2)
    frames_cpu = np.random.default_rng(3).standard_normal((4000, 1, n)).astype(np.float32)
    t0 = time.perf_counter()
    O.bench_ola_stream(frames_cpu, n, h, w, inside=False, native=native)
    res["per_call"]["cpu_AddFrameSoA_produce_us"] = round((time.perf_counter() - t0) / 4000 * 1e6, 3)
    res["note"] = ("GPU per-call numbers are one kernel launch (+ sync) each: the object API is "
                   "latency-bound on any GPU; the batched grid is the GPU-native OLA-only form")
    res["cpu_native_build"] = native
    return res


def suite_fft(pkg, torch, dev):
    """bench/micro_fft_benchmark.cc counterparts: IFftPlan::forward at 512/1024/2048,
    batch 1 and batch 4 (:117-214) per call, plus the batched GPU-native form
    (2^18 frames per launch) priced against HBM (4 N B in, 8 (N/2+1) B out)."""
    O, native = _oracle()
    res = {"suite": "fft", "reference": "bench/micro_fft_benchmark.cc", "sizes": []}
    g = torch.Generator(device=dev).manual_seed(12)
    for n in (512, 1024, 2048):
        plan = pkg.FftPlan(n, device=dev.index)
        t = torch.arange(n, device=dev, dtype=torch.float64) / 48000.0
        sig = (0.3 * torch.sin(2 * np.pi * 440 * t) + 0.2 * torch.sin(2 * np.pi * 880 * t)
               + 0.1 * torch.sin(2 * np.pi * 1760 * t)).float()
        one, four = sig[None].contiguous(), sig[None].repeat(4, 1).contiguous()
        B = 1 << 18
        big = torch.rand((B, n), generator=g, device=dev) - 0.5
        ms = _ev_time(torch, lambda: plan.forward(big), 10)
        gbs = B * (4 * n + 8 * (n // 2 + 1)) / (ms * 1e-3) / 1e9
        xc = big[:20000].cpu().numpy()
        O.bench_rfft(xc[:100], n, native=native)
        t0 = time.perf_counter()
        O.bench_rfft(xc, n, native=native)
        cpu_us = (time.perf_counter() - t0) / xc.shape[0] * 1e6
        res["sizes"].append({
            "nfft": n,
            "single_us_p50_synced": _sync_latency_us(torch, lambda: plan.forward(one), 300),
            "batch4_us_p50_synced": _sync_latency_us(torch, lambda: plan.forward(four), 300),
            "batched_frames": B, "batched_ms": round(ms, 4),
            "batched_ns_per_frame": round(ms * 1e6 / B, 3),
            "batched_gbs": round(gbs, 1), "hbm_frac": round(gbs / HBM_PEAK_GBS, 4),
            "cpu_us_per_frame_1thread": round(cpu_us, 3)})
        del big
    res["cpu_native_build"] = native
    return res


def suite_streaming(pkg, torch, dev):
    """BASELINE config 4 (64 ch, N=512 H=128, DROP, per hop): the C++ latency
    harness (harness/stream_latency: per-launch crlot_stream_push_hop and the
    resident crlot_stream_rt path) next to the oracle's per-hop CPU cost."""
    exe = os.path.join(ROOT, "harness", "stream_latency")
    r = subprocess.run([exe, "3750"], capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        raise RuntimeError(f"stream_latency failed: {r.stdout} {r.stderr}")
    res = {"suite": "streaming", **json.loads(r.stdout.strip().splitlines()[-1])}
    O, native = _oracle()
    hops = 2000
    xs = O.synth(hops * 128, 9)
    O.roundtrip(xs[:4096], 512, 128, mode=O.DROP)
    t0 = time.perf_counter()
    O.roundtrip(xs, 512, 128, mode=O.DROP)
    per_hop_1ch = (time.perf_counter() - t0) / hops
    res["hop_budget_us_realtime"] = round(128 / 48000 * 1e6, 1)
    res["cpu_oracle_1core_us_per_hop_64ch"] = round(per_hop_1ch * 64 * 1e6, 1)
    return res


def suite_config1(pkg, torch, dev):
    """BASELINE config 1: assets/oboe.wav (tests/golden/oboe.wav) -> WavReader ->
    mono mixdown (main/main.cc:155-160) -> N=1024/H=256 Hann round trip on the GPU,
    the oracle beside it; writes gpurun_out/oboe_roundtrip.wav through WavWriter."""
    O, _ = _oracle(native_try=False)
    x, sr = pkg.load_wav_mono(os.path.join(ROOT, "tests", "golden", "oboe.wav"))
    n, h = 1024, 256
    t0 = time.perf_counter()
    ref = O.roundtrip(x, n, h)
    cpu_s = time.perf_counter() - t0
    plan = pkg.Plan(frame_size=n, hop_size=h, device=dev.index)
    xd = torch.from_numpy(x[None]).to(dev)
    out = plan.roundtrip(xd)
    ms = _ev_time(torch, lambda: plan.roundtrip(xd, out), 20)
    y = out[0].cpu().numpy()
    d = y.astype(np.float64) - ref
    path = os.path.join(ROOT, "gpurun_out", "oboe_roundtrip.wav")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    w = pkg.WavWriter()
    assert w.open(path, 1, sr, 16)
    w.write(np.clip(y[:x.size], -1, 1))
    w.close()
    return {"suite": "config1", "config": "oboe.wav mono, N=1024 H=256 Hann", "samples": int(x.size),
            "sample_rate": sr, "gpu_ms": round(ms, 4), "gpu_msamples_s": round(x.size / ms / 1e3, 1),
            "cpu_oracle_ms_1thread": round(cpu_s * 1e3, 3),
            "rel_l2_vs_oracle": float(np.linalg.norm(d) / np.linalg.norm(ref)),
            "max_abs_vs_oracle": float(np.max(np.abs(d))), "wrote": os.path.relpath(path, ROOT)}


def suite_multichannel(pkg, torch, dev):
    """Interleaved multi-channel batches (Framer(N, H, C) PCM): 1024 streams as
    1024/C groups of C channels through crlot_roundtrip_interleaved, vs the same
    streams as mono rows (the headline shape), N=1024 H=256."""
    res = {"suite": "multichannel", "frame": N_FFT, "hop": HOP, "samples_per_channel": T_LEN, "runs": []}
    plan = pkg.Plan(frame_size=N_FFT, hop_size=HOP, device=dev.index)
    g = torch.Generator(device=dev).manual_seed(21)
    x = torch.rand((STREAMS, T_LEN), generator=g, device=dev) - 0.5
    y = torch.empty((STREAMS, plan.output_length(T_LEN)), device=dev)
    ms = _ev_time(torch, lambda: plan.roundtrip(x, y), 20)
    res["runs"].append({"layout": "mono rows", "channels": 1, "ms": round(ms, 4),
                        "msamples_s": round(STREAMS * T_LEN / ms / 1e3, 1)})
    del x, y
    chans = [int(v) for v in os.environ.get("CRLOT_MC_CHANNELS", "2,4,5,8,16").split(",")]
    for c in chans:
        G = STREAMS // c
        xi = torch.rand((G, T_LEN, c), generator=g, device=dev) - 0.5
        yi = torch.empty((G, plan.output_length(T_LEN), c), device=dev)
        ms = _ev_time(torch, lambda: plan.roundtrip_interleaved(xi, yi), 20)
        res["runs"].append({"layout": "interleaved", "channels": c, "groups": G, "ms": round(ms, 4),
                            "msamples_s": round(G * c * T_LEN / ms / 1e3, 1)})
        del xi, yi
    return res


def _harness(name, *args, timeout=300):
    exe = os.path.join(ROOT, "harness", name)
    r = subprocess.run([exe, *[str(a) for a in args]], capture_output=True, text=True, timeout=timeout)
    if r.returncode != 0:
        raise RuntimeError(f"{name} failed ({r.returncode}): {r.stdout[-500:]} {r.stderr[-1500:]}")
    return json.loads(r.stdout.strip().splitlines()[-1])


def _cpu_loop_us(O, native, x, n, h, reps=5, **ex):
    """Median seconds of the oracle's per-stream C loop (the reference's Framer /
    window / forward / inverse / push / produce chain, one thread) on x."""
    L = O.lib(native)
    T = x.size
    mode = ex.get("mode", O.ZERO_PAD)
    F = O.frames_for(T, n, h, mode, ex.get("center", True))
    y = np.zeros(max(F * h, 1), np.float32)
    ts = []
    for _ in range(reps + 1):
        t0 = time.perf_counter()
        if ex:
            L.or_roundtrip_ex(x, T, n, h, O.HANN, 0, mode, int(ex.get("center", True)), O.PAD_CONSTANT,
                              int(ex.get("analysis_window", True)), y, F * h, None, None)
        else:
            L.or_roundtrip(x, T, n, h, O.HANN, 0, O.ZERO_PAD, y, F * h, None, None)
        ts.append(time.perf_counter() - t0)
    ts = sorted(ts[1:])
    return ts[len(ts) // 2] * 1e6, F


def _cpu_gain_loop_us(O, native, x, n, h, reps=5):
    """Median microseconds of the oracle's e2e loop with the spectral step (every
    bin scaled by the e2e harness's gain 0.5 + 0.5 cos(pi k / (N/2))), one thread."""
    L = O.lib(native)
    g = (0.5 + 0.5 * np.cos(np.pi * np.arange(n // 2 + 1) / (n // 2))).astype(np.float32)
    T = x.size
    F = O.frames_for(T, n, h, O.ZERO_PAD, True)
    y = np.zeros(max(F * h, 1), np.float32)
    ts = []
    for _ in range(reps + 1):
        t0 = time.perf_counter()
        L.or_roundtrip_gain(x, T, n, h, O.HANN, 0, O.ZERO_PAD, g.ctypes.data, y, F * h)
        ts.append(time.perf_counter() - t0)
    ts = sorted(ts[1:])
    return ts[len(ts) // 2] * 1e6, F


def _cpu_harness_order_us(O, native, x, n, h, reps=5):
    """Median microseconds of the oracle's loop in e2e_benchmark.cc:152-179's
    literal order (every push, then the produce loop), one thread."""
    L = O.lib(native)
    T = x.size
    y = np.zeros(T, np.float32)
    ts = []
    for _ in range(reps + 1):
        t0 = time.perf_counter()
        L.or_roundtrip_harness_order(x, T, n, h, O.HANN, 0, y, T)
        ts.append(time.perf_counter() - t0)
    ts = sorted(ts[1:])
    return ts[len(ts) // 2] * 1e6


def suite_e2e(pkg, torch, dev):
    """bench/e2e_benchmark.cc counterpart: the per-frame drop-in loop through the
    C++ classes (harness/e2e_bench: Framer -> window -> IFftPlan::forward ->
    inverse -> push_frame_AoS -> produce, on the resident call kernels) at the
    harness's hop 512 and at 256, with the oracle's single-thread C loop of the
    same chain on the same 1 s, 3-tone input beside it."""
    O, native = _oracle()
    res = {"suite": "e2e", "reference": "bench/e2e_benchmark.cc", "runs": []}
    t = np.arange(48000) / 48000.0
    x = (0.5 * np.sin(2 * np.pi * 440 * t) + 0.3 * np.sin(2 * np.pi * 880 * t)
         + 0.2 * np.sin(2 * np.pi * 1320 * t)).astype(np.float32)
    # the reference's frame (1024) at its two hops, then 20 ms frames at 48 / 44.1 kHz
    # (the any-size call server)
    for n, h in ((1024, 256), (1024, 512), (960, 480), (960, 240), (882, 441)):
        g = _harness("e2e_bench", h, 200, n)
        cpu_us, F = _cpu_loop_us(O, native, x, n, h)
        g["cpu_oracle_1thread"] = {"ms_per_iteration": round(cpu_us / 1e3, 4), "us_per_frame": round(cpu_us / F, 3),
                                   "x_realtime": round(1e6 / cpu_us, 1)}
        hus = _cpu_harness_order_us(O, native, x, n, h)
        g["harness_order"]["cpu_oracle_1thread"] = {"ms_per_iteration": round(hus / 1e3, 4),
                                                    "us_per_frame": round(hus / F, 3),
                                                    "order": "every push, then the produce loop"}
        gus, _ = _cpu_gain_loop_us(O, native, x, n, h)
        g["spectral_gain"]["cpu_oracle_1thread"] = {"ms_per_iteration": round(gus / 1e3, 4),
                                                    "us_per_frame": round(gus / F, 3)}
        if "spectral_mask" in g:  # (the CPU does the same per-bin multiply per frame whichever mask it is)
            g["spectral_mask"]["cpu_oracle_1thread"] = dict(g["spectral_gain"]["cpu_oracle_1thread"],
                                                            note="the spectral_gain row's oracle loop")
        res["runs"].append(g)
    res["cpu_native_build"] = native
    return res


def suite_kernels(pkg, torch, dev):
    """bench/micro_kernels_benchmark.cc + bench/kernels_benchmark.cc counterparts
    (harness/kernels_bench: host-pointer calls on the call kernel per size, the
    OLA push / pull calls, the batched device forms against HBM), with the
    oracle's scalar kernels timed per call in C beside them."""
    O, native = _oracle()
    res = {"suite": "kernels", **_harness("kernels_bench", 2000)}
    cpu = []
    for n in (16, 32, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768):
        reps = max(2000, int(2e7 / n))
        cpu.append({"n": n, **{k: round(O.bench_kernel(op, n, reps, native=native) * 1e6, 4)
                               for op, k in enumerate(("axpy", "axpy_windowed", "normalize_and_clear"))}})
    res["cpu_oracle_us_per_call_1thread"] = cpu
    res["cpu_native_build"] = native
    return res


def suite_pipeline(pkg, torch, dev):
    """bench/performance_benchmark.cc:174-246 (IntegratedPipelinePerformance)
    counterparts: the per-frame loop through the drop-in classes
    (harness/pipeline_bench: FrameQueue(x, 16384, 1024, 512, centre) ->
    forward -> inverse -> add_frame_SoA(window) -> produce(hop)), and the
    GPU-native batched form of the same pipeline (crlot_roundtrip with
    FrameQueue framing, no analysis window) on 1024 streams x 480 000 samples,
    the oracle's single-thread C loop beside both."""
    O, native = _oracle()
    res = {"suite": "pipeline", "reference": "bench/performance_benchmark.cc:174-246",
           "per_frame": _harness("pipeline_bench", 200)}
    x16 = np.random.default_rng(42).standard_normal(16384).astype(np.float32)
    cpu_us, F = _cpu_loop_us(O, native, x16, 1024, 512, mode=O.FRAMEQUEUE, center=True, analysis_window=False)
    res["per_frame"]["cpu_oracle_1thread"] = {"us_per_iteration": round(cpu_us, 2), "frames": F,
                                              "us_per_frame": round(cpu_us / F, 3)}
    plan = pkg.Plan(frame_size=1024, hop_size=512, boundary_mode=pkg.FRAMEQUEUE, analysis_window=False,
                    device=dev.index)
    S, T = STREAMS, T_LEN
    g = torch.Generator(device=dev).manual_seed(31)
    xb = torch.rand((S, T), generator=g, device=dev) - 0.5
    yb = torch.empty((S, plan.output_length(T)), device=dev)
    ms = _ev_time(torch, lambda: plan.roundtrip(xb, yb), 20)
    xs = O.synth(T, 7)
    cpu1, _ = _cpu_loop_us(O, native, xs, 1024, 512, reps=3, mode=O.FRAMEQUEUE, center=True, analysis_window=False)
    res["batched"] = {"streams": S, "samples_per_stream": T, "frame": 1024, "hop": 512,
                      "framing": "FrameQueue centre, constant pad, no analysis window",
                      "gpu_ms": round(ms, 4), "gpu_msamples_s": round(S * T / ms / 1e3, 1),
                      "hbm_frac": round(8 * S * T / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                      "cpu_oracle_msamples_s_1thread": round(T / cpu1, 3)}
    res["cpu_native_build"] = native
    return res


def stft_bytes_per_sample(n: int, h: int) -> float:
    """Algorithmic HBM bytes per input sample of crlot_stft (4 read + the spectra,
    8 (N/2+1) per frame written) -- and of crlot_istft_ola, the other way round."""
    return 4.0 + 8.0 * (n // 2 + 1) / h


def suite_stft(pkg, torch, dev):
    """the round trip split at its spectral step
    (bench/e2e_benchmark.cc:160-162).  At 1024 streams x 480 000 per shape:
    crlot_stft (x -> spectra), crlot_istft_ola (spectra -> y), both back to back,
    the round trip with a per-frame mask shared by the streams and with one per
    stream and frame (crlot_plan_set_spectral_mask: one walk over HBM), and the
    unmasked round trip beside them; each priced against HBM with its algorithmic
    bytes.  Then the e2e harness's time-varying mask on one 1 s window of 48 kHz
    audio (188 frames at 1024/256): host x -> device -> masked round trip (and
    stft -> a torch edit -> istft_ola) -> host y, per frame, next to the oracle's
    single-thread masked loop."""
    O, native = _oracle()
    res = {"suite": "stft", "reference": "bench/e2e_benchmark.cc:160-162", "shapes": []}
    S, T = STREAMS, T_LEN
    g = torch.Generator(device=dev).manual_seed(41)
    x = (torch.rand((S, T), generator=g, device=dev) * 2 - 1) * 0.5
    for n, h in ((1024, 256), (4096, 1024), (512, 128), (2048, 512), (960, 240), (480, 120),
                 (882, 441), (1764, 441), (1920, 480)):  # (the last three: K_pairN's transforms)
        plan = pkg.Plan(frame_size=n, hop_size=h, device=dev.index)
        F, bins = plan.frame_count(T), n // 2 + 1
        spec = torch.empty((S, F, bins), dtype=torch.complex64, device=dev)
        y = torch.empty((S, F * h), device=dev)
        samples = S * T
        b1 = stft_bytes_per_sample(n, h)

        def row(name, ms, bps, kern=None):
            gbs = bps * samples / (ms * 1e-3) / 1e9
            r = {"op": name, "ms": round(ms, 4), "msamples_s": round(samples / ms / 1e3, 1),
                 "bytes_per_sample": round(bps, 3), "gbs": round(gbs, 1), "hbm_frac": round(gbs / HBM_PEAK_GBS, 4)}
            if kern:
                r["kernels"] = kern
            return r

        t_st = _ev_time(torch, lambda: plan.stft(x, spec), 10)
        k_st = plan.last_launch()["kernels"]
        t_is = _ev_time(torch, lambda: plan.istft_ola(spec, y), 10)
        k_is = plan.last_launch()["kernels"]
        t_both = _ev_time(torch, lambda: (plan.stft(x, spec), plan.istft_ola(spec, y)), 10)
        plan.set_frame_pairing(False)  # the per-frame kernels beside the frame-pair ones
        t_stf = _ev_time(torch, lambda: plan.stft(x, spec), 10)
        k_stf = plan.last_launch()["kernels"]
        t_isf = _ev_time(torch, lambda: plan.istft_ola(spec, y), 10)
        k_isf = plan.last_launch()["kernels"]
        plan.set_frame_pairing(True)
        shape = {"frame": n, "hop": h, "streams": S, "samples_per_stream": T, "frames_per_stream": F, "runs": [
            row("stft", t_st, b1, k_st), row("istft_ola", t_is, b1, k_is),
            row("stft+istft_ola", t_both, 2 * b1),
            row("stft, per frame", t_stf, b1, k_stf), row("istft_ola, per frame", t_isf, b1, k_isf)]}
        del spec
        mask = torch.rand((F, bins), generator=g, device=dev)
        plan.set_spectral_mask(mask)
        t_m = _ev_time(torch, lambda: plan.roundtrip(x, y), 10)
        shape["runs"].append(row("roundtrip, mask shared by the streams", t_m, 8.0, plan.last_launch()["kernels"]))
        del mask
        mask = torch.rand((S, F, bins), generator=g, device=dev)
        plan.set_spectral_mask(mask)
        t_ms = _ev_time(torch, lambda: plan.roundtrip(x, y), 10)
        shape["runs"].append(row("roundtrip, mask per stream and frame", t_ms, 8.0 + 4.0 * bins / h,
                                 plan.last_launch()["kernels"]))
        plan.set_frame_pairing(False)  # the per-frame walk beside the frame-pair one
        t_mf = _ev_time(torch, lambda: plan.roundtrip(x, y), 10)
        shape["runs"].append(row("roundtrip, mask per stream and frame, per-frame walk", t_mf,
                                 8.0 + 4.0 * bins / h, plan.last_launch()["kernels"]))
        plan.set_frame_pairing(True)
        plan.set_spectral_mask(None)
        del mask
        t_r = _ev_time(torch, lambda: plan.roundtrip(x, y), 10)
        shape["runs"].append(row("roundtrip (no mask)", t_r, 8.0, plan.last_launch()["kernels"]))
        res["shapes"].append(shape)
        del y
        torch.cuda.empty_cache()
    del x
    torch.cuda.empty_cache()
    # the e2e harness's spectral_mask row on one window: 1 s of the 3-tone signal,
    # 8 masks in turn (frame k takes mask k % 8), as harness/e2e_bench does per call
    n, h = 1024, 256
    t = np.arange(48000) / 48000.0
    xh = (0.5 * np.sin(2 * np.pi * 440 * t) + 0.3 * np.sin(2 * np.pi * 880 * t)
          + 0.2 * np.sin(2 * np.pi * 1320 * t)).astype(np.float32)
    plan = pkg.Plan(frame_size=n, hop_size=h, device=dev.index)
    F, bins = plan.frame_count(xh.size), n // 2 + 1
    kk = np.arange(bins) / (bins - 1)
    masks = np.stack([(0.5 + 0.5 * np.cos(np.pi * kk * (1 + j / 8.0))) for j in range(8)]).astype(np.float32)
    rows = masks[np.arange(F) % 8]
    mask_d = torch.from_numpy(rows).to(dev)
    x_pin = torch.from_numpy(xh[None].copy()).pin_memory()
    y_pin = torch.empty((1, F * h)).pin_memory()
    xd = torch.empty((1, xh.size), device=dev)
    yd = torch.empty((1, F * h), device=dev)
    specd = torch.empty((1, F, bins), dtype=torch.complex64, device=dev)

    def masked_walk():
        xd.copy_(x_pin, non_blocking=True)
        plan.roundtrip(xd, yd)
        y_pin.copy_(yd, non_blocking=True)

    def split_edit():
        xd.copy_(x_pin, non_blocking=True)
        plan.stft(xd, specd)
        specd.mul_(mask_d[None])  # any device-side edit between the halves
        plan.istft_ola(specd, yd)
        y_pin.copy_(yd, non_blocking=True)

    plan.set_spectral_mask(mask_d)
    us_walk = _sync_latency_us(torch, masked_walk, 300)
    k_walk = plan.last_launch()["kernels"]
    y_walk = y_pin.numpy().copy()
    plan.set_spectral_mask(None)
    us_split = _sync_latency_us(torch, split_edit, 300)
    y_split = y_pin.numpy().copy()
    L = O.lib(native)
    yc = np.zeros(F * h, np.float32)
    ts = []
    for _ in range(6):
        t0 = time.perf_counter()
        L.or_roundtrip_mask(xh, xh.size, n, h, O.HANN, 0, O.ZERO_PAD, 1, O.PAD_CONSTANT, 1, None,
                            np.ascontiguousarray(rows).ctypes.data, bins, yc, F * h, None)
        ts.append(time.perf_counter() - t0)
    cpu_us = sorted(ts[1:])[2] * 1e6
    d = y_walk[0].astype(np.float64) - yc
    res["e2e_window"] = {
        "frame": n, "hop": h, "samples": int(xh.size), "frames": F, "masks": 8,
        "masked_roundtrip_us_per_window_p50": us_walk, "masked_roundtrip_us_per_frame": round(us_walk / F, 3),
        "stft_edit_istft_us_per_window_p50": us_split, "stft_edit_istft_us_per_frame": round(us_split / F, 3),
        "includes": "H2D of x and D2H of y (pinned), launch and synchronize",
        "cpu_oracle_1thread": {"us_per_window": round(cpu_us, 1), "us_per_frame": round(cpu_us / F, 3)},
        "masked_roundtrip_kernels": k_walk,
        "rel_l2_vs_oracle": float(np.linalg.norm(d) / np.linalg.norm(yc)),
        "split_vs_walk_rel_l2": float(np.linalg.norm(y_walk.astype(np.float64) - y_split) / np.linalg.norm(y_split))}
    res["cpu_native_build"] = native
    return res


SUITES = {"ola": suite_ola, "multichannel": suite_multichannel, "fft": suite_fft, "streaming": suite_streaming,
          "config1": suite_config1, "e2e": suite_e2e, "kernels": suite_kernels, "pipeline": suite_pipeline,
          "stft": suite_stft}


def run_suite(name):
    import numpy as _np  # noqa: F401
    import torch
    from __graft_entry__ import load_pkg
    pkg = load_pkg()
    build = build_check(pkg)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    print(json.dumps({**SUITES[name](pkg, torch, dev), "build": build}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=50)  # ~130 ms: lets the clocks ramp
    ap.add_argument("--streams", type=int, default=STREAMS)
    ap.add_argument("--strong-streams", type=int, default=STRONG_STREAMS)
    ap.add_argument("--strong-steps", type=int, default=10)
    ap.add_argument("--no-strong", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--suite", choices=sorted(SUITES), help="run one reference bench/ counterpart instead")
    args = ap.parse_args()
    if args.suite:
        return run_suite(args.suite)

    from __graft_entry__ import load_pkg, load_dist
    D = load_dist()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no external launcher: start the N ranks here, before any GPU call
        sys.exit(D.launch(args.gpus, [os.path.abspath(__file__)] + sys.argv[1:]))

    import torch

    _, world, local = D.env_rank_world()
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world))
    n_dev = torch.cuda.device_count()
    dev = torch.device("cuda", D.device_for(local, n_dev))
    torch.cuda.set_device(dev)
    shared = local_world > n_dev
    rank, world = D.init("gloo" if shared else "nccl", dev)
    observed = D.observed_world(dev)  # what the process group really holds (all ranks agree)

    pkg = load_pkg()
    build = build_check(pkg)
    plan = pkg.Plan(frame_size=N_FFT, hop_size=HOP, device=dev.index)
    S, T = args.streams, T_LEN
    L = plan.output_length(T)

    # ---- weak phase (headline): S streams per rank
    x = synth_device(torch, S, T, dev, 0xC0FFEE + rank)
    y = torch.empty((S, L), dtype=torch.float32, device=dev)
    ramp, mine = {}, {}
    elapsed_max, kern_ms = timed_phase(plan, x, y, args.steps, args.warmup, D, dev, torch, ramp, mine)
    del x, y
    # every rank's device, kernel time and own wall time: who set the max (a first
    # 8-GPU run names its straggler)
    per = D.gather_over_ranks([kern_ms, mine["own_ms"]], dev)
    ranks = D.rank_report([p[0] for p in per], [p[1] for p in per], observed["device_keys"])

    samples_step_rank = S * T
    value = samples_step_rank * world * args.steps / elapsed_max / 1e6
    achieved_gbs = BYTES_PER_SAMPLE * samples_step_rank / (kern_ms * 1e-3) / 1e9
    fps = flop_per_sample(N_FFT, HOP)
    achieved_tf = fps * samples_step_rank / (kern_ms * 1e-3) / 1e12
    traffic, traffic_meta = load_pmc_traffic(f"{S}x{T}_N{N_FFT}_H{HOP}")

    # ---- strong phase (config 5): a fixed 8192-stream job sharded over the ranks
    strong = None
    if not args.no_strong and args.strong_streams > 0:
        lo, hi = D.stream_range(args.strong_streams, world, rank)
        xs = synth_device(torch, hi - lo, T, dev, 0x5EED0000 + lo)
        ys = torch.empty((hi - lo, L), dtype=torch.float32, device=dev)
        el_s, km_s = timed_phase(plan, xs, ys, args.strong_steps, 3, D, dev, torch)
        del xs, ys
        strong = {
            "workload": f"{args.strong_streams} streams x {T} samples in total (BASELINE config 5), "
                        f"rank r takes dist.stream_range({args.strong_streams}, {world}, r)",
            "scaling": "strong",
            "value": round(args.strong_streams * T * args.strong_steps / el_s / 1e6, 3),
            "unit": "Msamples/s",
            "steps": args.strong_steps,
            "ms_per_step": round(el_s / args.strong_steps * 1e3, 4),
            "streams_per_rank": [D.stream_range(args.strong_streams, world, r) for r in range(world)],
            "rank0_kernel_ms": round(km_s, 4),
        }

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline()
        except Exception as e:  # reported, never fatal to the GPU number
            cpu = {"value": None, "unit": "Msamples/s", "cores": 0, "kind": "port",
                   "sample": f"failed: {e}"}

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": observed["devices"],  # distinct devices (ranks may share one on a 1-GPU box)
            "ranks": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "clock_ramp": {"seconds": RAMP_S, "steps": ramp.get("clock_ramp_steps"),
                           "note": "untimed round trips before the warm-up steps while the GPU clock ramps"},
            "ms_per_step": round(elapsed_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: uniform[-0.5,0.5) float32 streams generated on device, HBM-resident",
            "config": {
                "workload": f"{S} mono streams x {T} samples (48 kHz, 10 s) per GPU, "
                            f"N={N_FFT} H={HOP} symmetric Hann, ZERO_PAD framing, "
                            "frame*w -> rfft -> irfft -> OLA(window inside) -> /max(norm,eps)",
                "streams_per_gpu": S,
                "samples_per_stream": T,
                "frame": N_FFT,
                "hop": HOP,
                "global_batch": S * world,
                "parallelism": f"streams sharded over {world} rank(s) on {min(world, n_dev)} device(s), "
                               f"no data-path collective (control plane over "
                               f"{'gloo' if shared else 'RCCL'})",
            },
            "roofline": {
                "bound": "valu",
                "achieved": round(achieved_gbs, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_meta,
                "kernel_ms": round(kern_ms, 4),
                "algorithmic_bytes_per_launch": BYTES_PER_SAMPLE * samples_step_rank,
                "valu": valu_block(fps, achieved_tf, traffic_meta.get("valu_issue"), kern_ms,
                                   S * plan.frame_count(T) / 2 / SIMDS),
                "note": "frac is the metric's HBM-roofline fraction (8 B/sample); the kernel "
                        "is bound on the VALU issue (DESIGN.md section 5), valu.frac prices "
                        "the same launches in SURVEY 8d flops",
            },
            "strong_scaling": strong,
            "ranks_report": ranks,
            "dist": {
                "backend": observed["backend"],
                "world_observed": observed["world"],
                "devices_observed": observed["devices"],
                "device_keys": observed["device_keys"],
                "note": "all-gathered over the process group before the timed phases: the world "
                        "size the group reports and the distinct devices (PCI ids) its ranks ran on",
            },
            "cpu_baseline": cpu,
            "build": build,
        }
        print(json.dumps(out), flush=True)
    D.finalize()


if __name__ == "__main__":
    main()
