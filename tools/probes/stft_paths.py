"""Probe: crlot_stft / crlot_istft_ola / masked round trip throughput per frame
size, walker vs staged form (the staged form is forced with 4-byte-aligned
output rows).  1024 streams x 480 000 samples.  Prints one JSON line per shape."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    from __graft_entry__ import load_pkg
    pkg = load_pkg()
    S, T = 1024, 480000
    g = torch.Generator(device="cuda").manual_seed(5)
    x = (torch.rand((S, T), generator=g, device="cuda") * 2 - 1) * 0.5

    def ev(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    shapes = [tuple(int(v) for v in a.split("/")) for a in sys.argv[1:]] or \
        [(256, 128), (512, 128), (1024, 256), (2048, 512), (4096, 1024)]
    for n, h in shapes:
        plan = pkg.Plan(frame_size=n, hop_size=h)
        plan.set_frame_pairing(os.environ.get("PROBE_PAIRING", "1") == "1")  # (0: the per-frame / staged forms)
        F, bins = plan.frame_count(T), n // 2 + 1
        spec = torch.empty((S, F, bins), dtype=torch.complex64, device="cuda")
        y = torch.empty((S, F * h), device="cuda")
        yo = torch.empty((S, F * h + 1), device="cuda")
        r = {"n": n, "h": h, "pairing": os.environ.get("PROBE_PAIRING", "1") == "1"}
        r["stft_ms"] = ev(lambda: plan.stft(x, spec))
        r["istft_walk_ms"] = ev(lambda: plan.istft_ola(spec, y))
        r["istft_staged_ms"] = ev(lambda: plan.istft_ola(spec, yo[:, :F * h]))
        del spec
        m = torch.rand((F, bins), generator=g, device="cuda")
        plan.set_spectral_mask(m)
        r["masked_walk_ms"] = ev(lambda: plan.roundtrip(x, y))
        r["masked_staged_ms"] = ev(lambda: plan.roundtrip(x, yo[:, :F * h]))
        plan.set_spectral_mask(None)
        r["roundtrip_ms"] = ev(lambda: plan.roundtrip(x, y))
        for k in list(r):
            if k.endswith("_ms"):
                r[k.replace("_ms", "_kMs")] = round(S * T / r[k] / 1e6, 1)
                r[k] = round(r[k], 3)
        print(json.dumps(r), flush=True)
        del y, yo, m
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
