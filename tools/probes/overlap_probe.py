"""Probe: does overlapping two K_pair launches on two HIP streams raise the
headline throughput (two ranks sharing one GPU measured +4-7 %)?  Times the
1024-stream batch as one launch, as two 512-stream halves on two streams, and
two full batches on two streams."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from __graft_entry__ import load_pkg
    pkg = load_pkg()
    S, T = 1024, 480000
    plan = pkg.Plan(frame_size=1024, hop_size=256)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = (torch.rand((2 * S, T), generator=g, device="cuda") * 2 - 1) * 0.5
    L = plan.output_length(T)
    y = torch.empty((2 * S, L), device="cuda")
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()

    def one():
        plan.roundtrip(x[:S], y[:S])

    def halves():
        h = S // 2
        sa.wait_stream(torch.cuda.current_stream())
        sb.wait_stream(torch.cuda.current_stream())
        plan.roundtrip(x[:h], y[:h], stream=int(sa.cuda_stream))
        plan.roundtrip(x[h:S], y[h:S], stream=int(sb.cuda_stream))
        torch.cuda.current_stream().wait_stream(sa)
        torch.cuda.current_stream().wait_stream(sb)

    def two_full():
        sa.wait_stream(torch.cuda.current_stream())
        sb.wait_stream(torch.cuda.current_stream())
        plan.roundtrip(x[:S], y[:S], stream=int(sa.cuda_stream))
        plan.roundtrip(x[S:], y[S:], stream=int(sb.cuda_stream))
        torch.cuda.current_stream().wait_stream(sa)
        torch.cuda.current_stream().wait_stream(sb)

    def two_serial():
        plan.roundtrip(x[:S], y[:S])
        plan.roundtrip(x[S:], y[S:])

    for rnd in range(2):
        for name, fn, samples in (("one launch", one, S * T), ("two halves, two streams", halves, S * T),
                                  ("two batches, one stream", two_serial, 2 * S * T),
                                  ("two batches, two streams", two_full, 2 * S * T)):
            t_end = time.perf_counter() + 0.2
            while time.perf_counter() < t_end:
                fn()
                torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(10):
                    fn()
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t0) / 10)
            ms = sorted(ts)[2] * 1e3
            print(json.dumps({"round": rnd, "case": name, "ms": round(ms, 4),
                              "Msamples_s": round(samples / ms / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
