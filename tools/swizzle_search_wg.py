"""swizzle_search.py generalised to L lanes per frame (L = 64 * waves): every
wave w sees lanes t = 64 w + l, so each exchange's cost is summed over the L/64
waves.  Prints, per exchange (NS, R), the cost of the per-wave swizzles already
in fft_wave.h and the best XOR swizzle i ^ (((i >> a) & mask) << b)."""
import argparse
import sys
sys.argv = sys.argv[:1] + [a for a in sys.argv[1:]]
src = open(__file__.replace("swizzle_search_wg.py", "lds_banks.py")).read()
exec(src.split('if __name__ == "__main__":')[0])


def radix(P, ns, E):
    return 8 if (P // ns) % 8 == 0 and E >= 8 else 4 if (P // ns) % 4 == 0 and E >= 4 else 2


def exch_cost(E, L, ns, R, f):
    tot = 0
    for w in range(L // 64):
        for b in range(E // R):
            for r in range(R):
                tot += cost([8 * f((((64 * w + l + L * b) // ns) * ns * R + ((64 * w + l + L * b) % ns) + r * ns))
                             for l in range(64)], "w64")[0]
        for m in range(E):
            tot += cost([8 * f(64 * w + l + L * m) for l in range(64)], "r64")[0]
    return tot


def split_cost(E, L, f):
    P = L * E
    tot = 0
    for w in range(L // 64):
        for m in range(E):
            tot += cost([8 * f(64 * w + l + L * m) for l in range(64)], "w64")[0]
            tot += cost([8 * f((P - (64 * w + l + L * m)) & (P - 1)) for l in range(64)], "r64")[0]
    return tot


def current(ns, R):
    if ns == 1: return lambda i: i ^ ((i >> 4) & (R - 1))
    if ns == 2: return lambda i: i ^ ((i >> 3) & 3)
    if ns == 4 and R == 4: return lambda i: i ^ (((i >> 4) & 3) << 2)
    if ns == 4: return lambda i: i ^ (((i >> 3) & 3) << 1)
    if ns == 8 and R == 8: return lambda i: i ^ (((i >> 4) & 7) << 1)
    if ns == 8: return lambda i: i ^ (((i >> 4) & 1) << 3)
    return lambda i: i


ap = argparse.ArgumentParser()
ap.add_argument("--E", type=int, default=8)
ap.add_argument("--L", type=int, default=256)
args = ap.parse_args()
E, L = args.E, args.L
P = L * E
print(f"E={E} L={L} P={P} split (unswizzled) cost {split_cost(E, L, lambda i: i)} ideal {(L // 64) * E * 6}")
ns = 1
while ns < P:
    R = radix(P, ns, E)
    if ns * R < P:
        ideal = (L // 64) * ((E // R) * R * 4 + E * 2)
        cur = exch_cost(E, L, ns, R, current(ns, R))
        best = (exch_cost(E, L, ns, R, lambda i: i), (0, 0, 0))
        for a in range(1, 10):
            for mask in (1, 3, 7, 15):
                for b in range(0, 6):
                    if b + mask.bit_length() > a:
                        continue
                    f = lambda i, a=a, mask=mask, b=b: i ^ (((i >> a) & mask) << b)
                    c = exch_cost(E, L, ns, R, f)
                    if c < best[0]:
                        best = (c, (a, mask, b))
        print(f"NS={ns:4d} R={R} ideal={ideal:4d} current={cur:4d} best={best[0]:4d} a,mask,b={best[1]}")
    ns *= R
