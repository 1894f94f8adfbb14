"""Pick, for every LDS exchange of the per-wave Stockham FFT, the XOR swizzle
phys(i) = i ^ (((i >> a) & mask) << b) that makes its ds_write_b64 scatter and
ds_read_b64 gather bank-conflict free (model: tools/lds_banks.py).  Emits the
table baked into crlot-dsp_amd/csrc/fft_wave.h (swz_params)."""
import sys
sys.argv = ["x"]
exec(open(__file__.replace("swizzle_search.py", "lds_banks.py")).read().split('if __name__ == "__main__":')[0])


def exch_cost(E, ns, R, f):
    tot = 0
    for b in range(E // R):
        for r in range(R):
            tot += cost([8 * f((((l + 64 * b) // ns) * ns * R + ((l + 64 * b) % ns) + r * ns))
                         for l in range(64)], "w64")[0]
    for m in range(E):
        tot += cost([8 * f(l + 64 * m) for l in range(64)], "r64")[0]
    return tot


def radix(P, ns, E):
    return 8 if (P // ns) % 8 == 0 and E >= 8 else 4 if (P // ns) % 4 == 0 and E >= 4 else 2


for E in (2, 4, 8, 16, 32):
    P = 64 * E
    ns = 1
    while ns < P:
        R = radix(P, ns, E)
        if ns * R < P:
            ideal = (E // R) * R * 4 + E * 2
            best = (exch_cost(E, ns, R, lambda i: i), (0, 0, 0))
            for a in range(1, 9):
                for mask in (1, 3, 7, 15):
                    for b in range(0, 5):
                        f = lambda i, a=a, mask=mask, b=b: i ^ (((i >> a) & mask) << b)
                        if b + mask.bit_length() > a:  # keep it a permutation inside aligned blocks
                            continue
                        c = exch_cost(E, ns, R, f)
                        if c < best[0]:
                            best = (c, (a, mask, b))
            print(f"E={E:2d} NS={ns:4d} R={R} ideal={ideal:4d} best={best[0]:4d} a,mask,b={best[1]}")
        ns *= R
