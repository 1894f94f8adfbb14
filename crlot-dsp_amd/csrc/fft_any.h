// fft_any.h -- mixed-radix complex FFT of ANY length P, one wave per transform.
//
// The power-of-two sizes of the hot path use the register-resident kernels of
// fft_wave.h; this is the general path behind the same entry points for every
// other frame size kissfft accepts (kiss_fft.c factors any n): N = 960 / 480
// (20 / 10 ms at 48 kHz), N < 256, odd P = N/2, primes.
//
// Stockham autosort passes through two LDS buffers of P elements: the pass with
// radix R and current sub-length Ns runs butterflies j < P/R (strided over the
// wave's 64 lanes): x_r = src[j + r P/R] * W_{Ns R}^{r (j mod Ns)}, a length-R
// DFT, dst[(j / Ns) Ns R + j mod Ns + r Ns] = y.  Factors follow kiss_fft's
// kf_factor order (4s, then 2s, then odd primes).  Radix 2/3/4/5 butterflies
// are written out (the kf_bfly2/3/4/5 formulas), radix 7 as the symmetric
// odd-prime DFT (kissfft's generic butterfly computes the same sums in another
// order: a tolerance claim like every FFT here); any other prime R uses an
// O(R^2) DFT that streams its inputs from LDS, so no size is excluded.
// Twiddles come from per-pass tables in global memory (L1/L2-resident; no
// integer division or modulo in the butterfly loop); the inverse conjugates
// them.  IEEE f32, explicit FMAs.
#pragma once

#include "fft_wave.h"

namespace crlot {
namespace dev {
namespace any {

constexpr int kMaxPasses = 24;

// Per-pass constants, built on the host (kernels.hip make_any_plan):
// twiddles of pass i live at tw[off + (q-1) ns + jm] = W_{ns r}^{q jm} (q < r);
// a generic prime radix also has W_r^e at tw[woff + e], e < r.
struct PassDesc {
    int r, ns, off, woff;
    float rcp_ns;  // 1 / ns, for the quotient j / ns
};

struct Plan {
    int p;  // complex points
    int n_pass;
    PassDesc pass[kMaxPasses];
};

// floor(j / ns) for 0 <= j < 2^23 from a float reciprocal, corrected to exact.
__device__ __forceinline__ int fdiv(int j, int ns, float rcp) {
    int q = int(float(j) * rcp);
    q -= (q * ns > j);
    q += ((q + 1) * ns <= j);
    return q;
}

template <bool INV>
__device__ __forceinline__ cf twv(const cf* tw, int i) {
    const cf w = tw[i];
    return INV ? cf{w.r, -w.i} : w;
}

// One Stockham pass with a compile-time radix R (2, 3, 4, 5), src -> dst.
// (lane: this thread's first butterfly, step: the threads sharing the pass --
// one wave, or a whole workgroup between barriers; every butterfly computes the
// same whoever runs it)
template <bool INV, int R>
__device__ __forceinline__ void pass_r(const cf* __restrict__ src, cf* __restrict__ dst,
                                       const cf* __restrict__ tw, int p, const PassDesc& d,
                                       int lane, int step = 64) {
    const int ns = d.ns;
    const int m = p / R;  // butterflies
    const cf* twp = tw + d.off;
    for (int j = lane; j < m; j += step) {
        const int jb = fdiv(j, ns, d.rcp_ns);
        const int jm = j - jb * ns;
        const int ob = jb * ns * R + jm;
        const cf* t = twp + jm;  // t[(q-1) ns] = W^{q jm}
        cf x[R];
        x[0] = src[j];
#pragma unroll
        for (int q = 1; q < R; ++q) x[q] = cmul(src[j + q * m], twv<INV>(t, (q - 1) * ns));
        if constexpr (R == 2) {
            dft2<INV>(x[0], x[1]);
        } else if constexpr (R == 4) {
            dft4<INV>(x[0], x[1], x[2], x[3]);
        } else if constexpr (R == 3) {
            // kf_bfly3: y0 = a + b + c, y1/2 = a - (b + c)/2 -/+ i sin(2pi/3) (b - c)
            constexpr float s3 = 0.86602540378443864676f;
            const cf s = cadd(x[1], x[2]), dd = csub(x[1], x[2]);
            const cf h = {__builtin_fmaf(s.r, -0.5f, x[0].r), __builtin_fmaf(s.i, -0.5f, x[0].i)};
            const cf e = mul_mi<INV>(cf{dd.r * s3, dd.i * s3});  // -i sin(2pi/3) (b - c) forward
            x[0] = cadd(x[0], s);
            x[1] = cadd(h, e);
            x[2] = csub(h, e);
        } else if constexpr (R == 7) {
            // y_s = x0 + sum_q cos(2 pi qs/7) (x_q + x_{7-q}) -/+ i sum_q sin(2 pi qs/7) (x_q - x_{7-q})
            // (kissfft runs 7 through kf_bfly_generic: the same sums, another order)
            constexpr float c1 = 0.62348980185873353053f, c2 = -0.22252093395631440429f,
                            c3 = -0.90096886790241912624f;
            constexpr float s1 = 0.78183148246802980871f, s2 = 0.97492791218182360702f,
                            s3 = 0.43388373911755812048f;
            const cf x0 = x[0];
            const cf t1 = cadd(x[1], x[6]), t2 = cadd(x[2], x[5]), t3 = cadd(x[3], x[4]);
            const cf u1 = csub(x[1], x[6]), u2 = csub(x[2], x[5]), u3 = csub(x[3], x[4]);
            auto lin = [](const cf& b, float k1, const cf& p, float k2, const cf& q, float k3, const cf& r) {
                return cf{__builtin_fmaf(k3, r.r, __builtin_fmaf(k2, q.r, __builtin_fmaf(k1, p.r, b.r))),
                          __builtin_fmaf(k3, r.i, __builtin_fmaf(k2, q.i, __builtin_fmaf(k1, p.i, b.i)))};
            };
            const cf z = {0.0f, 0.0f};
            const cf a1 = lin(x0, c1, t1, c2, t2, c3, t3), b1 = lin(z, s1, u1, s2, u2, s3, u3);
            const cf a2 = lin(x0, c2, t1, c3, t2, c1, t3), b2 = lin(z, s2, u1, -s3, u2, -s1, u3);
            const cf a3 = lin(x0, c3, t1, c1, t2, c2, t3), b3 = lin(z, s3, u1, -s1, u2, s2, u3);
            x[0] = cadd(cadd(x0, t1), cadd(t2, t3));
            const cf e1 = mul_mi<INV>(b1), e2 = mul_mi<INV>(b2), e3 = mul_mi<INV>(b3);
            x[1] = cadd(a1, e1);
            x[6] = csub(a1, e1);
            x[2] = cadd(a2, e2);
            x[5] = csub(a2, e2);
            x[3] = cadd(a3, e3);
            x[4] = csub(a3, e3);
        } else {
            static_assert(R == 5, "radix");
            // kf_bfly5 with ya = W5^1, yb = W5^2
            constexpr float c1 = 0.30901699437494742410f, s1 = 0.95105651629515357212f;
            constexpr float c2 = -0.80901699437494742410f, s2 = 0.58778525229247312917f;
            const cf x0 = x[0];
            const cf s7 = cadd(x[1], x[4]), s10 = csub(x[1], x[4]);
            const cf s8 = cadd(x[2], x[3]), s9 = csub(x[2], x[3]);
            constexpr float sg = INV ? -1.0f : 1.0f;  // forward W5 = c - i s
            const cf s5 = {__builtin_fmaf(s7.r, c1, __builtin_fmaf(s8.r, c2, x0.r)),
                           __builtin_fmaf(s7.i, c1, __builtin_fmaf(s8.i, c2, x0.i))};
            const cf s6 = {sg * __builtin_fmaf(s10.i, s1, s9.i * s2),
                           -sg * __builtin_fmaf(s10.r, s1, s9.r * s2)};
            const cf s11 = {__builtin_fmaf(s7.r, c2, __builtin_fmaf(s8.r, c1, x0.r)),
                            __builtin_fmaf(s7.i, c2, __builtin_fmaf(s8.i, c1, x0.i))};
            const cf s12 = {sg * __builtin_fmaf(s9.i, -s1, s10.i * s2),
                            -sg * __builtin_fmaf(s9.r, -s1, s10.r * s2)};
            x[0] = {x0.r + s7.r + s8.r, x0.i + s7.i + s8.i};
            x[1] = cadd(s5, s6);
            x[4] = csub(s5, s6);
            x[2] = cadd(s11, s12);
            x[3] = csub(s11, s12);
        }
#pragma unroll
        for (int q = 0; q < R; ++q) dst[ob + q * ns] = x[q];
    }
}

// Any other (prime) radix: y_s = sum_q (x_q W^{q jm}) W_r^{q s}, inputs re-read per output.
template <bool INV>
__device__ __noinline__ void pass_generic(const cf* src, cf* dst, const cf* tw, int p,
                                          const PassDesc d, int lane, int step = 64) {
    const int r = d.r, ns = d.ns;
    const int m = p / r;
    const cf* wr = tw + d.woff;
    for (int j = lane; j < m; j += step) {
        const int jb = fdiv(j, ns, d.rcp_ns);
        const int jm = j - jb * ns;
        const int ob = jb * ns * r + jm;
        const cf* t = tw + d.off + jm;
        for (int s = 0; s < r; ++s) {
            cf acc = src[j];
            int e = 0;  // (q s) mod r
            for (int q = 1; q < r; ++q) {
                e += s;
                if (e >= r) e -= r;
                const cf xq = cmul(src[j + q * m], twv<INV>(t, (q - 1) * ns));
                acc = cadd(acc, cmul(xq, twv<INV>(wr, e)));
            }
            dst[ob + s * ns] = acc;
        }
    }
}

template <bool INV>
__device__ __forceinline__ void pass(const cf* src, cf* dst, const cf* tw, int p, const PassDesc& d,
                                     int lane, int step = 64) {
    switch (d.r) {
        case 2: pass_r<INV, 2>(src, dst, tw, p, d, lane, step); break;
        case 3: pass_r<INV, 3>(src, dst, tw, p, d, lane, step); break;
        case 4: pass_r<INV, 4>(src, dst, tw, p, d, lane, step); break;
        case 5: pass_r<INV, 5>(src, dst, tw, p, d, lane, step); break;
        case 7: pass_r<INV, 7>(src, dst, tw, p, d, lane, step); break;
        default: pass_generic<INV>(src, dst, tw, p, d, lane, step); break;
    }
}

// In-place (from the caller's view) P-point FFT of buf a; returns the buffer
// holding the result (a or b).  Every pass is followed by a wave fence.
template <bool INV>
__device__ __forceinline__ cf* fft(cf* a, cf* b, const Plan& pl, const cf* tw, int lane) {
    for (int i = 0; i < pl.n_pass; ++i) {
        pass<INV>(a, b, tw, pl.p, pl.pass[i], lane);
        wave_lds_fence();
        cf* t = a;
        a = b;
        b = t;
    }
    return a;
}

// kiss_fftr split of bin k < P from the P-point FFT z of the packed real frame:
// X[k], and X[P] when k = 0 (st: exp(-i pi (k/P + 1/2))).  k_fft_any's forward
// and the call server's (call_rt.hip) share it, so their spectra are bit-identical.
__device__ __forceinline__ void rsplit(const cf* z, int p, const cf* st, int k, cf& xk, cf& xp) {
    const cf zk = z[k];
    const cf fpnk = conj(z[(p - k) % p]);
    const cf f1 = cadd(zk, fpnk), f2 = csub(zk, fpnk);
    const cf w = st[k];
    const cf t = cmul(f2, cf{w.r * 0.5f, w.i * 0.5f});
    xk = {__builtin_fmaf(f1.r, 0.5f, t.r), __builtin_fmaf(f1.i, 0.5f, t.i)};
    if (k == 0) dc_split(zk, xk, xp);
}
// kiss_fftri merge of bins xk = X[k], xpk = X[P-k] into Z[k] (w = st[k])
__device__ __forceinline__ cf rmerge(const cf& xk, const cf& xpk, const cf& w, int k) {
    const cf fek = {xk.r + xpk.r, xk.i - xpk.i};
    const cf tmp = {xk.r - xpk.r, xk.i + xpk.i};
    return k == 0 ? dc_merge(xk, xpk)
                  : cf{__builtin_fmaf(tmp.r, w.r, __builtin_fmaf(tmp.i, w.i, fek.r)),
                       __builtin_fmaf(tmp.i, w.r, __builtin_fmaf(-tmp.r, w.i, fek.i))};
}

// kiss_fftr split -> gain -> kiss_fftri merge, src (Z) -> dst (Z'), with the
// arithmetic of fft_wave.h real_split_hook_merge.  spec (optional) gets X[k],
// k <= P.  st: exp(-i pi (k/P + 1/2)), k < P.
template <bool HAS_GAIN>
__device__ __forceinline__ void split_merge(const cf* src, cf* dst, int p, const cf* st,
                                            const float* gain, cf* spec, int lane) {
    for (int k = lane; k < p; k += 64) {
        const cf zk = src[k];
        const cf fpnk = conj(src[(p - k) % p]);
        const cf f1 = cadd(zk, fpnk);
        const cf f2 = csub(zk, fpnk);
        const cf w = st[k];
        const cf t = cmul(f2, cf{w.r * 0.5f, w.i * 0.5f});
        cf xk = {__builtin_fmaf(f1.r, 0.5f, t.r), __builtin_fmaf(f1.i, 0.5f, t.i)};
        cf xpk = {__builtin_fmaf(f1.r, 0.5f, -t.r), __builtin_fmaf(f1.i, -0.5f, t.i)};
        if (k == 0) dc_split(zk, xk, xpk);
        if constexpr (HAS_GAIN) {
            const float gk = gain[k], gpk = gain[p - k];
            xk = {xk.r * gk, xk.i * gk};
            xpk = {xpk.r * gpk, xpk.i * gpk};
        }
        if (spec) {
            spec[k] = xk;
            if (k == 0) spec[p] = xpk;
        }
        const cf fek = {xk.r + xpk.r, xk.i - xpk.i};
        const cf tmp = {xk.r - xpk.r, xk.i + xpk.i};
        dst[k] = k == 0 ? dc_merge(xk, xpk)
                        : cf{__builtin_fmaf(tmp.r, w.r, __builtin_fmaf(tmp.i, w.i, fek.r)),
                             __builtin_fmaf(tmp.i, w.r, __builtin_fmaf(-tmp.r, w.i, fek.i))};
    }
}

}  // namespace any
}  // namespace dev
}  // namespace crlot
