// fft_wave.h -- one-wavefront complex FFT building blocks for gfx950 (CDNA4).
//
// A real frame of N samples is transformed as a complex sequence of P = N/2
// points z[n] = x[2n] + i x[2n+1] (the kiss_fftr split, kiss_fftr.c), held by
// ONE 64-lane wave: lane l owns z[l + 64 m], m = 0..E-1, E = P/64 ("lane-major").
//
// The complex FFT is a radix-8/4/2 Stockham autosort (decimation in time):
//   pass with current sub-length Ns and radix R: butterfly j in [0, P/R) reads
//   x[j + r P/R] (r < R), twiddles by W_{Ns R}^{r (j mod Ns)}, runs a length-R
//   DFT and writes y[(j / Ns) Ns R + (j mod Ns) + r Ns].
// With j = lane + 64 b every read is lane-major (no data movement), the first
// pass (Ns = 1) needs no twiddles, and the LAST pass writes lane-major too, so a
// P-point FFT costs (passes - 1) LDS exchanges and leaves its output in natural
// order in registers.  Exchanges go through a per-wave LDS buffer of P elements
// under a per-exchange XOR swizzle that keeps them bank-conflict free.
//
// Arithmetic is IEEE f32; the translation unit is built with -ffp-contract=off,
// so every FMA below is explicit.
#pragma once

#include <hip/hip_runtime.h>

namespace crlot {
namespace dev {

struct cf {
    float r, i;
};

__device__ __forceinline__ cf cadd(cf a, cf b) { return {a.r + b.r, a.i + b.i}; }
__device__ __forceinline__ cf csub(cf a, cf b) { return {a.r - b.r, a.i - b.i}; }
__device__ __forceinline__ cf conj(cf a) { return {a.r, -a.i}; }
// a * w with two FMAs
__device__ __forceinline__ cf cmul(cf a, cf w) {
    return {__builtin_fmaf(a.r, w.r, -(a.i * w.i)), __builtin_fmaf(a.r, w.i, a.i * w.r)};
}
// a * conj(w)
__device__ __forceinline__ cf cmulc(cf a, cf w) {
    return {__builtin_fmaf(a.r, w.r, a.i * w.i), __builtin_fmaf(a.i, w.r, -(a.r * w.i))};
}
// multiply by -i (forward) / +i (inverse)
template <bool INV>
__device__ __forceinline__ cf mul_mi(cf a) {
    return INV ? cf{-a.i, a.r} : cf{a.i, -a.r};
}

// ------------------------------------------------------------- small DFTs
template <bool INV>
__device__ __forceinline__ void dft2(cf& a, cf& b) {
    cf t = a;
    a = cadd(t, b);
    b = csub(t, b);
}

template <bool INV>
__device__ __forceinline__ void dft4(cf& x0, cf& x1, cf& x2, cf& x3) {
    cf s0 = cadd(x0, x2), s1 = csub(x0, x2), s2 = cadd(x1, x3), s3 = csub(x1, x3);
    cf t = mul_mi<INV>(s3);
    x0 = cadd(s0, s2);
    x2 = csub(s0, s2);
    x1 = cadd(s1, t);
    x3 = csub(s1, t);
}

template <bool INV>
__device__ __forceinline__ void dft8(cf* x) {
    constexpr float c = 0.70710678118654752440f;
    cf a0 = x[0], a1 = x[2], a2 = x[4], a3 = x[6];
    cf b0 = x[1], b1 = x[3], b2 = x[5], b3 = x[7];
    dft4<INV>(a0, a1, a2, a3);
    dft4<INV>(b0, b1, b2, b3);
    // W8^1 b1 = (p1, q1) c and W8^3 b3 = (p3, q3) c, folded into FMAs
    float p1, q1, p3, q3;
    if (!INV) {
        p1 = b1.r + b1.i;
        q1 = b1.i - b1.r;
        p3 = b3.i - b3.r;
        q3 = -(b3.r + b3.i);
    } else {
        p1 = b1.r - b1.i;
        q1 = b1.r + b1.i;
        p3 = -(b3.r + b3.i);
        q3 = b3.r - b3.i;
    }
    cf w2 = mul_mi<INV>(b2);
    x[0] = cadd(a0, b0);
    x[4] = csub(a0, b0);
    x[1] = {__builtin_fmaf(p1, c, a1.r), __builtin_fmaf(q1, c, a1.i)};
    x[5] = {__builtin_fmaf(p1, -c, a1.r), __builtin_fmaf(q1, -c, a1.i)};
    x[2] = cadd(a2, w2);
    x[6] = csub(a2, w2);
    x[3] = {__builtin_fmaf(p3, c, a3.r), __builtin_fmaf(q3, c, a3.i)};
    x[7] = {__builtin_fmaf(p3, -c, a3.r), __builtin_fmaf(q3, -c, a3.i)};
}

template <int R, bool INV>
__device__ __forceinline__ void dftR(cf* x) {
    if constexpr (R == 2) {
        dft2<INV>(x[0], x[1]);
    } else if constexpr (R == 4) {
        dft4<INV>(x[0], x[1], x[2], x[3]);
    } else {
        static_assert(R == 8, "radix");
        dft8<INV>(x);
    }
}

// ------------------------------------------------------------- LDS exchange
// Each exchange stores the pass outputs at their Stockham positions and reads
// them back lane-major.  The XOR swizzle below (a permutation inside aligned
// blocks, so the buffer stays P elements) makes both the ds_write_b64 scatter
// and the ds_read_b64 gather bank-conflict free for every exchange of every
// supported size; it was found by tools/swizzle_search.py with the gfx950 LDS
// model in tools/lds_banks.py (ds_write_b64: 16-lane groups, 32 banks;
// ds_read_b64: 32-lane groups, 64 banks).
template <int NS, int R>
__device__ __forceinline__ int swz(int i) {
    if constexpr (NS == 1) return i ^ ((i >> 4) & (R - 1));
    else if constexpr (NS == 2) return i ^ ((i >> 3) & 3);
    else if constexpr (NS == 4 && R == 4) return i ^ (((i >> 4) & 3) << 2);
    else if constexpr (NS == 4) return i ^ (((i >> 3) & 3) << 1);
    else if constexpr (NS == 8 && R == 8) return i ^ (((i >> 4) & 7) << 1);
    else if constexpr (NS == 8) return i ^ (((i >> 4) & 1) << 3);
    else return i;
}

// Orders this wave's LDS writes before its later LDS reads (and vice versa)
// without a workgroup barrier: DS instructions of one wave execute in order,
// the fences only stop the compiler from moving memory ops across.
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Radix schedule: largest radix in {8,4,2} dividing what is left, not above E.
__host__ __device__ constexpr int radix_for(int rem, int e) {
    return (rem % 8 == 0 && e >= 8) ? 8 : (rem % 4 == 0 && e >= 4) ? 4 : 2;
}

// Per-pass twiddle table layout (host + device): pass (NS > 1, R) owns
// (R-1)*NS entries T[(r-1)*NS + jm] = W_{NS R}^{r jm}, jm = j mod NS, so a
// wave's twiddle reads are contiguous (or broadcast) -- conflict free.
__host__ __device__ constexpr int twiddle_table_size(int e) {
    int p = 64 * e, ns = 1, n = 0;
    while (ns < p) {
        const int r = radix_for(p / ns, e);
        if (ns > 1) n += (r - 1) * ns;
        ns *= r;
    }
    return n;
}

// Per-lane twiddles of one pass: w[b][r-1] for butterfly j = lane + 64 b.
template <int E, int R, int NS>
struct PassTw {
    cf w[E / R][R - 1];
};

template <int E, int R, int NS, int TOFF>
__device__ __forceinline__ void load_pass_tw(PassTw<E, R, NS>& t, const cf* twp, int lane) {
#pragma unroll
    for (int b = 0; b < E / R; ++b)
#pragma unroll
        for (int r = 1; r < R; ++r) t.w[b][r - 1] = twp[TOFF + (r - 1) * NS + (lane + 64 * b) % NS];
}

// One Stockham pass on the lane-major registers v[E]; NS = current sub-length.
// Twiddles arrive pre-loaded in `tw` (unused when NS == 1).
template <int E, int R, int NS, bool INV>
__device__ __forceinline__ void stockham_compute(cf (&v)[E], const PassTw<E, R, NS>& tw) {
    constexpr int B = E / R;  // butterflies per lane
#pragma unroll
    for (int b = 0; b < B; ++b) {
        cf x[R];
#pragma unroll
        for (int r = 0; r < R; ++r) x[r] = v[b + r * B];
        if constexpr (NS > 1) {
#pragma unroll
            for (int r = 1; r < R; ++r) x[r] = INV ? cmulc(x[r], tw.w[b][r - 1]) : cmul(x[r], tw.w[b][r - 1]);
        }
        dftR<R, INV>(x);
#pragma unroll
        for (int r = 0; r < R; ++r) v[b + r * B] = x[r];
    }
}

// y[(j/NS) NS R + (j mod NS) + r NS] -> LDS, then read back x[lane + 64 m].
template <int E, int R, int NS>
__device__ __forceinline__ void stockham_exchange(cf (&v)[E], cf* buf, int lane) {
    constexpr int B = E / R;
#ifdef CRLOT_ABL_NOXCHG  // timing-only ablation: wrong results
    return;
#endif
#pragma unroll
    for (int b = 0; b < B; ++b) {
        const int j = lane + 64 * b;
        const int base = (j / NS) * NS * R + (j % NS);
#pragma unroll
        for (int r = 0; r < R; ++r) buf[swz<NS, R>(base + r * NS)] = v[b + r * B];
    }
    wave_lds_fence();
#pragma unroll
    for (int m = 0; m < E; ++m) v[m] = buf[swz<NS, R>(lane + 64 * m)];
    wave_lds_fence();
}

// Pass NS (twiddles already in `tw`); the next pass's twiddles are issued
// BEFORE this pass's exchange so their LDS latency hides under it.
template <int E, int NS, int TOFF, bool INV, typename TW>
__device__ __forceinline__ void fft_passes(cf (&v)[E], cf* buf, const cf* twp, int lane,
                                           const TW& tw) {
    constexpr int P = 64 * E;
    if constexpr (NS < P) {
        constexpr int R = radix_for(P / NS, E);
        stockham_compute<E, R, NS, INV>(v, tw);
        if constexpr (NS * R < P) {
            constexpr int NS2 = NS * R;
            constexpr int R2 = radix_for(P / NS2, E);
            constexpr int TOFF2 = TOFF + (NS > 1 ? (R - 1) * NS : 0);
            PassTw<E, R2, NS2> tw2;
            load_pass_tw<E, R2, NS2, TOFF2>(tw2, twp, lane);
            stockham_exchange<E, R, NS>(v, buf, lane);
            fft_passes<E, NS2, TOFF2, INV>(v, buf, twp, lane, tw2);
        }
    }
}

// In-place P-point complex FFT (unnormalised) of the lane-major registers.
// twp: per-pass forward twiddles (inverse uses their conjugates).
template <int E, bool INV>
__device__ __forceinline__ void fft_wave(cf (&v)[E], cf* buf, const cf* twp, int lane) {
    constexpr int R = radix_for(64 * E, E);
    PassTw<E, R, 1> none;
    fft_passes<E, 1, 0, INV>(v, buf, twp, lane, none);
}

// ---- two frames per wave: the same passes on v0 and v1, sharing the twiddle
// loads and one fence pair per exchange, so the two instruction streams interleave.
template <int E, int R, int NS>
__device__ __forceinline__ void stockham_exchange2(cf (&v0)[E], cf (&v1)[E], cf* buf0, cf* buf1,
                                                   int lane) {
    constexpr int B = E / R;
#pragma unroll
    for (int b = 0; b < B; ++b) {
        const int j = lane + 64 * b;
        const int base = (j / NS) * NS * R + (j % NS);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            buf0[swz<NS, R>(base + r * NS)] = v0[b + r * B];
            buf1[swz<NS, R>(base + r * NS)] = v1[b + r * B];
        }
    }
    wave_lds_fence();
#pragma unroll
    for (int m = 0; m < E; ++m) {
        v0[m] = buf0[swz<NS, R>(lane + 64 * m)];
        v1[m] = buf1[swz<NS, R>(lane + 64 * m)];
    }
    wave_lds_fence();
}

template <int E, int NS, int TOFF, bool INV, typename TW>
__device__ __forceinline__ void fft_passes2(cf (&v0)[E], cf (&v1)[E], cf* buf0, cf* buf1,
                                            const cf* twp, int lane, const TW& tw) {
    constexpr int P = 64 * E;
    if constexpr (NS < P) {
        constexpr int R = radix_for(P / NS, E);
        stockham_compute<E, R, NS, INV>(v0, tw);
        stockham_compute<E, R, NS, INV>(v1, tw);
        if constexpr (NS * R < P) {
            constexpr int NS2 = NS * R;
            constexpr int R2 = radix_for(P / NS2, E);
            constexpr int TOFF2 = TOFF + (NS > 1 ? (R - 1) * NS : 0);
            PassTw<E, R2, NS2> tw2;
            load_pass_tw<E, R2, NS2, TOFF2>(tw2, twp, lane);
            stockham_exchange2<E, R, NS>(v0, v1, buf0, buf1, lane);
            fft_passes2<E, NS2, TOFF2, INV>(v0, v1, buf0, buf1, twp, lane, tw2);
        }
    }
}

template <int E, bool INV>
__device__ __forceinline__ void fft_wave2(cf (&v0)[E], cf (&v1)[E], cf* buf0, cf* buf1,
                                          const cf* twp, int lane) {
    constexpr int R = radix_for(64 * E, E);
    PassTw<E, R, 1> none;
    fft_passes2<E, 1, 0, INV>(v0, v1, buf0, buf1, twp, lane, none);
}

// All passes' per-lane twiddles held in registers (they do not depend on the
// frame, so a wave that walks many frames loads them once).
template <int E, int NS, bool END = (NS >= 64 * E)>
struct TwChain {
    static constexpr int R = radix_for(64 * E / NS, E);
    PassTw<E, R, NS> here;
    TwChain<E, NS * R> next;
};
template <int E, int NS>
struct TwChain<E, NS, true> {};

template <int E, int NS, int TOFF>
__device__ __forceinline__ void load_chain(TwChain<E, NS>& c, const cf* twp, int lane) {
    if constexpr (NS < 64 * E) {
        constexpr int R = radix_for(64 * E / NS, E);
        if constexpr (NS > 1) load_pass_tw<E, R, NS, TOFF>(c.here, twp, lane);
        load_chain<E, NS * R, TOFF + (NS > 1 ? (R - 1) * NS : 0)>(c.next, twp, lane);
    }
}

template <int E, int NS, bool INV>
__device__ __forceinline__ void fft_passes_reg(cf (&v)[E], cf* buf, const TwChain<E, NS>& c,
                                               int lane) {
    constexpr int P = 64 * E;
    if constexpr (NS < P) {
        constexpr int R = radix_for(P / NS, E);
        stockham_compute<E, R, NS, INV>(v, c.here);
        if constexpr (NS * R < P) {
            stockham_exchange<E, R, NS>(v, buf, lane);
            fft_passes_reg<E, NS * R, INV>(v, buf, c.next, lane);
        }
    }
}

template <int E, bool INV>
__device__ __forceinline__ void fft_wave_reg(cf (&v)[E], cf* buf, const TwChain<E, 1>& c,
                                             int lane) {
    fft_passes_reg<E, 1, INV>(v, buf, c, lane);
}

// ------------------------------------------------------------- workgroup FFT
// The same Stockham schedule spread over L = 64 * W lanes of one workgroup
// (lane t owns z[t + L m], m < E), for frames too large for one wave's
// registers (N = 4096 at E = 8, L = 256).  All twiddles live in registers
// (loaded once per kernel; they do not depend on the frame), exchanges go
// through LDS with ONE workgroup barrier each: consecutive exchanges alternate
// between two buffers, so a buffer is rewritten only after the next exchange's
// barrier, which every wave reaches after finishing its reads of it.  The
// per-wave XOR swizzles above stay bank-conflict free at L = 256
// (tools/swizzle_search_wg.py).
template <int E, int R, int NS, int L, int TOFF>
__device__ __forceinline__ void load_pass_tw_wg(PassTw<E, R, NS>& t, const cf* twp, int lane) {
#pragma unroll
    for (int b = 0; b < E / R; ++b)
#pragma unroll
        for (int r = 1; r < R; ++r) t.w[b][r - 1] = twp[TOFF + (r - 1) * NS + (lane + L * b) % NS];
}

template <int E, int L, int NS, bool END = (NS >= L * E)>
struct TwChainWg {
    static constexpr int R = radix_for(L * E / NS, E);
    PassTw<E, R, NS> here;
    TwChainWg<E, L, NS * R> next;
};
template <int E, int L, int NS>
struct TwChainWg<E, L, NS, true> {};

template <int E, int L, int NS, int TOFF>
__device__ __forceinline__ void load_chain_wg(TwChainWg<E, L, NS>& c, const cf* twp, int lane) {
    if constexpr (NS < L * E) {
        constexpr int R = radix_for(L * E / NS, E);
        if constexpr (NS > 1) load_pass_tw_wg<E, R, NS, L, TOFF>(c.here, twp, lane);
        load_chain_wg<E, L, NS * R, TOFF + (NS > 1 ? (R - 1) * NS : 0)>(c.next, twp, lane);
    }
}

template <int E, int R, int NS, int L>
__device__ __forceinline__ void stockham_exchange_wg(cf (&v)[E], cf* buf, int lane) {
    constexpr int B = E / R;
#pragma unroll
    for (int b = 0; b < B; ++b) {
        const int j = lane + L * b;
        const int base = (j / NS) * NS * R + (j % NS);
#pragma unroll
        for (int r = 0; r < R; ++r) buf[swz<NS, R>(base + r * NS)] = v[b + r * B];
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < E; ++m) v[m] = buf[swz<NS, R>(lane + L * m)];
}

// XI = index of the next exchange; it uses buffer XI & 1.
template <int E, int L, int NS, int XI, bool INV>
__device__ __forceinline__ void fft_passes_wg(cf (&v)[E], cf* buf0, cf* buf1,
                                              const TwChainWg<E, L, NS>& c, int lane) {
    constexpr int P = L * E;
    if constexpr (NS < P) {
        constexpr int R = radix_for(P / NS, E);
        stockham_compute<E, R, NS, INV>(v, c.here);
        if constexpr (NS * R < P) {
            stockham_exchange_wg<E, R, NS, L>(v, (XI & 1) ? buf1 : buf0, lane);
            fft_passes_wg<E, L, NS * R, XI + 1, INV>(v, buf0, buf1, c.next, lane);
        }
    }
}

// Number of exchanges of one P-point FFT.
__host__ __device__ constexpr int fft_exchanges(int p, int e) {
    int ns = 1, n = 0;
    while (ns < p) {
        const int r = radix_for(p / ns, e);
        if (ns * r < p) ++n;
        ns *= r;
    }
    return n;
}

// ------------------------------------------------------------- sanitize
// KissFftPlan sanitize (kissfft_adapter.cc:102-110, 156-163):
// NaN/Inf -> 0, |v| < 1e-30 -> 0.
__device__ __forceinline__ float sanit(float v) {
#ifdef CRLOT_ABL_NOSANIT  // timing-only ablation
    return v;
#endif
    const float a = __builtin_fabsf(v);
    return (a >= 1e-30f && a <= 3.402823466e+38f) ? v : 0.0f;
}

// sanit(v * 2^-k) == sanit_scaled<2^k>(v) * 2^-k exactly (v * 2^-k is exact for
// every v the threshold keeps; inf/NaN still map to 0): lets the fused kernels
// fold the inverse's 1/N into the synthesis window.
template <int NPOW2>
__device__ __forceinline__ float sanit_scaled(float v) {
#ifdef CRLOT_ABL_NOSANIT
    return v;
#endif
    constexpr float lo = 1e-30f * float(NPOW2);
    const float a = __builtin_fabsf(v);
    return (a >= lo && a <= 3.402823466e+38f) ? v : 0.0f;
}
// sanit_scaled for a v known to be finite (K_pair's paired regime): the threshold alone.
template <int NPOW2>
__device__ __forceinline__ float sanit_scaled_finite(float v) {
#ifdef CRLOT_ABL_NOSANIT
    return v;
#endif
    constexpr float lo = 1e-30f * float(NPOW2);
    return __builtin_fabsf(v) >= lo ? v : 0.0f;
}

// ------------------------------------------------------------- real split
// DC / Nyquist bins exactly as kissfft forms them: kiss_fftr sets
// X[0] = (Z0.r + Z0.i, 0), X[P] = (Z0.r - Z0.i, 0); kiss_fftri rebuilds
// Z'[0] = (X0.r + XP.r, X0.r - XP.r) from the REAL parts only (kiss_fftr.c).
__device__ __forceinline__ void dc_split(cf z0, cf& x0, cf& xp) {
    x0 = {z0.r + z0.i, 0.0f};
    xp = {z0.r - z0.i, 0.0f};
}
__device__ __forceinline__ cf dc_merge(cf x0, cf xp) { return {x0.r + xp.r, x0.r - xp.r}; }

// Given Z = FFT_P(z) lane-major in v, produce the spectrum X[k] (k = 0..P) of
// the real 2P-point frame (kiss_fftr), apply the optional real per-bin gain
// (spectral hook; the reference's step is the identity), then rebuild Z' such
// that IFFT_P(Z') is the unnormalised inverse real FFT (kiss_fftri).  Each lane
// works on its own k = lane + 64 m and needs Z[P-k], read from LDS.
//   st : super twiddles exp(-i pi (k/P + 1/2)), k in [0, P)
//   sth: 0.5 * st (exact), so X[k] = fma(f1, 1/2, f2 * sth) with no extra multiply
// spec (optional): receives X[k] for k = lane + 64 m and X[P] from lane 0.
template <int E, bool HAS_GAIN, bool WRITE_SPEC>
__device__ __forceinline__ void real_split_hook_merge(cf (&v)[E], cf* buf, const cf* st,
                                                      const cf* sth, const float* gain,
                                                      int lane, cf* spec = nullptr) {
    constexpr int P = 64 * E;
#pragma unroll
    for (int m = 0; m < E; ++m) buf[lane + 64 * m] = v[m];  // conflict free unswizzled
    wave_lds_fence();
    cf zp[E];
#pragma unroll
    for (int m = 0; m < E; ++m) zp[m] = buf[(P - (lane + 64 * m)) & (P - 1)];
    wave_lds_fence();
#ifdef CRLOT_ABL_NOSPLITX  // timing-only ablation: wrong results
#pragma unroll
    for (int m = 0; m < E; ++m) zp[m] = v[E - 1 - m];
#endif
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const int k = lane + 64 * m;
        const cf zk = v[m];
        const cf fpnk = conj(zp[m]);
        const cf f1 = cadd(zk, fpnk);
        const cf f2 = csub(zk, fpnk);
        const cf t = cmul(f2, sth[k]);  // 0.5 * f2 * st
        cf xk = {__builtin_fmaf(f1.r, 0.5f, t.r), __builtin_fmaf(f1.i, 0.5f, t.i)};
        cf xpk = {__builtin_fmaf(f1.r, 0.5f, -t.r), __builtin_fmaf(f1.i, -0.5f, t.i)};  // X[P-k]
        if (m == 0 && lane == 0) dc_split(zk, xk, xpk);
        if constexpr (HAS_GAIN) {
            const float gk = gain[k], gpk = gain[P - k];
            xk = {xk.r * gk, xk.i * gk};
            xpk = {xpk.r * gpk, xpk.i * gpk};
        }
        if constexpr (WRITE_SPEC) {
            spec[k] = xk;
            if (k == 0) spec[P] = xpk;
        }
        // kiss_fftri merge: Z'[k] = (X[k] + conj X[P-k]) + (X[k] - conj X[P-k]) conj(st)
        const cf w = st[k];
        const cf fek = {xk.r + xpk.r, xk.i - xpk.i};
        const cf tmp = {xk.r - xpk.r, xk.i + xpk.i};
        v[m].r = __builtin_fmaf(tmp.r, w.r, __builtin_fmaf(tmp.i, w.i, fek.r));
        v[m].i = __builtin_fmaf(tmp.i, w.r, __builtin_fmaf(-tmp.r, w.i, fek.i));
        if (m == 0 && lane == 0) v[0] = dc_merge(xk, xpk);
    }
}

// One element of the split -> gain -> merge (the arithmetic of real_split_hook_merge).
template <bool HAS_GAIN>
__device__ __forceinline__ cf split_merge_elem(cf zk, cf zp, cf w, cf wh, const float* gain, int k,
                                               int P, bool dc) {
    const cf fpnk = conj(zp);
    const cf f1 = cadd(zk, fpnk);
    const cf f2 = csub(zk, fpnk);
    const cf t = cmul(f2, wh);
    cf xk = {__builtin_fmaf(f1.r, 0.5f, t.r), __builtin_fmaf(f1.i, 0.5f, t.i)};
    cf xpk = {__builtin_fmaf(f1.r, 0.5f, -t.r), __builtin_fmaf(f1.i, -0.5f, t.i)};
    if (dc) dc_split(zk, xk, xpk);
    if constexpr (HAS_GAIN) {
        const float gk = gain[k], gpk = gain[P - k];
        xk = {xk.r * gk, xk.i * gk};
        xpk = {xpk.r * gpk, xpk.i * gpk};
    }
    const cf fek = {xk.r + xpk.r, xk.i - xpk.i};
    const cf tmp = {xk.r - xpk.r, xk.i + xpk.i};
    cf o = {__builtin_fmaf(tmp.r, w.r, __builtin_fmaf(tmp.i, w.i, fek.r)),
            __builtin_fmaf(tmp.i, w.r, __builtin_fmaf(-tmp.r, w.i, fek.i))};
    if (dc) o = dc_merge(xk, xpk);
    return o;
}

// Two frames at once (fft_wave2 companion): the st/sth reads are shared.
template <int E, bool HAS_GAIN>
__device__ __forceinline__ void real_split_hook_merge2(cf (&v0)[E], cf (&v1)[E], cf* buf0, cf* buf1,
                                                       const cf* st, const cf* sth,
                                                       const float* gain, int lane) {
    constexpr int P = 64 * E;
#pragma unroll
    for (int m = 0; m < E; ++m) {
        buf0[lane + 64 * m] = v0[m];
        buf1[lane + 64 * m] = v1[m];
    }
    wave_lds_fence();
    cf zp0[E], zp1[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const int pk = (P - (lane + 64 * m)) & (P - 1);
        zp0[m] = buf0[pk];
        zp1[m] = buf1[pk];
    }
    wave_lds_fence();
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const int k = lane + 64 * m;
        const cf w = st[k], wh = sth[k];
        const bool dc = m == 0 && lane == 0;
        v0[m] = split_merge_elem<HAS_GAIN>(v0[m], zp0[m], w, wh, gain, k, P, dc);
        v1[m] = split_merge_elem<HAS_GAIN>(v1[m], zp1[m], w, wh, gain, k, P, dc);
    }
}

// Workgroup form of the split/hook/merge: st[m] = st(k) for k = lane + L m in
// registers (sth = 0.5 st is formed on the fly, exact), the partner Z[P-k]
// exchanged through `buf` with one barrier.  Same arithmetic as above.
template <int E, int L, bool HAS_GAIN>
__device__ __forceinline__ void real_split_hook_merge_wg(cf (&v)[E], cf* buf, const cf (&st)[E],
                                                         const float* gain, int lane) {
    constexpr int P = L * E;
#pragma unroll
    for (int m = 0; m < E; ++m) buf[lane + L * m] = v[m];
    __syncthreads();
    cf zp[E];
#pragma unroll
    for (int m = 0; m < E; ++m) zp[m] = buf[(P - (lane + L * m)) & (P - 1)];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const int k = lane + L * m;
        const cf zk = v[m];
        const cf fpnk = conj(zp[m]);
        const cf f1 = cadd(zk, fpnk);
        const cf f2 = csub(zk, fpnk);
        const cf w = st[m];
        const cf t = cmul(f2, cf{w.r * 0.5f, w.i * 0.5f});
        cf xk = {__builtin_fmaf(f1.r, 0.5f, t.r), __builtin_fmaf(f1.i, 0.5f, t.i)};
        cf xpk = {__builtin_fmaf(f1.r, 0.5f, -t.r), __builtin_fmaf(f1.i, -0.5f, t.i)};
        if (m == 0 && lane == 0) dc_split(zk, xk, xpk);
        if constexpr (HAS_GAIN) {
            const float gk = gain[k], gpk = gain[P - k];
            xk = {xk.r * gk, xk.i * gk};
            xpk = {xpk.r * gpk, xpk.i * gpk};
        }
        const cf fek = {xk.r + xpk.r, xk.i - xpk.i};
        const cf tmp = {xk.r - xpk.r, xk.i + xpk.i};
        v[m].r = __builtin_fmaf(tmp.r, w.r, __builtin_fmaf(tmp.i, w.i, fek.r));
        v[m].i = __builtin_fmaf(tmp.i, w.r, __builtin_fmaf(-tmp.r, w.i, fek.i));
        if (m == 0 && lane == 0) v[0] = dc_merge(xk, xpk);
    }
}

// ------------------------------------------------------------- buffer access
// Raw buffer descriptors: 32-bit offsets, hardware range check (loads past
// num_bytes return 0, stores past it are dropped).  Build them from
// wave-uniform values only (readfirstlane'd), see cdna_hip_programming.md T20.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    const uint64_t a = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(a));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(a >> 32));
    const uint64_t b = (uint64_t(hi) << 32) | lo;
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(b), 0,
                                             int(__builtin_amdgcn_readfirstlane(bytes)),
                                             0x00020000);
}
// NOTE (ROCm 7.2 clang): __builtin_bit_cast applied directly to an element of the
// vector returned by raw_buffer_load_b64/b128 is miscompiled into a single-dword
// load (upper half garbage); copying each element to a scalar first is correct.
__device__ __forceinline__ float2 bload2(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0);
    const unsigned lo = v[0], hi = v[1];
    return make_float2(__builtin_bit_cast(float, lo), __builtin_bit_cast(float, hi));
}
__device__ __forceinline__ float bload1(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
__device__ __forceinline__ void bstore2(float2 v, __amdgpu_buffer_rsrc_t r, int voff, int soff) {
    typedef unsigned int u2 __attribute__((ext_vector_type(2)));
    const float lo = v.x, hi = v.y;  // (scalars first: tools/bitcast_lint.py)
    u2 w = {__builtin_bit_cast(unsigned, lo), __builtin_bit_cast(unsigned, hi)};
    __builtin_amdgcn_raw_buffer_store_b64(w, r, voff, soff, 0);
}

}  // namespace dev
}  // namespace crlot
