// stft.hip -- the round trip split at its spectral step (the
// reference marks the processing point at bench/e2e_benchmark.cc:160-162), so
// any device-side spectral processing -- a mask, a Wiener gain, a model -- can
// sit between the two halves, plus the round trip with a per-frame mask.
//
// K_stft   k_stft<E>: x -> spectra.  Framing (Framer ZERO_PAD / DROP, or the
//          FrameQueue's centre padding and pad modes), analysis window (frame * w,
//          e2e_benchmark.cc:154-156), sanitize and kiss_fftr
//          (IFftPlan::forward, kissfft_adapter.cc:83-122): spectrum k of stream s,
//          N/2+1 bins, written to HBM.  The arithmetic is k_rfft's, so the bits
//          equal crlot_rfft_batched on the windowed frames.  A wave walks a run of
//          consecutive frames of one stream with the twiddles and super-twiddles
//          staged once per workgroup; the next frame is loaded while the current
//          one transforms.
// K_istft  k_istft<E,S,XIN>: spectra -> the plan's spectral step (per-bin real gain,
//          then the per-frame mask) -> kiss_fftri merge, inverse FFT, *1/N and
//          sanitize (IFftPlan::inverse, kissfft_adapter.cc:124-168), synthesis
//          window and ascending-k overlap-add (push_frame_AoS, OLAAccumulator.cc
//          :124-160, kernels.cc:24-28), / max(norm, eps) per H-sample block
//          (produce, OLAAccumulator.cc:162-221).  A wave walks a run of
//          consecutive frames of one stream (NB-1 warm-up frames recomputed),
//          the open OLA blocks in registers, as K_fused does; the 1/N fold and
//          Markstein's division are K_fused's exact rewrites, so the output
//          equals crlot_irfft_batched + crlot_ola_gather bit for bit.  XIN: the
//          input is x itself, transformed first with K_stft's arithmetic -- the
//          round trip with a per-frame mask in one pass over HBM, bit-identical to
//          K_istft(K_stft(x)).
// k_frames_w / k_spec_step: the staged forms (any hop, any frame size, any row
//          alignment) through a workspace: windowed frames for the mixed-radix
//          rfft, and the spectral step over spectra in HBM.
#include <algorithm>
#include <cstdint>

#include "fft_wave.h"
#include "fused_common.h"
#include "kernels.h"

namespace crlot {

using dev::cf;

namespace {

using namespace fk;

constexpr int kW = 4;  // waves per workgroup, each walking its own frames

struct StftArgs {
    DevTables t;
    const float* x;        // K_stft / XIN input: stream s at x + s ld_x
    const float* sin;      // K_istft input spectra: (s, k) at sin + s ld_spec + k ld_frame
    float* spec;           // K_stft output spectra, same layout
    float* y;              // stream s at y + s ld_y, F H samples
    SpecMask mask;
    int64_t ld_x, T, ld_spec, ld_frame, ld_y;
    int n_streams, F, n_chunks, M, ring_blocks, h, pad, pad_mode;
    float gain;            // push_frame_AoS gain
};

// x[j] of a T-sample stream with the plan's padding outside [0, T)
// (Indexing.h:18-68 via FrameQueue; zeros for the Framer): 0 zeros, 1 reflect101, 2 edge.
__device__ __forceinline__ float xat(const float* xs, int64_t j, int64_t T, int mode) {
    if (mode == 1) {
        if (T <= 1) {
            j = 0;
        } else {
            while (j < 0 || j >= T) j = j < 0 ? -j - 1 : 2 * T - 2 - j;
        }
    } else if (mode == 2) {
        j = j < 0 ? 0 : (j >= T ? T - 1 : j);
    }
    return (j >= 0 && j < T) ? xs[j] : 0.0f;
}

// Raw samples of registers m in [M0, M0 + CNT) of the frame at origin o:
// r[m] = (x[o + 2i], x[o + 2i + 1]), i = lane + 64 m.  A part wholly inside the
// stream takes one 8-byte load per lane and register when the address is
// 8-byte aligned (wave-uniform), else two 4-byte loads; parts crossing an edge
// map every sample through the padding rule.
template <int M0, int CNT, int E>
__device__ __forceinline__ void load_part(float2 (&r)[E], const float* xs, int64_t o, int64_t T, int mode,
                                          int lane) {
    const int64_t lo = o + 128 * M0, hi = o + 128 * (M0 + CNT);
    if (lo >= 0 && hi <= T) {
        const float* p = xs + o;
        if ((reinterpret_cast<uintptr_t>(p) & 7u) == 0) {
#pragma unroll
            for (int m = M0; m < M0 + CNT; ++m) r[m] = reinterpret_cast<const float2*>(p)[lane + 64 * m];
        } else {
#pragma unroll
            for (int m = M0; m < M0 + CNT; ++m) {
                const int i = 2 * (lane + 64 * m);
                r[m] = make_float2(p[i], p[i + 1]);
            }
        }
    } else {
#pragma unroll
        for (int m = M0; m < M0 + CNT; ++m) {
            const int64_t j = o + 2 * (lane + 64 * m);
            r[m] = make_float2(xat(xs, j, T, mode), xat(xs, j + 1, T, mode));
        }
    }
}

// kiss_fftr's split of one bin (k_rfft's arithmetic): X[b] from Z[b] and Z[P-b]
// with sth = st[b] / 2 (exact).
__device__ __forceinline__ cf split_bin(cf zk, cf zpk, cf sth) {
    const cf fpnk = dev::conj(zpk);
    const cf f1 = dev::cadd(zk, fpnk);
    const cf f2 = dev::csub(zk, fpnk);
    const cf t = dev::cmul(f2, sth);
    return {__builtin_fmaf(f1.r, 0.5f, t.r), __builtin_fmaf(f1.i, 0.5f, t.i)};
}

// kiss_fftri's merge (k_irfft's arithmetic): Z'[b] from X[b], X[P-b] and st[b].
__device__ __forceinline__ cf merge_bin(cf xk, cf xpk, cf w) {
    const cf fek = {xk.r + xpk.r, xk.i - xpk.i};
    const cf tmp = {xk.r - xpk.r, xk.i + xpk.i};
    return {__builtin_fmaf(tmp.r, w.r, __builtin_fmaf(tmp.i, w.i, fek.r)),
            __builtin_fmaf(tmp.i, w.r, __builtin_fmaf(-tmp.r, w.i, fek.i))};
}

__device__ __forceinline__ cf scale(cf v, float g) { return {v.r * g, v.i * g}; }

template <int E>
struct Cfg {
    static constexpr int P = 64 * E, N = 2 * P;
    static constexpr int TW = dev::twiddle_table_size(E);
    // N <= 2048: super-twiddles and windows staged in LDS (and the analysis window
    // of K_stft in registers); N = 4096 reads them from L2, so the LDS holds only
    // the twiddles and the four exchange buffers
    static constexpr bool TL = E <= 16;
    static constexpr bool WREG = E <= 8;  // K_stft: the analysis window in registers
};

// ------------------------------------------------------------------ K_stft
template <int E>
struct StftOcc {
    static constexpr int value = E <= 2 ? 8 : E <= 4 ? 6 : E <= 8 ? 4 : E <= 16 ? 3 : 2;
};

template <int E>
__global__ __launch_bounds__(64 * kW, StftOcc<E>::value) void k_stft(const StftArgs a) {
    using C = Cfg<E>;
    constexpr int P = C::P;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    cf* sth = tw + C::TW;                       // [P] when TL
    cf* bufs = sth + (C::TL ? P : 0);
    const cf* gst = reinterpret_cast<const cf*>(a.t.st);
    {
        const cf* gtw = reinterpret_cast<const cf*>(a.t.tw);
        for (int i = threadIdx.x; i < C::TW; i += 64 * kW) tw[i] = gtw[i];
        if constexpr (C::TL) {
            for (int i = threadIdx.x; i < P; i += 64 * kW) {
                const cf w = gst[i];
                sth[i] = cf{w.r * 0.5f, w.i * 0.5f};  // exact
            }
        }
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    cf* buf = bufs + wave * P;
    const int gw = blockIdx.x * kW + wave;
    if (gw >= a.n_streams * a.n_chunks) return;
    const int s = gw / a.n_chunks, c = gw - s * a.n_chunks;
    const int k0 = c * a.M, k1 = min(a.F, k0 + a.M);
    const float* xs = a.x + int64_t(s) * a.ld_x;
    float* so = a.spec + int64_t(s) * a.ld_spec;
    const float2* wa2 = reinterpret_cast<const float2*>(a.t.wa);
    float2 wr[C::WREG ? E : 1];
    if constexpr (C::WREG) {
#pragma unroll
        for (int m = 0; m < E; ++m) wr[m] = wa2[lane + 64 * m];
    }
    float2 xr[E];
    load_part<0, E, E>(xr, xs, int64_t(k0) * a.h - a.pad, a.T, a.pad_mode, lane);
    for (int k = k0; k < k1; ++k) {
        cf v[E];
#pragma unroll
        for (int m = 0; m < E; ++m) {
            float2 w;
            if constexpr (C::WREG) w = wr[m];
            else w = wa2[lane + 64 * m];
            v[m].r = dev::sanit(xr[m].x * w.x);  // harness frame[i] * w[i], then the adapter's sanitize
            v[m].i = dev::sanit(xr[m].y * w.y);
        }
        if (k + 1 < k1) load_part<0, E, E>(xr, xs, int64_t(k + 1) * a.h - a.pad, a.T, a.pad_mode, lane);
        dev::fft_wave<E, false>(v, buf, tw, lane);
#pragma unroll
        for (int m = 0; m < E; ++m) buf[lane + 64 * m] = v[m];
        dev::wave_lds_fence();
        float2* out = reinterpret_cast<float2*>(so + int64_t(k) * a.ld_frame);
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int b = lane + 64 * m;
            cf h;
            if constexpr (C::TL) h = sth[b];
            else h = cf{gst[b].r * 0.5f, gst[b].i * 0.5f};
            cf xk = split_bin(v[m], buf[(P - b) & (P - 1)], h), xp;
            if (b == 0) dev::dc_split(v[m], xk, xp);
            out[b] = make_float2(xk.r, xk.i);
            if (b == 0) out[P] = make_float2(xp.r, xp.i);
        }
        dev::wave_lds_fence();
    }
}

// ------------------------------------------------------------------ K_istft
// Waves per SIMD the walkers are compiled for (registers: 512 / waves per lane).
template <int E, bool XIN>
struct IstftOcc {
    static constexpr int value = E <= 2 ? 6 : E <= 4 ? 5 : E <= 8 ? 3 : 2;
};

// Per-wave LDS of K_istft: the spectrum of the frame (P + 2 float pairs, X[0..P];
// the inverse FFT's exchange buffer once the merge has read it) and its mask row
// (P + 2 floats).
template <int E>
constexpr int istft_wave_floats() {
    return 2 * (64 * E + 2) + (64 * E + 2);
}

template <int E, int S, bool XIN>
__global__ __launch_bounds__(64 * kW, (IstftOcc<E, XIN>::value)) void k_istft(const StftArgs a) {
    using C = Cfg<E>;
    constexpr int P = C::P, N = C::N, H = 128 * S, NB = E / S;
    static_assert(NB * S == E, "N = NB * H");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    cf* st = tw + C::TW;                                          // [P] when TL
    float* wsn = reinterpret_cast<float*>(st + (C::TL ? P : 0));  // [N] when TL
    float* wa = wsn + (C::TL ? N : 0);                            // [N] when TL and XIN
    float* gl = wa + (C::TL && XIN ? N : 0);                      // [P + 2] when TL (gain)
    float* wbase = gl + (C::TL ? P + 2 : 0);                      // per wave: istft_wave_floats
    const cf* gst = reinterpret_cast<const cf*>(a.t.st);
    const bool has_gain = a.t.gain != nullptr;
    {
        const cf* gtw = reinterpret_cast<const cf*>(a.t.tw);
        for (int i = threadIdx.x; i < C::TW; i += 64 * kW) tw[i] = gtw[i];
        if constexpr (C::TL) {
            for (int i = threadIdx.x; i < P; i += 64 * kW) st[i] = gst[i];
            for (int i = threadIdx.x; i < N; i += 64 * kW) {
                wsn[i] = a.t.wsn[i];
                if constexpr (XIN) wa[i] = a.t.wa[i];
            }
            // the gain table (ones without a gain: x * 1 == x, so the step is branch-free)
            for (int i = threadIdx.x; i <= P; i += 64 * kW) gl[i] = has_gain ? a.t.gain[i] : 1.0f;
        }
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    cf* buf = reinterpret_cast<cf*>(wbase + wave * istft_wave_floats<E>());  // [P + 2]: spectrum / FFT exchange
    float* mb = reinterpret_cast<float*>(buf + P + 2);                       // [P + 2]: mask row
    const int gw = blockIdx.x * kW + wave;
    if (gw >= a.n_streams * a.n_chunks) return;
    if constexpr (C::TL) {
        if (!a.mask.p) {  // no mask: a row of ones, set once (the step stays branch-free)
#pragma unroll
            for (int m = 0; m < E; ++m) mb[lane + 64 * m] = 1.0f;
            if (lane == 0) mb[P] = 1.0f;
        }
    }
    const int s = gw / a.n_chunks, c = gw - s * a.n_chunks;
    const int f0 = c * a.M;
    const int f1 = min(a.F, f0 + a.M);
    const int fs = max(0, f0 - (NB - 1));
    const float* xs = XIN ? a.x + int64_t(s) * a.ld_x : nullptr;
    const float* ss = XIN ? nullptr : a.sin + int64_t(s) * a.ld_spec;
    float* ys = a.y + int64_t(s) * a.ld_y;
    const float* gain = C::TL ? gl : a.t.gain;
    const float* mbase = a.mask.p ? a.mask.p + int64_t(s) * a.mask.ld_stream : nullptr;
    const float g = a.gain;
    const float2* wa2 = reinterpret_cast<const float2*>(XIN && C::TL ? wa : a.t.wa);
    const float2* ws2 = reinterpret_cast<const float2*>(C::TL ? wsn : a.t.wsn);

    // frame k's spectrum row X[0..P] (lane l: X[l + 64 m], lane 0 also X[P]) and mask
    // row, into registers: issued one step ahead, stored to the wave's LDS when used
    float2 ps[XIN ? 1 : E], pP = make_float2(0.f, 0.f);
    float pm[E], pmP = 0.f;
    auto load_rows = [&](int k) {
        if constexpr (!XIN) {
            const float2* row = reinterpret_cast<const float2*>(ss + int64_t(k) * a.ld_frame);
#pragma unroll
            for (int m = 0; m < E; ++m) ps[m] = row[lane + 64 * m];
            if (lane == 0) pP = row[P];
        }
        if (mbase) {
            const float* mr = mbase + int64_t(k) * a.mask.ld_frame;
#pragma unroll
            for (int m = 0; m < E; ++m) pm[m] = mr[lane + 64 * m];
            if (lane == 0) pmP = mr[P];
        }
    };

    float2 acc[NB][S];
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int q = 0; q < S; ++q) acc[j][q] = make_float2(0.f, 0.f);
    float2 xin[XIN ? E : 1];
    if constexpr (XIN) {
        load_part<0, E, E>(xin, xs, int64_t(fs) * H - a.pad, a.T, a.pad_mode, lane);
    } else {
        load_rows(fs);
    }

    for (int k = fs; k < f1; ++k) {
        // prefetch: frame k+1's new hop (XIN) and block k's divisors, consumed at the
        // end of this iteration, so their latency hides under the transforms
        float2 nxt[XIN ? E : 1];
        if constexpr (XIN) {
            if (k + 1 < f1) load_part<E - S, S, E>(nxt, xs, int64_t(k + 1) * H - a.pad, a.T, a.pad_mode, lane);
            load_rows(k);  // the mask row: lands during the forward transform
        }
        float2 dn[S], rn[S];
        if (k >= f0) {
            const float2* d2 = reinterpret_cast<const float2*>(a.t.den + (k % a.ring_blocks) * H);
            const float2* r2 = reinterpret_cast<const float2*>(a.t.rden + (k % a.ring_blocks) * H);
#pragma unroll
            for (int q = 0; q < S; ++q) {
                dn[q] = d2[lane + 64 * q];
                rn[q] = r2[lane + 64 * q];
            }
        }
        cf v[E];
        if constexpr (XIN) {
#pragma unroll
            for (int m = 0; m < E; ++m) {
                const float2 w = wa2[lane + 64 * m];
                v[m].r = dev::sanit(xin[m].x * w.x);
                v[m].i = dev::sanit(xin[m].y * w.y);
            }
            dev::fft_wave<E, false>(v, buf, tw, lane);
#pragma unroll
            for (int m = 0; m < E; ++m) buf[lane + 64 * m] = v[m];
        } else {
#pragma unroll
            for (int m = 0; m < E; ++m) buf[lane + 64 * m] = cf{ps[m].x, ps[m].y};
            if (lane == 0) buf[P] = cf{pP.x, pP.y};
        }
        if (mbase) {
#pragma unroll
            for (int m = 0; m < E; ++m) mb[lane + 64 * m] = pm[m];
            if (lane == 0) mb[P] = pmP;
        }
        dev::wave_lds_fence();
        if constexpr (!XIN) {
            if (k + 1 < f1) load_rows(k + 1);  // in flight during this frame's inverse
        }
        // per bin b = lane + 64 m: X[b] and X[P-b] (from the spectrum, or -- XIN -- as
        // k_rfft's lanes b and P-b compute them from Z), the spectral step (the plan's
        // gain, then row k of the mask), then kiss_fftri's merge into Z'[b]
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int b = lane + 64 * m;
            cf xk, xp;
            if constexpr (XIN) {
                const cf zp = buf[(P - b) & (P - 1)];
                cf h0, h1;
                if constexpr (C::TL) {
                    h0 = st[b];
                    h1 = st[(P - b) & (P - 1)];
                } else {
                    h0 = gst[b];
                    h1 = gst[(P - b) & (P - 1)];
                }
                xk = split_bin(v[m], zp, cf{h0.r * 0.5f, h0.i * 0.5f});
                xp = split_bin(zp, v[m], cf{h1.r * 0.5f, h1.i * 0.5f});
                if (b == 0) dev::dc_split(v[m], xk, xp);
            } else {
                xk = buf[b];
                xp = buf[P - b];  // (b = 0: X[P])
            }
            if (C::TL || has_gain) {
                xk = scale(xk, gain[b]);
                xp = scale(xp, gain[P - b]);
            }
            if (C::TL || mbase) {
                xk = scale(xk, mb[b]);
                xp = scale(xp, mb[P - b]);
            }
            cf w;
            if constexpr (C::TL) w = st[b];
            else w = gst[b];
            v[m] = b == 0 ? dev::dc_merge(xk, xp) : merge_bin(xk, xp, w);
        }
        dev::wave_lds_fence();
        dev::fft_wave<E, true>(v, buf, tw, lane);
        // *1/N and sanitize (folded: sanit_scaled, ws / N), synthesis window, OLA in ascending k
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const float2 w = ws2[lane + 64 * m];
            const float o0 = dev::sanit_scaled<N>(v[m].r);
            const float o1 = dev::sanit_scaled<N>(v[m].i);
            float2& r = acc[m / S][m % S];
            r.x = __builtin_fmaf(__builtin_fmaf(o0, w.x, 0.0f), g, r.x);
            r.y = __builtin_fmaf(__builtin_fmaf(o1, w.y, 0.0f), g, r.y);
        }
        // block k is complete: produce(H) = acc / max(norm, eps)
        if (k >= f0) {
            float2* yo = reinterpret_cast<float2*>(ys + int64_t(k) * H);
            bool ok = true;
#pragma unroll
            for (int q = 0; q < S; ++q) ok = ok && mk_ok(acc[0][q].x) && mk_ok(acc[0][q].y);
            if (__builtin_amdgcn_ballot_w64(!ok) == 0) {
#pragma unroll
                for (int q = 0; q < S; ++q)
                    yo[lane + 64 * q] = make_float2(mk_div(acc[0][q].x, dn[q].x, rn[q].x),
                                                    mk_div(acc[0][q].y, dn[q].y, rn[q].y));
            } else {
#pragma unroll
                for (int q = 0; q < S; ++q)
                    yo[lane + 64 * q] = make_float2(acc[0][q].x / dn[q].x, acc[0][q].y / dn[q].y);
            }
        }
#pragma unroll
        for (int j = 0; j < NB - 1; ++j)
#pragma unroll
            for (int q = 0; q < S; ++q) acc[j][q] = acc[j + 1][q];
#pragma unroll
        for (int q = 0; q < S; ++q) acc[NB - 1][q] = make_float2(0.f, 0.f);
        if constexpr (XIN) {
#pragma unroll
            for (int m = 0; m < E - S; ++m) xin[m] = xin[m + S];
#pragma unroll
            for (int m = E - S; m < E; ++m) xin[m] = nxt[m];
        }
        dev::wave_lds_fence();  // (the next frame's stores to buf follow this one's reads)
    }
}

// ------------------------------------------------------------------ workgroup walkers (N = 2048, 4096)
// One frame on a workgroup of L lanes, E = 8 complex points per lane (lane t
// holds z[t + L m]), so registers stay at the per-wave E = 8 budget.  The
// Stockham passes are the per-wave schedule's (radix 8, 8, 8, 4 at P = 2048;
// 8, 8, 4, ... identical radices and twiddle indices), exchanged through two LDS
// buffers with one barrier each (fft_wave.h stockham_exchange_wg), so the bits
// equal the per-wave kernels' (k_rfft / k_irfft) -- crlot_rfft_batched and
// crlot_irfft_batched + crlot_ola_gather stay the checks.  Twiddles and
// super-twiddles are staged in LDS (the walks are memory-bound: registers go to
// the frames in flight).
template <int E, int L, int NS, int XI, int TOFF, bool INV, typename TW>
__device__ __forceinline__ void fft_passes_wg_t(cf (&v)[E], cf* buf0, cf* buf1, const cf* twp, int t,
                                                const TW& tw) {
    constexpr int P = L * E;
    if constexpr (NS < P) {
        constexpr int R = dev::radix_for(P / NS, E);
        dev::stockham_compute<E, R, NS, INV>(v, tw);
        if constexpr (NS * R < P) {
            constexpr int NS2 = NS * R;
            constexpr int R2 = dev::radix_for(P / NS2, E);
            constexpr int TOFF2 = TOFF + (NS > 1 ? (R - 1) * NS : 0);
            dev::PassTw<E, R2, NS2> tw2;
            dev::load_pass_tw_wg<E, R2, NS2, L, TOFF2>(tw2, twp, t);
            dev::stockham_exchange_wg<E, R, NS, L>(v, (XI & 1) ? buf1 : buf0, t);
            fft_passes_wg_t<E, L, NS2, XI + 1, TOFF2, INV>(v, buf0, buf1, twp, t, tw2);
        }
    }
}
template <int L, bool INV>
__device__ __forceinline__ void fft_wg(cf (&v)[8], cf* buf0, cf* buf1, const cf* twp, int t) {
    constexpr int E = 8, R = dev::radix_for(L * E, E);
    dev::PassTw<E, R, 1> none;
    fft_passes_wg_t<E, L, 1, 0, 0, INV>(v, buf0, buf1, twp, t, none);
}
template <int L>
struct WgCfg {
    static constexpr int E = 8, P = L * E, N = 2 * P;
    static constexpr int TW = dev::twiddle_table_size(P / 64);  // (the per-wave table of this P)
};

// frame part at origin o for the workgroup layout: r[m] = (x[o + 2i], x[o + 2i + 1]), i = t + L m
template <int M0, int CNT, int L>
__device__ __forceinline__ void load_part_wg(float2 (&r)[8], const float* xs, int64_t o, int64_t T, int mode,
                                             int t) {
    const int64_t lo = o + 2 * L * M0, hi = o + 2 * L * (M0 + CNT);
    if (lo >= 0 && hi <= T) {
        const float* p = xs + o;
        if ((reinterpret_cast<uintptr_t>(p) & 7u) == 0) {
#pragma unroll
            for (int m = M0; m < M0 + CNT; ++m) r[m] = reinterpret_cast<const float2*>(p)[t + L * m];
        } else {
#pragma unroll
            for (int m = M0; m < M0 + CNT; ++m) {
                const int i = 2 * (t + L * m);
                r[m] = make_float2(p[i], p[i + 1]);
            }
        }
    } else {
#pragma unroll
        for (int m = M0; m < M0 + CNT; ++m) {
            const int64_t j = o + 2 * (t + L * m);
            r[m] = make_float2(xat(xs, j, T, mode), xat(xs, j + 1, T, mode));
        }
    }
}

// K_stft on a workgroup: blockIdx = (stream, chunk), frames k0 .. k1-1 in order.
template <int L>
__global__ __launch_bounds__(L) void k_stft_wg(const StftArgs a) {
    using C = WgCfg<L>;
    constexpr int E = 8, P = C::P;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    cf* bufA = tw + C::TW;
    cf* bufB = bufA + P;
    const int t = threadIdx.x;
    for (int i = t; i < C::TW; i += L) tw[i] = reinterpret_cast<const cf*>(a.t.tw)[i];
    const int s = blockIdx.x / a.n_chunks, c = blockIdx.x - s * a.n_chunks;
    const int k0 = c * a.M, k1 = min(a.F, k0 + a.M);
    const float* xs = a.x + int64_t(s) * a.ld_x;
    float* so = a.spec + int64_t(s) * a.ld_spec;
    const cf* gst = reinterpret_cast<const cf*>(a.t.st);
    float2 wa[E];
    cf sth[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        wa[m] = reinterpret_cast<const float2*>(a.t.wa)[t + L * m];
        const cf w = gst[t + L * m];
        sth[m] = cf{w.r * 0.5f, w.i * 0.5f};
    }
    float2 xr[E];
    load_part_wg<0, E, L>(xr, xs, int64_t(k0) * a.h - a.pad, a.T, a.pad_mode, t);
    __syncthreads();
    for (int k = k0; k < k1; ++k) {
        cf v[E];
#pragma unroll
        for (int m = 0; m < E; ++m) {
            v[m].r = dev::sanit(xr[m].x * wa[m].x);
            v[m].i = dev::sanit(xr[m].y * wa[m].y);
        }
        if (k + 1 < k1) load_part_wg<0, E, L>(xr, xs, int64_t(k + 1) * a.h - a.pad, a.T, a.pad_mode, t);
        // (exchanges A B A, then the split partner through B: 4 per frame, so the
        // alternation holds across frames)
        static_assert(dev::fft_exchanges(P, E) == 3, "buffer alternation");
        fft_wg<L, false>(v, bufA, bufB, tw, t);
        cf* bx = bufB;
#pragma unroll
        for (int m = 0; m < E; ++m) bx[t + L * m] = v[m];
        __syncthreads();
        float2* out = reinterpret_cast<float2*>(so + int64_t(k) * a.ld_frame);
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int b = t + L * m;
            cf xk = split_bin(v[m], bx[(P - b) & (P - 1)], sth[m]), xp;
            if (b == 0) dev::dc_split(v[m], xk, xp);
            out[b] = make_float2(xk.r, xk.i);
            if (b == 0) out[P] = make_float2(xp.r, xp.i);
        }
    }
}

// K_istft on a workgroup (XIN: from x, the masked round trip).  The spectral
// step is applied to each lane's own bins as the spectrum is staged in LDS
// (X'[b] = X[b] * gain[b] * mask[b]), so the merge reads X'[b] and X'[P-b] with
// no per-bin tables in LDS.  XIN computes its own bins' X[b] first, exactly as
// K_stft's lane b does (split of Z[b], Z[P-b] through one exchange), then
// stages X'[b].  LDS: the twiddles and the two exchange buffers.
template <int L, int S, bool XIN>
__global__ __launch_bounds__(L) void k_istft_wg(const StftArgs a) {
    using C = WgCfg<L>;
    constexpr int E = 8, P = C::P, N = C::N, H = 2 * L * S, NB = E / S;
    static_assert(NB * S == E, "N = NB * H");
    // exchanges per frame: XIN forward A B A, Z partner B, staging A, inverse B A B;
    // else staging B, inverse A B A -- consecutive exchanges alternate buffers
    // within and across frames (a buffer is rewritten only behind the barrier of
    // the exchange that followed its last reads)
    static_assert(dev::fft_exchanges(P, E) == 3, "buffer alternation");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    cf* bufA = tw + C::TW;     // [P + 2]
    cf* bufB = bufA + P + 2;   // [P + 2]
    const int t = threadIdx.x;
    for (int i = t; i < C::TW; i += L) tw[i] = reinterpret_cast<const cf*>(a.t.tw)[i];
    const int s = blockIdx.x / a.n_chunks, c = blockIdx.x - s * a.n_chunks;
    const int f0 = c * a.M;
    const int f1 = min(a.F, f0 + a.M);
    const int fs = max(0, f0 - (NB - 1));
    const float* xs = XIN ? a.x + int64_t(s) * a.ld_x : nullptr;
    const float* ss = XIN ? nullptr : a.sin + int64_t(s) * a.ld_spec;
    float* ys = a.y + int64_t(s) * a.ld_y;
    const float* mbase = a.mask.p ? a.mask.p + int64_t(s) * a.mask.ld_stream : nullptr;
    const float g = a.gain;
    const cf* gst = reinterpret_cast<const cf*>(a.t.st);
    // this lane's bins b = t + L m: super-twiddle, gain (1 without one), windows
    float2 wsn[E], wa[XIN ? E : 1];
    cf st[E];
    float gb[E], gP = 1.0f;
#pragma unroll
    for (int m = 0; m < E; ++m) {
        wsn[m] = reinterpret_cast<const float2*>(a.t.wsn)[t + L * m];
        if constexpr (XIN) wa[m] = reinterpret_cast<const float2*>(a.t.wa)[t + L * m];
        st[m] = gst[t + L * m];
        gb[m] = a.t.gain ? a.t.gain[t + L * m] : 1.0f;
    }
    if (t == 0 && a.t.gain) gP = a.t.gain[P];
    // frame k's spectrum and mask rows, this lane's bins (issued one frame ahead)
    float2 ps[XIN ? 1 : E], pP = make_float2(0.f, 0.f);
    float pm[E], pmP = 1.0f;
#pragma unroll
    for (int m = 0; m < E; ++m) pm[m] = 1.0f;
    auto load_rows = [&](int k) {
        if constexpr (!XIN) {
            const float2* row = reinterpret_cast<const float2*>(ss + int64_t(k) * a.ld_frame);
#pragma unroll
            for (int m = 0; m < E; ++m) ps[m] = row[t + L * m];
            if (t == 0) pP = row[P];
        }
        if (mbase) {
            const float* mr = mbase + int64_t(k) * a.mask.ld_frame;
#pragma unroll
            for (int m = 0; m < E; ++m) pm[m] = mr[t + L * m];
            if (t == 0) pmP = mr[P];
        }
    };
    float2 acc[NB][S];
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int q = 0; q < S; ++q) acc[j][q] = make_float2(0.f, 0.f);
    float2 xin[E];
    if constexpr (XIN) load_part_wg<0, E, L>(xin, xs, int64_t(fs) * H - a.pad, a.T, a.pad_mode, t);
    load_rows(fs);
    __syncthreads();

    for (int k = fs; k < f1; ++k) {
        float2 nxt[E];
        if constexpr (XIN) {
            if (k + 1 < f1) load_part_wg<E - S, S, L>(nxt, xs, int64_t(k + 1) * H - a.pad, a.T, a.pad_mode, t);
        }
        float2 dn[S], rn[S];
        if (k >= f0) {
            const float2* d2 = reinterpret_cast<const float2*>(a.t.den + (k % a.ring_blocks) * H);
            const float2* r2 = reinterpret_cast<const float2*>(a.t.rden + (k % a.ring_blocks) * H);
#pragma unroll
            for (int q = 0; q < S; ++q) {
                dn[q] = d2[t + L * q];
                rn[q] = r2[t + L * q];
            }
        }
        // this lane's X[b] (and lane 0's X[P])
        cf xk[E], xP = cf{0.f, 0.f};
        if constexpr (XIN) {
            cf v[E];
#pragma unroll
            for (int m = 0; m < E; ++m) {
                v[m].r = dev::sanit(xin[m].x * wa[m].x);
                v[m].i = dev::sanit(xin[m].y * wa[m].y);
            }
            fft_wg<L, false>(v, bufA, bufB, tw, t);
#pragma unroll
            for (int m = 0; m < E; ++m) bufB[t + L * m] = v[m];
            __syncthreads();
#pragma unroll
            for (int m = 0; m < E; ++m) {
                const int b = t + L * m;
                xk[m] = split_bin(v[m], bufB[(P - b) & (P - 1)], cf{st[m].r * 0.5f, st[m].i * 0.5f});
                if (b == 0) dev::dc_split(v[m], xk[m], xP);
            }
        } else {
#pragma unroll
            for (int m = 0; m < E; ++m) xk[m] = cf{ps[m].x, ps[m].y};
            xP = cf{pP.x, pP.y};
        }
        // the spectral step on this lane's bins, staged for the merge
        cf* bx = XIN ? bufA : bufB;
#pragma unroll
        for (int m = 0; m < E; ++m) bx[t + L * m] = scale(scale(xk[m], gb[m]), pm[m]);
        if (t == 0) bx[P] = scale(scale(xP, gP), pmP);
        __syncthreads();
        if (k + 1 < f1) load_rows(k + 1);  // in flight during the merge and the inverse
        cf v[E];
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int b = t + L * m;
            const cf x0 = bx[b], x1 = bx[P - b];  // (b = 0: X'[P])
            v[m] = b == 0 ? dev::dc_merge(x0, x1) : merge_bin(x0, x1, st[m]);
        }
        if constexpr (XIN) fft_wg<L, true>(v, bufB, bufA, tw, t);
        else fft_wg<L, true>(v, bufA, bufB, tw, t);
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const float o0 = dev::sanit_scaled<N>(v[m].r);
            const float o1 = dev::sanit_scaled<N>(v[m].i);
            float2& r = acc[m / S][m % S];
            r.x = __builtin_fmaf(__builtin_fmaf(o0, wsn[m].x, 0.0f), g, r.x);
            r.y = __builtin_fmaf(__builtin_fmaf(o1, wsn[m].y, 0.0f), g, r.y);
        }
        if (k >= f0) {
            float2* yo = reinterpret_cast<float2*>(ys + int64_t(k) * H);
            bool ok = true;
#pragma unroll
            for (int q = 0; q < S; ++q) ok = ok && mk_ok(acc[0][q].x) && mk_ok(acc[0][q].y);
            // (a per-wave choice: both divisions give the same bits where Markstein's is valid)
            if (__builtin_amdgcn_ballot_w64(!ok) == 0) {
#pragma unroll
                for (int q = 0; q < S; ++q)
                    yo[t + L * q] = make_float2(mk_div(acc[0][q].x, dn[q].x, rn[q].x),
                                                mk_div(acc[0][q].y, dn[q].y, rn[q].y));
            } else {
#pragma unroll
                for (int q = 0; q < S; ++q)
                    yo[t + L * q] = make_float2(acc[0][q].x / dn[q].x, acc[0][q].y / dn[q].y);
            }
        }
#pragma unroll
        for (int j = 0; j < NB - 1; ++j)
#pragma unroll
            for (int q = 0; q < S; ++q) acc[j][q] = acc[j + 1][q];
#pragma unroll
        for (int q = 0; q < S; ++q) acc[NB - 1][q] = make_float2(0.f, 0.f);
        if constexpr (XIN) {
#pragma unroll
            for (int m = 0; m < E - S; ++m) xin[m] = xin[m + S];
#pragma unroll
            for (int m = E - S; m < E; ++m) xin[m] = nxt[m];
        }
    }
}

// ------------------------------------------------------------------ staged forms
// frames[r][i] = x[k H - pad + i] * wa[i] (padding rule outside [0, T)), r = s F + k:
// the analysis products of every frame, for the mixed-radix rfft (which sanitizes).
__global__ __launch_bounds__(256) void k_frames_w(const float* __restrict__ x, int64_t ld_x, int64_t T,
                                                  const float* __restrict__ wa, float* __restrict__ frames,
                                                  int64_t F, int n, int h, int pad, int mode) {
    const int64_t r = blockIdx.x;
    const int64_t s = r / F, k = r - s * F;
    const float* xs = x + s * ld_x;
    const int64_t o = k * h - pad;
    float* fr = frames + r * n;
    for (int i = threadIdx.x; i < n; i += 256) fr[i] = xat(xs, o + i, T, mode) * wa[i];
}

// out row r = s F + k (2 bins floats apart) = spectrum (s, k) * gain * mask row (s, k);
// in place when out is the input with that layout.
__global__ __launch_bounds__(256) void k_spec_step(const float* in, int64_t ld_spec, int64_t ld_frame, float* out,
                                                   int64_t F, int bins, const float* gain, SpecMask mask) {
    const int64_t r = blockIdx.x;
    const int64_t s = r / F, k = r - s * F;
    const float2* src = reinterpret_cast<const float2*>(in + s * ld_spec + k * ld_frame);
    float2* dst = reinterpret_cast<float2*>(out + r * 2 * bins);
    const float* mr = mask.p ? mask.p + s * mask.ld_stream + k * mask.ld_frame : nullptr;
    for (int b = threadIdx.x; b < bins; b += 256) {
        cf v = {src[b].x, src[b].y};
        if (gain) v = scale(v, gain[b]);
        if (mr) v = scale(v, mr[b]);
        dst[b] = make_float2(v.r, v.i);
    }
}

int e_of_n(int n) {
    switch (n) {
        case 256: return 2;
        case 512: return 4;
        case 1024: return 8;
        case 2048: return 16;
        case 4096: return 32;
        default: return 0;
    }
}

template <int E>
size_t stft_lds() {
    using C = Cfg<E>;
    return sizeof(cf) * (C::TW + (C::TL ? C::P : 0) + kW * C::P);
}
template <int E, bool XIN>
size_t istft_lds() {
    using C = Cfg<E>;
    return sizeof(cf) * (C::TW + (C::TL ? C::P : 0)) +
           sizeof(float) * ((C::TL ? (XIN ? 2 : 1) * C::N + C::P + 2 : 0) + kW * istft_wave_floats<E>());
}
template <int L>
size_t stft_wg_lds() {
    return sizeof(cf) * (WgCfg<L>::TW + 2 * WgCfg<L>::P);
}
template <int L>
size_t istft_wg_lds() {
    return sizeof(cf) * (WgCfg<L>::TW + 2 * (WgCfg<L>::P + 2));
}

int cus() {
    static const int v = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        return n;
    }();
    return v;
}

// Chunks per stream: enough walkers for two resident rounds of the device
// (`resident` walkers at once), chunks of about 128 frames while the grid stays
// that deep, at least `min_m` frames each (the istft walk recomputes NB-1
// warm-up frames per chunk); the plan's chunk knob overrides.
void pick_chunks(int64_t F, int n_streams, int64_t resident, int min_m, int& n_chunks, int& m) {
    const int64_t S = std::max(1, n_streams);
    int64_t n = (F + 127) / 128;
    n = std::max<int64_t>(n, (2 * std::max<int64_t>(1, resident) + S - 1) / S);
    n = std::min<int64_t>(n, std::max<int64_t>(1, F / std::max(1, min_m)));
    if (const int64_t c = chunks_or(0, F); c > 0) n = c;
    n = std::max<int64_t>(1, std::min<int64_t>(n, F));
    m = int((F + n - 1) / n);
    n_chunks = int((F + m - 1) / m);
}

// walkers the device holds at once: workgroups per CU x walkers per workgroup x CUs
template <typename K>
int64_t resident_walkers(K kernel, int threads, size_t lds, int walkers_per_block) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void*>(kernel), threads, lds) !=
            hipSuccess ||
        nb <= 0)
        nb = 1;
    return int64_t(nb) * walkers_per_block * cus();
}

// one launch of a walker kernel: `walkers` (stream, chunk) walks, `per_block` per workgroup
template <typename K>
hipError_t launch_walk(K kernel, int32_t id, int threads, int per_block, size_t lds, int min_m, StftArgs& a,
                       hipStream_t stream) {
    hipError_t e = set_lds(kernel, lds);
    if (e != hipSuccess) return e;
    pick_chunks(a.F, a.n_streams, resident_walkers(kernel, threads, lds, per_block), min_m, a.n_chunks, a.M);
    note_chunks(a.n_chunks);
    const int64_t grid = (int64_t(a.n_streams) * a.n_chunks + per_block - 1) / per_block;
    note_launch(id, grid);
    hipLaunchKernelGGL(kernel, dim3(unsigned(grid)), dim3(threads), lds, stream, a);
    return hipGetLastError();
}

template <int E, int S, bool XIN>
hipError_t istft_es(StftArgs& a, hipStream_t stream) {
    if constexpr (S > E) {
        return hipErrorInvalidValue;
    } else {
        return launch_walk(k_istft<E, S, XIN>, XIN ? CRLOT_K_STFT_MASKED : CRLOT_K_ISTFT, 64 * kW, kW,
                           istft_lds<E, XIN>(), std::max(4, E / S), a, stream);
    }
}
template <int E, bool XIN>
hipError_t istft_e(int s, StftArgs& a, hipStream_t stream) {
    switch (s) {
        case 1: return istft_es<E, 1, XIN>(a, stream);
        case 2: return istft_es<E, 2, XIN>(a, stream);
        case 4: return istft_es<E, 4, XIN>(a, stream);
        case 8: return istft_es<E, 8, XIN>(a, stream);
        default: return hipErrorInvalidValue;
    }
}
template <int L, int S, bool XIN>
hipError_t istft_wg_s(StftArgs& a, hipStream_t stream) {
    return launch_walk(k_istft_wg<L, S, XIN>, XIN ? CRLOT_K_STFT_MASKED : CRLOT_K_ISTFT, L, 1, istft_wg_lds<L>(),
                       std::max(4, 8 / S), a, stream);
}
template <int L, bool XIN>
hipError_t istft_wg(int s, StftArgs& a, hipStream_t stream) {
    switch (s) {
        case 1: return istft_wg_s<L, 1, XIN>(a, stream);
        case 2: return istft_wg_s<L, 2, XIN>(a, stream);
        case 4: return istft_wg_s<L, 4, XIN>(a, stream);
        case 8: return istft_wg_s<L, 8, XIN>(a, stream);
        default: return hipErrorInvalidValue;
    }
}

// N <= 1024: one frame per wave; N = 2048 / 4096: one frame per 128 / 256-lane workgroup
template <bool XIN>
hipError_t istft_dispatch(int n, int h, StftArgs& a, hipStream_t stream) {
    switch (n) {
        case 256: return istft_e<2, XIN>(h / 128, a, stream);
        case 512: return istft_e<4, XIN>(h / 128, a, stream);
        case 1024: return istft_e<8, XIN>(h / 128, a, stream);
        case 2048: return istft_wg<128, XIN>(h / 256, a, stream);
        case 4096: return istft_wg<256, XIN>(h / 512, a, stream);
        default: return hipErrorInvalidValue;
    }
}

StftArgs base_args(const Geometry& g, const DevTables& t, int n_streams, int64_t F) {
    StftArgs a{};
    a.t = t;
    a.n_streams = n_streams;
    a.F = int(F);
    a.h = g.h;
    a.pad = g.pad;
    a.pad_mode = g.pad_mode;
    a.ring_blocks = g.h > 0 ? g.ring_len / g.h : 1;
    a.gain = g.gain;
    return a;
}

}  // namespace

bool stft_supported(int n) { return e_of_n(n) != 0; }

bool istft_walk_supported(int n, int h) {
    if (e_of_n(n) == 0 || h <= 0 || n % h != 0) return false;
    const int unit = n <= 1024 ? 128 : n / 8;  // per-wave: 2 x 64 lanes; workgroup: 2 x n / 16 lanes
    if (h % unit != 0) return false;
    const int s = h / unit;
    return s == 1 || s == 2 || s == 4 || s == 8;
}

hipError_t launch_stft(const Geometry& g, const DevTables& t, const float* x, int n_streams, int64_t T,
                       int64_t ld_x, int64_t F, float* spec, int64_t ld_spec, int64_t ld_frame, hipStream_t stream) {
    if (!stft_supported(g.n) || F <= 0 || n_streams <= 0 || F > INT32_MAX) return hipErrorInvalidValue;
    StftArgs a = base_args(g, t, n_streams, F);
    a.x = x;
    a.T = T;
    a.ld_x = ld_x;
    a.spec = spec;
    a.ld_spec = ld_spec;
    a.ld_frame = ld_frame;
    switch (g.n) {
        case 256: return launch_walk(k_stft<2>, CRLOT_K_STFT, 64 * kW, kW, stft_lds<2>(), 1, a, stream);
        case 512: return launch_walk(k_stft<4>, CRLOT_K_STFT, 64 * kW, kW, stft_lds<4>(), 1, a, stream);
        case 1024: return launch_walk(k_stft<8>, CRLOT_K_STFT, 64 * kW, kW, stft_lds<8>(), 1, a, stream);
        case 2048: return launch_walk(k_stft_wg<128>, CRLOT_K_STFT, 128, 1, stft_wg_lds<128>(), 1, a, stream);
        case 4096: return launch_walk(k_stft_wg<256>, CRLOT_K_STFT, 256, 1, stft_wg_lds<256>(), 1, a, stream);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_istft(const Geometry& g, const DevTables& t, const SpecMask& m, const float* spec,
                        int64_t ld_spec, int64_t ld_frame, float* y, int n_streams, int64_t F, int64_t ld_y,
                        hipStream_t stream) {
    if (!istft_walk_supported(g.n, g.h) || !t.wsn || !t.rden || F <= 0 || n_streams <= 0 || F > INT32_MAX ||
        g.ring_len % g.h != 0)
        return hipErrorInvalidValue;
    StftArgs a = base_args(g, t, n_streams, F);
    a.sin = spec;
    a.ld_spec = ld_spec;
    a.ld_frame = ld_frame;
    a.y = y;
    a.ld_y = ld_y;
    a.mask = m;
    return istft_dispatch<false>(g.n, g.h, a, stream);
}

hipError_t launch_roundtrip_masked(const Geometry& g, const DevTables& t, const SpecMask& m, const float* x,
                                   float* y, int n_streams, int64_t T, int64_t ld_x, int64_t ld_y, int64_t F,
                                   hipStream_t stream) {
    if (!istft_walk_supported(g.n, g.h) || !t.wsn || !t.rden || F <= 0 || n_streams <= 0 || F > INT32_MAX ||
        g.ring_len % g.h != 0 || (g.pad & 1))
        return hipErrorInvalidValue;
    StftArgs a = base_args(g, t, n_streams, F);
    a.x = x;
    a.T = T;
    a.ld_x = ld_x;
    a.y = y;
    a.ld_y = ld_y;
    a.mask = m;
    return istft_dispatch<true>(g.n, g.h, a, stream);
}

hipError_t launch_frames_windowed(const Geometry& g, const DevTables& t, const float* x, int n_streams, int64_t T,
                                  int64_t ld_x, int64_t F, float* frames, hipStream_t stream) {
    const int64_t rows = int64_t(n_streams) * F;
    if (rows <= 0 || rows > INT32_MAX) return hipErrorInvalidValue;
    note_launch(CRLOT_K_FRAMES_W, rows);
    hipLaunchKernelGGL(k_frames_w, dim3(unsigned(rows)), dim3(256), 0, stream, x, ld_x, T, t.wa, frames, F, g.n,
                       g.h, g.pad, g.pad_mode);
    return hipGetLastError();
}

hipError_t launch_spec_step(const DevTables& t, const SpecMask& m, const float* spec, int64_t ld_spec,
                            int64_t ld_frame, float* out, int n_streams, int64_t F, int bins, hipStream_t stream) {
    const int64_t rows = int64_t(n_streams) * F;
    if (rows <= 0 || rows > INT32_MAX) return hipErrorInvalidValue;
    note_launch(CRLOT_K_SPEC_STEP, rows);
    hipLaunchKernelGGL(k_spec_step, dim3(unsigned(rows)), dim3(256), 0, stream, spec, ld_spec, ld_frame, out, F,
                       bins, t.gain, m);
    return hipGetLastError();
}

}  // namespace crlot
