// pairn_spec.hip -- the spectral entries and the masked round trip as frame
// pairs at K_pairN's sizes 882 (20 ms at 44.1 kHz), 1000, 640, 400, 320 (one wave
// per transform) and 1764, 1920 (40 ms at 44.1 / 48 kHz; two waves, one walk per
// workgroup), any hop H >= 32 whose ring the plan allows:
//   K_pair_stft   k_pn_stft<K>        (crlot_stft)
//   K_pair_istft  k_pn_istft<K,MASK>  (crlot_istft_ola)
//   K_pair_mask   k_pn_mask<K>        (crlot_roundtrip with a per-frame mask)
// on fft_pairn.h's transform (compile-time Stockham passes over composite
// radices in one LDS buffer per transform, natural order in and out), frames
// loaded whole and the overlap-add in a per-walk LDS ring, as K_pairN
// (pair_n.hip).  At 1764 and 1920 the transform spans the two waves of a workgroup (its
// fences are barriers) and the regime verdicts are shared through LDS.
//
// The spectrum of the pair z = a w + i b w is in natural order in the wave's
// buffer after the forward passes, so each lane works on its own real bins
// kr = t + L i <= N/2 and their partners N - kr, with no bin map:
//   stft:  A[k] = (Z[k] + conj Z[-k]) / 2, B[k] = (Z[k] - conj Z[-k]) / 2i;
//   istft: Z[k] = A' + i B' and Z[N-k] = conj A' + i conj B' written from the
//          stepped rows, then the inverse passes;
//   mask:  Z'[k] = c1 Z[k] + c2 conj Z[-k] in place, c1 = (Ga + Gb) / 2,
//          c2 = (Ga - Gb) / 2.
// Regimes per pair, wave-uniform: the pair when its samples keep px_lo <= |x| <=
// px_hi (/ 2^20 with a mask, whose values must be finite and within 2^20) and
// its stepped spectra are finite and below 2^60; otherwise each frame alone with
// the full sanitize.  The inverse output is scaled and sanitized as
// kissfft_adapter.cc:154-163 does (o = sanit(v / N)), pushed with fma(o, ws g,
// ring), divided by the plan's den (IEEE).  Results equal the per-frame kissfft
// formulation within float32 rounding.
#include <algorithm>

#include "fft_pairn.h"
#include "fused_common.h"

namespace crlot {
namespace fk {

namespace {

constexpr int kNW = 4;  // waves per workgroup at the one-wave sizes (one walk each)

template <int K>
struct QN {
    static constexpr int N = K % 100000, L = dev::pn_lanes(K);  // lanes per transform
    static constexpr int WALKS = L == 64 ? kNW : 1, THREADS = WALKS * L;  // per workgroup
    static constexpr int E = (N + L - 1) / L, LAST = N - L * (E - 1), P2 = N / 2;
    static constexpr int IB = (P2 + 1 + L - 1) / L;  // natural real-bin rows per lane
    static constexpr dev::PnFac FAC = dev::pn_factor(K);
    static_assert(FAC.rest == 1 && N % 2 == 0, "a plan of an even N");
    static __device__ __forceinline__ bool valid(int m, int t) { return m + 1 < E || t < LAST; }
    static __device__ __forceinline__ void fwd(dev::pc* buf, const dev::pc* tw, int t) {
        dev::pn_passes<false, K, 0, FAC.n>(buf, tw, dev::pn_opaque(t));
    }
    static __device__ __forceinline__ void inv(dev::pc* buf, const dev::pc* tw, int t) {
        dev::pn_passes<true, K, 0, FAC.n>(buf, tw, dev::pn_opaque(t));
    }
};

__host__ __device__ inline int qn_ring(int n, int h) {
    const int span = h * ((n + h - 1) / h);
    int r = 1;
    while (r < span) r <<= 1;
    return r;
}
// LDS: [twiddles tw_len cf] | per walk [buffer N cf] | per walk [ring RL f]
// (synthesis kernels) | the verdicts of the walk's waves (two-wave walks)
template <int K>
size_t qn_lds(int h, bool ring) {
    using G = QN<K>;
    return sizeof(dev::pc) * size_t(G::FAC.tw_len + G::WALKS * G::N) +
           (ring ? sizeof(float) * qn_ring(G::N, h) * G::WALKS : 0) + 16;
}

template <int K>
struct QNSmem {
    dev::pc* tw;
    dev::pc* buf;
    float* ring;
    uint32_t* votes;
    __device__ QNSmem(char* smem, int pw, int RL) {
        using G = QN<K>;
        tw = reinterpret_cast<dev::pc*>(smem);
        buf = tw + G::FAC.tw_len + pw * G::N;
        float* rings = reinterpret_cast<float*>(tw + G::FAC.tw_len + G::WALKS * G::N);
        ring = rings + pw * RL;
        votes = reinterpret_cast<uint32_t*>(rings + G::WALKS * RL);
    }
    // the walk's verdict: the wave's ballot (one-wave walks), or both waves' (two-wave
    // walks: posted in LDS between barriers, which the transform's fences are anyway)
    __device__ __forceinline__ bool all(bool wave_ok) const {
        if constexpr (QN<K>::L == 64) {
            return wave_ok;
        } else {
            const int wave = threadIdx.x >> 6;
            if ((threadIdx.x & 63) == 0) votes[wave] = wave_ok ? 1u : 0u;
            __syncthreads();
            const bool r = (votes[0] & votes[1]) != 0u;
            __syncthreads();  // (both read before the next post)
            return r;
        }
    }
};
// the plan's pass twiddles into LDS (the whole workgroup), then a barrier
template <int K>
__device__ __forceinline__ void qn_stage_tw(dev::pc* tw, const float* g) {
    const dev::pc* gp = reinterpret_cast<const dev::pc*>(g);
    for (int i = threadIdx.x; i < QN<K>::FAC.tw_len; i += QN<K>::THREADS) tw[i] = gp[i];
    __syncthreads();
}

// frame at `origin`: x[origin + t + L m] (m < E, the last row partial), the
// plan's padding outside [0, T)
template <int K>
__device__ __forceinline__ void qn_load(float (&f)[QN<K>::E], __amdgpu_buffer_rsrc_t rx, int t, int origin, int T,
                                        int mode) {
    using G = QN<K>;
    if (origin >= 0 && origin + G::N <= T) {
#pragma unroll
        for (int m = 0; m < G::E; ++m)
            f[m] = G::valid(m, t) ? dev::bload1(rx, (origin + t) * 4 + m * (4 * G::L), 0) : 0.0f;
    } else {
#pragma unroll
        for (int m = 0; m < G::E; ++m) f[m] = G::valid(m, t) ? fetch_x(rx, origin + t + G::L * m, T, mode) : 0.0f;
    }
}
template <int E>
__device__ __forceinline__ bool qn_ok(const float (&f)[E], float lo, float hi) {
    bool bad = false;
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const float a = __builtin_fabsf(f[m]);
        bad |= !((a >= lo) & (a <= hi)) & (a != 0.0f);
    }
    return __builtin_amdgcn_ballot_w64(bad) == 0;
}

// The per-walk OLA ring over the natural-order inverse output in the buffer:
// push frame k (o = sanit(v / N), fma(o, ws g, ring) in ascending k), produce
// block k (ring / den, clear; stored when k >= f0).
template <int K>
struct QNOla {
    static constexpr int N = QN<K>::N, E = QN<K>::E, L = QN<K>::L;
    float* ring;
    int H, RM, ring_blocks, f0, t;
    const float* den;
    __amdgpu_buffer_rsrc_t ry, ry_null;
    __device__ __forceinline__ void clear() {
        for (int i = t; i <= RM; i += L) ring[i] = 0.0f;
        dev::pn_fence<K>();
    }
    template <bool IMAG>
    __device__ __forceinline__ void push(const dev::pc* buf, const float (&wsg)[E], float inv_n, int k) {
        const int base = k * H + t;  // k H < 2^27 (host-checked)
#pragma unroll
        for (int m = 0; m < E; ++m) {
            if (QN<K>::valid(m, t)) {
                const dev::pc v = buf[t + L * m];
                const int pos = (base + L * m) & RM;
                const float o = dev::sanit((IMAG ? v.y : v.x) * inv_n);
                ring[pos] = __builtin_fmaf(o, wsg[m], ring[pos]);
            }
        }
        dev::pn_fence<K>();
    }
    __device__ __forceinline__ void produce(int k) {
        const int base = k * H;
        const float* dk = den + (k % ring_blocks) * H;
        const __amdgpu_buffer_rsrc_t rk = k >= f0 ? ry : ry_null;
        for (int j = t; j < H; j += L) {
            const int pos = (base + j) & RM;
            const float s = ring[pos];
            ring[pos] = 0.0f;
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, s / dk[j]), rk, (base + j) * 4, 0, 0);
        }
        dev::pn_fence<K>();
    }
};

struct QNWalk {
    int s, f0, f1, fs;
};
__device__ __forceinline__ bool qn_walk(const FusedArgs& a, int gw, int NB, QNWalk& w) {
    if (gw >= a.n_streams * a.n_chunks) return false;
    w.s = gw / a.n_chunks;
    const int c = gw - w.s * a.n_chunks;
    w.f0 = c * a.M;
    w.f1 = min(a.F, w.f0 + a.M);
    w.fs = max(0, w.f0 - (NB - 1)) & ~1;  // pairs start on even frames
    return true;
}
template <int K>
__device__ __forceinline__ void qn_ola_init(QNOla<K>& o, const FusedArgs& a, float* ring, int RL, const QNWalk& w,
                                            int t) {
    o.ring = ring;
    o.H = a.hop;
    o.RM = RL - 1;
    o.ring_blocks = a.ring_blocks;
    o.f0 = w.f0;
    o.t = t;
    o.den = a.t.den;
    o.ry = dev::make_rsrc(a.y + int64_t(w.s) * a.ld_y, span_bytes(a.out_len, 1));
    o.ry_null = dev::make_rsrc(a.y, 0u);
    o.clear();
}

// ------------------------------------------------------------------ K_pair_stft
template <int K>
__global__ __launch_bounds__(QN<K>::THREADS, 2) void k_pn_stft(const PairSpecArgs pa) {
    using G = QN<K>;
    const FusedArgs& a = pa.f;
    constexpr int N = G::N, E = G::E, P2 = G::P2, IB = G::IB;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int t = threadIdx.x % G::L;
    const int pw = __builtin_amdgcn_readfirstlane(threadIdx.x / G::L);  // the walk in the workgroup
    QNSmem<K> sm(smem, pw, 0);
    qn_stage_tw<K>(sm.tw, a.t.ptwn);
    const int gw = blockIdx.x * G::WALKS + pw;
    if (gw >= a.n_streams * a.n_chunks) return;
    const int s = gw / a.n_chunks, c = gw - s * a.n_chunks;
    const int f0 = c * a.M, f1 = min(a.F, f0 + a.M);  // (M even: chunks start on even frames)
    const int H = a.hop;
    const __amdgpu_buffer_rsrc_t rx = dev::make_rsrc(a.x + int64_t(s) * a.ld_x, span_bytes(a.T, 1));
    float* so = pa.spec + int64_t(s) * pa.ld_spec;
    float wa[E];
#pragma unroll
    for (int m = 0; m < E; ++m) wa[m] = G::valid(m, t) ? a.t.wa[t + G::L * m] : 0.0f;
    const float xlo = a.t.px_lo, xhi = a.t.px_hi;
    float fa[E], fb[E];
    auto load = [&](float (&f)[E], int k) { qn_load<K>(f, rx, t, k * H - a.pad, a.T, a.pad_mode); };
    load(fa, f0);
    load(fb, f0 + 1);
    for (int k = f0; k < f1; k += 2) {
        const bool two = k + 1 < f1;
        float2* ra = reinterpret_cast<float2*>(so + int64_t(k) * pa.ld_frame);
        float2* rb = reinterpret_cast<float2*>(so + int64_t(k + 1) * pa.ld_frame);
        const bool paired = sm.all(qn_ok(fa, xlo, xhi) && qn_ok(fb, xlo, xhi));
        auto pass = [&](auto pc_) {  // P = 0 / 1: frame k / k+1 alone; paired: both (P = 0)
            constexpr int P = decltype(pc_)::value;
#pragma unroll
            for (int m = 0; m < E; ++m)
                if (G::valid(m, t))
                    sm.buf[t + G::L * m] = paired ? dev::pc_mk(fa[m] * wa[m], fb[m] * wa[m])
                                                : dev::pc_mk(dev::sanit((P ? fb[m] : fa[m]) * wa[m]), 0.0f);
            dev::pn_fence<K>();
            G::fwd(sm.buf, sm.tw, t);
#pragma unroll
            for (int i = 0; i < IB; ++i) {
                const int kr = t + G::L * i;
                if (kr <= P2) {
                    const dev::pc z = sm.buf[kr];
                    if (paired) {
                        const dev::pc zp = sm.buf[kr == 0 ? 0 : N - kr];
                        ra[kr] = make_float2(0.5f * (z.x + zp.x), 0.5f * (z.y - zp.y));
                        if (two) rb[kr] = make_float2(0.5f * (z.y + zp.y), 0.5f * (zp.x - z.x));
                    } else {  // (DC and Nyquist: imaginary part exactly 0, as kiss_fftr writes them)
                        (P ? rb : ra)[kr] = make_float2(z.x, (kr == 0 || kr == P2) ? 0.0f : z.y);
                    }
                }
            }
            dev::pn_fence<K>();  // (the reads before the next transform's writes)
        };
        pass(std::integral_constant<int, 0>());
        if (!paired && two) pass(std::integral_constant<int, 1>());
        load(fa, k + 2);
        load(fb, k + 3);
    }
}

// ------------------------------------------------------------------ K_pair_istft
template <int K, bool MASK>
__global__ __launch_bounds__(QN<K>::THREADS, 2) void k_pn_istft(const PairSpecArgs pa) {
    using G = QN<K>;
    const FusedArgs& a = pa.f;
    constexpr int N = G::N, E = G::E, P2 = G::P2, IB = G::IB;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int t = threadIdx.x % G::L;
    const int pw = __builtin_amdgcn_readfirstlane(threadIdx.x / G::L);  // the walk in the workgroup
    const int H = a.hop, NB = (N + H - 1) / H, RL = qn_ring(N, H);
    QNSmem<K> sm(smem, pw, RL);
    qn_stage_tw<K>(sm.tw, a.t.ptwn);
    QNWalk w;
    if (!qn_walk(a, blockIdx.x * G::WALKS + pw, NB, w)) return;
    QNOla<K> ola;
    qn_ola_init<K>(ola, a, sm.ring, RL, w, t);
    float wsg[E];
#pragma unroll
    for (int m = 0; m < E; ++m) wsg[m] = G::valid(m, t) ? a.t.ws[t + G::L * m] * a.gain : 0.0f;
    const float* sb = pa.sin + int64_t(w.s) * pa.ld_spec;
    const float* mrow0 = MASK ? pa.mask.p + int64_t(w.s) * pa.mask.ld_stream : nullptr;
    // the pair's rows (and mask rows) by real bin kr = t + L i <= N/2, coalesced;
    // stepped -- (X g) m, re and im each; DC and Nyquist imaginary parts dropped
    float2 ra_[IB], rb_[IB];
    auto load_rows = [&](int k) -> bool {
        const float2* ra = reinterpret_cast<const float2*>(sb + int64_t(k) * pa.ld_frame);
        const float2* rb = reinterpret_cast<const float2*>(sb + int64_t(k + 1) * pa.ld_frame);
        const bool two = k + 1 < a.F;
        const float* m0 = MASK ? mrow0 + int64_t(k) * pa.mask.ld_frame : nullptr;
        const float* m1 = MASK && two ? m0 + pa.mask.ld_frame : m0;
        bool bad = false;
#pragma unroll
        for (int i = 0; i < IB; ++i) {
            const int kr = t + G::L * i;
            const bool on = kr <= P2;
            const float2 xa = on ? ra[kr] : make_float2(0.f, 0.f);
            const float2 xb = on && two ? rb[kr] : make_float2(0.f, 0.f);
            const float g = on && a.t.gain ? a.t.gain[kr] : 1.0f;
            float ax = xa.x * g, ay = xa.y * g, bx = xb.x * g, by = xb.y * g;
            if constexpr (MASK) {
                const float ma = on ? m0[kr] : 0.f, mb = on ? m1[kr] : 0.f;
                ax *= ma;
                ay *= ma;
                bx *= mb;
                by *= mb;
            }
            if (kr == 0 || kr == P2) ay = by = 0.0f;
            const float mx = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(ax), __builtin_fabsf(ay)),
                                             __builtin_fmaxf(__builtin_fabsf(bx), __builtin_fabsf(by)));
            bad |= !(mx <= 0x1p60f) | (ax != ax) | (ay != ay) | (bx != bx) | (by != by);  // (NaN, Inf, huge)
            ra_[i] = make_float2(ax, ay);
            rb_[i] = make_float2(bx, by);
        }
        return __builtin_amdgcn_ballot_w64(bad) == 0;
    };
    // the full spectrum in natural order: the pair form Z = A' + i B' (conjugate-
    // extended above N/2), or frame p's own X (Hermitian)
    auto put = [&](int form) {
#pragma unroll
        for (int i = 0; i < IB; ++i) {
            const int kr = t + G::L * i;
            if (kr <= P2) {
                const float2 A = ra_[i], B = rb_[i];
                dev::pc lo, hi;
                if (form == 0) {
                    lo = dev::pc_mk(A.x - B.y, A.y + B.x);
                    hi = dev::pc_mk(A.x + B.y, B.x - A.y);
                } else {
                    const float2 X = form == 1 ? A : B;
                    lo = dev::pc_mk(X.x, X.y);
                    hi = dev::pc_mk(X.x, -X.y);
                }
                sm.buf[kr] = lo;
                if (kr != 0 && kr != P2) sm.buf[N - kr] = hi;
            }
        }
        dev::pn_fence<K>();
    };
    for (int k = w.fs; k < w.f1; k += 2) {
        if (sm.all(load_rows(k))) {
            put(0);
            G::inv(sm.buf, sm.tw, t);
            ola.template push<false>(sm.buf, wsg, a.inv_n, k);
            ola.produce(k);
            ola.template push<true>(sm.buf, wsg, a.inv_n, k + 1);
            if (k + 1 < w.f1) ola.produce(k + 1);
        } else {  // each frame alone, full sanitize
            put(1);
            G::inv(sm.buf, sm.tw, t);
            ola.template push<false>(sm.buf, wsg, a.inv_n, k);
            ola.produce(k);
            if (k + 1 < w.f1) {
                put(2);
                G::inv(sm.buf, sm.tw, t);
                ola.template push<false>(sm.buf, wsg, a.inv_n, k + 1);
                ola.produce(k + 1);
            }
        }
    }
}

// ------------------------------------------------------------------ K_pair_mask
template <int K>
__global__ __launch_bounds__(QN<K>::THREADS, 2) void k_pn_mask(const PairSpecArgs pa) {
    using G = QN<K>;
    const FusedArgs& a = pa.f;
    constexpr int N = G::N, E = G::E, P2 = G::P2, IB = G::IB;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int t = threadIdx.x % G::L;
    const int pw = __builtin_amdgcn_readfirstlane(threadIdx.x / G::L);  // the walk in the workgroup
    const int H = a.hop, NB = (N + H - 1) / H, RL = qn_ring(N, H);
    QNSmem<K> sm(smem, pw, RL);
    qn_stage_tw<K>(sm.tw, a.t.ptwn);
    QNWalk w;
    if (!qn_walk(a, blockIdx.x * G::WALKS + pw, NB, w)) return;
    QNOla<K> ola;
    qn_ola_init<K>(ola, a, sm.ring, RL, w, t);
    const __amdgpu_buffer_rsrc_t rx = dev::make_rsrc(a.x + int64_t(w.s) * a.ld_x, span_bytes(a.T, 1));
    float wa[E], wsg[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        wa[m] = G::valid(m, t) ? a.t.wa[t + G::L * m] : 0.0f;
        wsg[m] = G::valid(m, t) ? a.t.ws[t + G::L * m] * a.gain : 0.0f;
    }
    const float xlo = a.t.px_lo, xhi = a.t.px_hi * 0x1p-20f;  // (mask values up to 2^20)
    const float* mrow0 = pa.mask.p + int64_t(w.s) * pa.mask.ld_stream;
    auto row_a = [&](int k) { return mrow0 + int64_t(k) * pa.mask.ld_frame; };
    auto row_b = [&](int k) { return k + 1 < a.F ? row_a(k) + pa.mask.ld_frame : row_a(k); };  // (past F: unused)
    float ma[IB], mb[IB];  // the pair's mask rows by real bin t + L i (<= N/2; 1 beyond)
    auto load_rows = [&](int k) {
        const float* r0 = row_a(k);
        const float* r1 = row_b(k);
#pragma unroll
        for (int i = 0; i < IB; ++i) {
            const int kr = t + G::L * i;
            ma[i] = kr <= P2 ? r0[kr] : 1.0f;
            mb[i] = kr <= P2 ? r1[kr] : 1.0f;
        }
    };
    auto rows_ok = [&]() {
        bool bad = false;
#pragma unroll
        for (int i = 0; i < IB; ++i)
            bad |= !(__builtin_fabsf(ma[i]) <= 0x1p20f) | !(__builtin_fabsf(mb[i]) <= 0x1p20f);  // (NaN too)
        return __builtin_amdgcn_ballot_w64(bad) == 0;
    };
    float fa[E], fb[E];
    auto load = [&](float (&f)[E], int k) { qn_load<K>(f, rx, t, k * H - a.pad, a.T, a.pad_mode); };
    load(fa, w.fs);
    load(fb, w.fs + 1);
    load_rows(w.fs);
    for (int k = w.fs; k < w.f1; k += 2) {
        const bool paired = sm.all(qn_ok(fa, xlo, xhi) && qn_ok(fb, xlo, xhi) && rows_ok());
        const bool partner_frame = k + 1 < a.F;  // frame k+1 past the last: imaginary part 0
        if (paired) {
#pragma unroll
            for (int m = 0; m < E; ++m)
                if (G::valid(m, t)) sm.buf[t + G::L * m] = dev::pc_mk(fa[m] * wa[m], partner_frame ? fb[m] * wa[m] : 0.0f);
            dev::pn_fence<K>();
            G::fwd(sm.buf, sm.tw, t);
            // the step on this lane's bin pairs {kr, N - kr}, in place
#pragma unroll
            for (int i = 0; i < IB; ++i) {
                const int kr = t + G::L * i;
                if (kr <= P2) {
                    const int jr = kr == 0 ? 0 : N - kr;
                    const float g = a.t.gain ? a.t.gain[kr] : 1.0f;
                    const float ga = g * ma[i], gb = g * mb[i];
                    const float c1 = 0.5f * (ga + gb), c2 = 0.5f * (ga - gb);
                    const dev::pc z = sm.buf[kr], zp = sm.buf[jr];
                    sm.buf[kr] = dev::pc_mk(__builtin_fmaf(c2, zp.x, c1 * z.x), __builtin_fmaf(-c2, zp.y, c1 * z.y));
                    if (jr != kr)
                        sm.buf[jr] = dev::pc_mk(__builtin_fmaf(c2, z.x, c1 * zp.x), __builtin_fmaf(-c2, z.y, c1 * zp.y));
                }
            }
            dev::pn_fence<K>();
            load(fa, k + 2);  // (in flight during the inverse and the OLA)
            load(fb, k + 3);
            if (k + 2 < w.f1) load_rows(k + 2);
            G::inv(sm.buf, sm.tw, t);
            ola.template push<false>(sm.buf, wsg, a.inv_n, k);
            ola.produce(k);
            ola.template push<true>(sm.buf, wsg, a.inv_n, k + 1);
            if (k + 1 < w.f1) ola.produce(k + 1);
        } else {  // each frame alone, full sanitize, its own gain g m
            auto pass = [&](const float (&f)[E], const float* r, int kk) {
#pragma unroll
                for (int m = 0; m < E; ++m)
                    if (G::valid(m, t)) sm.buf[t + G::L * m] = dev::pc_mk(dev::sanit(f[m] * wa[m]), 0.0f);
                dev::pn_fence<K>();
                G::fwd(sm.buf, sm.tw, t);
#pragma unroll
                for (int m = 0; m < E; ++m) {
                    if (G::valid(m, t)) {
                        const int n = t + G::L * m, kr = n <= P2 ? n : N - n;
                        sm.buf[n] = sm.buf[n] * ((a.t.gain ? a.t.gain[kr] : 1.0f) * r[kr]);
                    }
                }
                dev::pn_fence<K>();
                G::inv(sm.buf, sm.tw, t);
                ola.template push<false>(sm.buf, wsg, a.inv_n, kk);
                ola.produce(kk);
            };
            pass(fa, row_a(k), k);
            if (k + 1 < w.f1) pass(fb, row_b(k), k + 1);
            load(fa, k + 2);
            load(fb, k + 3);
            if (k + 2 < w.f1) load_rows(k + 2);
        }
    }
}

template <int K, typename KF>
hipError_t qn_launch(KF kernel, const PairSpecArgs& a, int64_t walks, int32_t kind, bool ring, hipStream_t stream) {
    using G = QN<K>;
    const size_t lds = qn_lds<K>(a.f.hop, ring);
    hipError_t e = set_lds(kernel, lds);
    if (e != hipSuccess) return e;
    const int64_t grid = (walks + G::WALKS - 1) / G::WALKS;
    note_launch(kind, grid);
    hipLaunchKernelGGL(kernel, dim3(unsigned(grid)), dim3(G::THREADS), lds, stream, a);
    return hipGetLastError();
}

// chunks: about two resident rounds of walks, each >= `min_m` frames, an even length
int64_t qn_chunks(FusedArgs& f, int64_t F, int n_streams, int64_t min_m) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    const int64_t resident = int64_t(cus) * 8, S = std::max(1, n_streams);  // (walks a CU holds, about)
    int64_t c = std::max<int64_t>(1, std::min<int64_t>(F / min_m, (2 * resident + S - 1) / S));
    c = chunks_or(c, F);
    int64_t m = (F + c - 1) / c;
    m += m & 1;
    f.M = int(m);
    f.n_chunks = int((F + m - 1) / m);
    note_chunks(f.n_chunks);
    return S * f.n_chunks;
}

// the plan keys (fft_pairn.h pn_factor; the release plans' radix lists; 1764, 1920: two waves)
template <typename F>
bool qn_dispatch(int n, F&& f) {
    switch (n) {
        case 1764: f(std::integral_constant<int, 1001764>{}); return true;
        case 1920: f(std::integral_constant<int, 1001920>{}); return true;
        case 320: f(std::integral_constant<int, 320>{}); return true;
        case 400: f(std::integral_constant<int, 400>{}); return true;
        case 640: f(std::integral_constant<int, 640>{}); return true;
        case 882: f(std::integral_constant<int, 882>{}); return true;
        case 1000: f(std::integral_constant<int, 1000>{}); return true;
        default: return false;
    }
}

}  // namespace

}  // namespace fk

bool pairn_spec_supported(int n, int h, int ring_len) {
    return fk::qn_dispatch(n, [](auto) {}) && h >= 32 && h <= n && ring_len % h == 0;
}

// crlot_stft at K_pairN's one-wave sizes as frame pairs
hipError_t launch_pairn_stft(const Geometry& g, const DevTables& t, const float* x, int n_streams, int64_t T,
                             int64_t ld_x, int64_t F, float* spec, int64_t ld_spec, int64_t ld_frame,
                             hipStream_t stream) {
    if (!pairn_spec_supported(g.n, g.h, g.ring_len) || F <= 0 || n_streams <= 0 || !t.ptwn || !t.wa ||
        T >= (int64_t(1) << 27))
        return hipErrorInvalidValue;
    fk::PairSpecArgs a{};
    a.f.t = t;
    a.f.x = x;
    a.f.ld_x = ld_x;
    a.f.T = int(T);
    a.f.n_streams = n_streams;
    a.f.F = int(F);
    a.f.hop = g.h;
    a.f.pad = g.pad;
    a.f.pad_mode = g.pad_mode;
    a.spec = spec;
    a.ld_spec = ld_spec;
    a.ld_frame = ld_frame;
    const int64_t waves = fk::qn_chunks(a.f, F, n_streams, 32);
    hipError_t e = hipErrorInvalidValue;
    fk::qn_dispatch(g.n, [&](auto kc) {
        constexpr int K = decltype(kc)::value;
        e = fk::qn_launch<K>(fk::k_pn_stft<K>, a, waves, CRLOT_K_PAIR_STFT, false, stream);
    });
    return e;
}

// crlot_istft_ola at K_pairN's one-wave sizes as frame pairs (the plan's mask, if any, applied)
hipError_t launch_pairn_istft(const Geometry& g, const DevTables& t, const SpecMask& m, const float* spec,
                              int64_t ld_spec, int64_t ld_frame, float* y, int n_streams, int64_t F, int64_t ld_y,
                              hipStream_t stream) {
    if (!pairn_spec_supported(g.n, g.h, g.ring_len) || F <= 0 || n_streams <= 0 || !t.ptwn || !t.ws || !t.den ||
        F * g.h + g.n >= (int64_t(1) << 27))
        return hipErrorInvalidValue;
    fk::PairSpecArgs a{};
    a.f.t = t;
    a.f.y = y;
    a.f.ld_y = ld_y;
    a.f.out_len = int(F * g.h);
    a.f.n_streams = n_streams;
    a.f.F = int(F);
    a.f.hop = g.h;
    a.f.ring_blocks = g.ring_len / g.h;
    a.f.inv_n = g.inv_n;
    a.f.gain = g.gain;
    a.sin = spec;
    a.ld_spec = ld_spec;
    a.ld_frame = ld_frame;
    a.mask = m;
    const int64_t waves = fk::qn_chunks(a.f, F, n_streams, 48);
    hipError_t e = hipErrorInvalidValue;
    fk::qn_dispatch(g.n, [&](auto kc) {
        constexpr int K = decltype(kc)::value;
        e = m.p ? fk::qn_launch<K>(fk::k_pn_istft<K, true>, a, waves, CRLOT_K_PAIR_ISTFT, true, stream)
                : fk::qn_launch<K>(fk::k_pn_istft<K, false>, a, waves, CRLOT_K_PAIR_ISTFT, true, stream);
    });
    return e;
}

// crlot_roundtrip at K_pairN's one-wave sizes with a per-frame mask, one walk
hipError_t launch_pairn_masked(const Geometry& g, const DevTables& t, const SpecMask& m, const float* x, float* y,
                               int n_streams, int64_t T, int64_t ld_x, int64_t ld_y, int64_t F, int64_t out_len,
                               hipStream_t stream) {
    if (!pairn_spec_supported(g.n, g.h, g.ring_len) || F <= 0 || n_streams <= 0 || !m.p || !t.ptwn || !t.wa ||
        !t.ws || !t.den || T >= (int64_t(1) << 27) || out_len + g.n >= (int64_t(1) << 27))
        return hipErrorInvalidValue;
    fk::PairSpecArgs a{};
    a.f.t = t;
    a.f.x = x;
    a.f.y = y;
    a.f.ld_x = ld_x;
    a.f.ld_y = ld_y;
    a.f.T = int(T);
    a.f.out_len = int(out_len);
    a.f.n_streams = n_streams;
    a.f.F = int(F);
    a.f.hop = g.h;
    a.f.ring_blocks = g.ring_len / g.h;
    a.f.pad = g.pad;
    a.f.pad_mode = g.pad_mode;
    a.f.inv_n = g.inv_n;
    a.f.gain = g.gain;
    a.mask = m;
    const int64_t waves = fk::qn_chunks(a.f, F, n_streams, 48);
    hipError_t e = hipErrorInvalidValue;
    fk::qn_dispatch(g.n, [&](auto kc) {
        constexpr int K = decltype(kc)::value;
        e = fk::qn_launch<K>(fk::k_pn_mask<K>, a, waves, CRLOT_K_PAIR_MASK, true, stream);
    });
    return e;
}

}  // namespace crlot
