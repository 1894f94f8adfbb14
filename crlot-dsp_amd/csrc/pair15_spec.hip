// pair15_spec.hip -- the spectral entries and the masked round trip as frame
// pairs at N = 960 (20 ms at 48 kHz) and N = 480 (10 ms), any hop H >= 32 whose
// ring the plan allows:
//   K_pair_stft   k_p15_stft<L>          (crlot_stft)
//   K_pair_istft  k_p15_istft<L,MASK,PF> (crlot_istft_ola)
//   K_pair_mask   k_p15_mask<L>          (crlot_roundtrip with a per-frame mask)
// on K_pair15's transforms (fft_pair15.h: Good-Thomas 15 over the registers, then
// a 64-lane stage -- N = 960, L = 64, one walk per wave -- or a 32-lane one --
// N = 480, L = 32, the two halves of a wave walk streams 2u and 2u+1 over the same
// chunk), frames loaded whole (H is not a lane multiple) and the overlap-add in a
// per-walk LDS ring, as K_pair15 (pair_any.hip).
//
// Bin maps (half-lane h = lane mod L; tests/test_pair_bin_maps.py checks them
// exhaustively):
//   960: bin k1 + 15 (j + 4 d), k1 = (h & 3) + 4 (h >> 4), j = (h >> 2) & 3
//        (pair15_bin); partner N - k in register 15 - d of lane
//        (15 - k1 & 3) + 4 (3 - j) + 16 (15 - k1 >> 2), for k1 = 0 lane 4 (4 - j);
//   480: bin k1 + 15 (c + 2 e), k1 = (h & 7) + 8 (h >> 4), c = (h >> 3) & 1
//        (pair15h_bin); partner in register 15 - e of half-lane
//        (15 - k1 & 7) + 8 (1 - c) + 16 (15 - k1 >> 3), for k1 = 0 itself;
// in both, half-lane 0's partners are its own registers (16 - d) mod 16 and k1 =
// 15 is the zero row (no bins; stays zero).  The real bins 0 .. N/2 are registers
// d < 8 of the bin lanes plus register 8 of half-lane 0 (bin N/2), as at N = 1024,
// so the split / merge / step are pair_stft.hip's and pair_mask.hip's:
//   stft:  A[k] = (Z[k] + conj Z[-k]) / 2, B[k] = (Z[k] - conj Z[-k]) / 2i;
//   istft: the stepped rows staged by real bin in the wave's transpose buffer
//          (one region per half), read back scrambled as Z = A' + i B';
//   mask:  Z' = c1 Z + c2 conj Z[-k], c1 = (Ga + Gb) / 2, c2 = (Ga - Gb) / 2.
// Regimes per pair, wave-uniform (at N = 480 both halves' streams together): the
// pair when its samples keep px_lo <= |x| <= px_hi (/ 2^20 with a mask, whose
// values must be finite and within 2^20) and its stepped spectra are finite and
// below 2^60; otherwise each frame alone with the full sanitize.  The inverse
// output is scaled and sanitized as kissfft_adapter.cc:154-163 does
// (o = sanit(v / N)) and pushed with fma(o, ws g, ring); produce divides by the
// plan's den (IEEE; the divisors of both blocks fetched ahead when H <= 4 L).
// Results equal the per-frame kissfft formulation within float32 rounding.
#include <algorithm>
#include <type_traits>

#include "fft_pair15.h"
#include "fused_common.h"

namespace crlot {
namespace fk {

namespace {

constexpr int kQW = 4;   // waves per workgroup
constexpr int kQE = 15;  // samples per lane per frame

template <int L>
struct Q15 {
    static constexpr int N = 15 * L, P2 = N / 2, HALVES = 64 / L;
    static constexpr int SB = 2 * (P2 + 1);  // staging per half: A' | B' by real bin
    static_assert(HALVES * SB <= dev::kPairXbuf, "staging fits the transpose buffer");
    using Tw = std::conditional_t<L == 64, dev::Pair15Tw, dev::Pair15hTw>;
    static __device__ __forceinline__ void tw_load(Tw& tw, const float* g, int hl) {
        if constexpr (L == 64)
            dev::pair15_tw_load(tw, reinterpret_cast<const dev::pc*>(g), hl);
        else
            dev::pair15h_tw_load(tw, reinterpret_cast<const dev::pc*>(g), hl);
    }
    static __device__ __forceinline__ void fwd(dev::pc (&v)[16], dev::pc* buf, const Tw& tw, int lane) {
        if constexpr (L == 64)
            dev::pair15_fwd(v, buf, tw, lane);
        else
            dev::pair15h_fwd(v, buf, tw, lane);
    }
    static __device__ __forceinline__ void inv(dev::pc (&v)[16], dev::pc* buf, const Tw& tw, int lane) {
        if constexpr (L == 64)
            dev::pair15_inv(v, buf, tw, lane);
        else
            dev::pair15h_inv(v, buf, tw, lane);
    }
    static __device__ __forceinline__ int bin(int lane, int d) {
        return L == 64 ? dev::pair15_bin(lane, d) : dev::pair15h_bin(lane, d);
    }
    static __device__ __forceinline__ int k1(int h) { return L == 64 ? (h & 3) + 4 * (h >> 4) : (h & 7) + 8 * (h >> 4); }
    // the half-lane holding the partners of half-lane h's bins (register 15 - d;
    // half-lane 0 uses its own registers (16 - d) mod 16 instead)
    static __device__ __forceinline__ int partner(int h) {
        const int a = k1(h);
        if (a == 15) return h;  // (the zero row: no bins)
        if constexpr (L == 64) {
            const int j = (h >> 2) & 3;
            if (a == 0) return j == 0 ? 0 : 4 * (4 - j);
            const int kp = 15 - a;
            return (kp & 3) + 4 * (3 - j) + 16 * (kp >> 2);
        } else {
            if (a == 0) return h;
            const int c = (h >> 3) & 1, kp = 15 - a;
            return (kp & 7) + 8 * (1 - c) + 16 * (kp >> 3);
        }
    }
};

// LDS: per wave the transpose buffer (also the staging between transforms), then
// per walk the OLA ring (synthesis kernels): the next power of two >= H ceil(N/H)
// floats, so a position wraps with one AND
__host__ __device__ inline int q15_ring(int n, int h) {
    const int span = h * ((n + h - 1) / h);
    int r = 1;
    while (r < span) r <<= 1;
    return r;
}
struct Q15Lds {
    static constexpr size_t bufs = sizeof(dev::pc) * dev::kPairXbuf * kQW;
    static size_t bytes(int n, int h, bool ring) {
        return bufs + (ring ? sizeof(float) * q15_ring(n, h) * kQW * (n == 480 ? 2 : 1) : 0);
    }
};

// (takes the value as a scalar: a bit cast applied to an ext_vector element
// directly is miscompiled by this clang)
__device__ __forceinline__ float q_bperm(int src_lane, float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src_lane * 4, __builtin_bit_cast(int, v)));
}

// The walk of one wave: unit u = (stream group, chunk); at N = 480 half h walks
// stream u * 2 + h (a missing second stream reads zeros and stores nothing).
template <int L>
struct Q15Walk {
    int s0, s, f0, f1, fs, xo, yo;
    bool have;  // this half's stream exists
};
template <int L>
__device__ __forceinline__ bool q15_walk(const FusedArgs& a, int gw, int NB, int half, Q15Walk<L>& w) {
    constexpr int HALVES = Q15<L>::HALVES;
    const int units = (a.n_streams + HALVES - 1) / HALVES;
    if (gw >= units * a.n_chunks) return false;
    const int u = gw / a.n_chunks, c = gw - u * a.n_chunks;
    w.s0 = u * HALVES;
    w.s = w.s0 + half;
    w.have = w.s < a.n_streams;
    if (!w.have) w.s = w.s0;  // (row pointers stay in range; nothing is stored)
    w.f0 = c * a.M;
    w.f1 = min(a.F, w.f0 + a.M);
    w.fs = max(0, w.f0 - (NB - 1)) & ~1;  // pairs start on even frames
    w.xo = half * int(a.ld_x);             // < 2^27 (host-checked)
    w.yo = half * int(a.ld_y);
    return true;
}
// one descriptor over the wave's streams (the half's stream is an offset)
template <int L>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t q15_rsrc(const float* base, int s0, int64_t ld, int len,
                                                          int n_streams) {
    const bool full = Q15<L>::HALVES == 2 && s0 + 1 < n_streams;
    return dev::make_rsrc(base + int64_t(s0) * ld, uint32_t((full ? int(ld) + len : len) * 4));
}

// frame at `origin`: x[origin + h + L m] of the half's stream (offset xo), the
// plan's padding outside [0, T) (Indexing.h:18-68 via FrameQueue; zeros for the Framer)
template <int L>
__device__ __forceinline__ void q15_load(float (&f)[kQE], __amdgpu_buffer_rsrc_t rx, int hl, int xo, int origin,
                                         int T, int mode) {
    if (origin >= 0 && origin + 15 * L <= T) {  // (uniform: both halves share k and T)
#pragma unroll
        for (int m = 0; m < kQE; ++m) f[m] = dev::bload1(rx, (xo + origin + hl) * 4 + m * (4 * L), 0);
    } else {
#pragma unroll
        for (int m = 0; m < kQE; ++m) {
            int j = origin + hl + L * m;
            if (mode == 1) j = reflect101(j, T);
            else if (mode == 2) j = j < 0 ? 0 : (j >= T ? T - 1 : j);
            const bool ok = j >= 0 && j < T;
            const float v = dev::bload1(rx, (xo + (ok ? j : 0)) * 4, 0);
            f[m] = ok ? v : 0.0f;
        }
    }
}
// true when every sample of the frame (whole wave) is 0 or in [lo, hi]
__device__ __forceinline__ bool q15_ok(const float (&f)[kQE], float lo, float hi) {
    bool bad = false;
#pragma unroll
    for (int m = 0; m < kQE; ++m) {
        const float t = __builtin_fabsf(f[m]);
        bad |= !((t >= lo) & (t <= hi)) & (t != 0.0f);
    }
    return __builtin_amdgcn_ballot_w64(bad) == 0;
}
// Z[-k] of registers d = 0 .. 15 (the partner half-lane's register 15 - d; half-lane 0: its own (16 - d) mod 16)
__device__ __forceinline__ void q15_partners(const dev::pc (&v)[16], dev::pc (&zp)[16], bool self, int partner_lane) {
#pragma unroll
    for (int d = 0; d < 16; ++d) {
        const float px = v[(15 - d) & 15].x, py = v[(15 - d) & 15].y;
        const float ox = v[(16 - d) & 15].x, oy = v[(16 - d) & 15].y;
        zp[d] = dev::pc_mk(q_bperm(partner_lane, px), q_bperm(partner_lane, py));
        if (self) zp[d] = dev::pc_mk(ox, oy);
    }
}

// The per-walk OLA ring: push frame k (o = sanit(v / N), fma(o, ws g, ring) in
// ascending k), produce block k (ring / den, clear; stored when k >= f0).
template <int L>
struct Q15Ola {
    float* ring;
    int H, RM, ring_blocks, f0, yo, hl;
    const float* den;
    __amdgpu_buffer_rsrc_t ry, ry_null, rd;  // (rd: den, ring_blocks H floats)
    __device__ __forceinline__ void clear() {
        for (int i = hl; i <= RM; i += L) ring[i] = 0.0f;
        dev::wave_lds_fence();
    }
    template <bool IMAG>
    __device__ __forceinline__ void push(const dev::pc (&v)[16], const float (&wsg)[kQE], float inv_n, int k) {
        const int base = k * H + hl;  // k H < 2^27 (host-checked)
#pragma unroll
        for (int m = 0; m < kQE; ++m) {
            const int pos = (base + L * m) & RM;
            const float o = dev::sanit((IMAG ? v[m].y : v[m].x) * inv_n);
            ring[pos] = __builtin_fmaf(o, wsg[m], ring[pos]);
        }
        dev::wave_lds_fence();
    }
    __device__ __forceinline__ void produce(int k) {
        const int base = k * H;
        const float* dk = den + (k % ring_blocks) * H;
        const __amdgpu_buffer_rsrc_t rk = k >= f0 ? ry : ry_null;
        for (int j = hl; j < H; j += L) {
            const int pos = (base + j) & RM;
            const float s = ring[pos];
            ring[pos] = 0.0f;
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, s / dk[j]), rk, (yo + base + j) * 4, 0,
                                                  0);
        }
        dev::wave_lds_fence();
    }
    // H <= 4 L: a block is at most 4 rows of the walk; its divisors are fetched
    // before the pushes (a divisor load waits on every earlier store too: one
    // vmcnt counter), as K_pair15's DPRE form does
    __device__ __forceinline__ void den4(int k, float (&d)[4]) const {
        const int dbase = (k % ring_blocks) * H;
#pragma unroll
        for (int i = 0; i < 4; ++i) d[i] = dev::bload1(rd, (hl + L * i) * 4, dbase * 4);  // (past the table: 0, unused)
    }
    __device__ __forceinline__ void produce4(int k, const float (&d)[4]) {
        const int base = k * H;
        const __amdgpu_buffer_rsrc_t rk = k >= f0 ? ry : ry_null;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int j = hl + L * i;
            if (j < H) {
                const int pos = (base + j) & RM;
                const float s = ring[pos];
                ring[pos] = 0.0f;
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, s / d[i]), rk, (yo + base + j) * 4,
                                                      0, 0);
            }
        }
        dev::wave_lds_fence();
    }
    // a pair's two frames: push k, produce k, push k+1, produce k+1 (when k+1 < f1)
    template <bool PRE>
    __device__ __forceinline__ void pair(const dev::pc (&v)[16], const float (&wsg)[kQE], float inv_n, int k, int f1) {
        if (PRE && H <= 4 * L) {
            float d0[4], d1[4];
            den4(k, d0);
            den4(k + 1, d1);
            push<false>(v, wsg, inv_n, k);
            produce4(k, d0);
            push<true>(v, wsg, inv_n, k + 1);
            if (k + 1 < f1) produce4(k + 1, d1);
        } else {
            push<false>(v, wsg, inv_n, k);
            produce(k);
            push<true>(v, wsg, inv_n, k + 1);
            if (k + 1 < f1) produce(k + 1);
        }
    }
};
template <int L>
__device__ __forceinline__ void q15_ola_init(Q15Ola<L>& o, const FusedArgs& a, char* smem, const Q15Walk<L>& w,
                                             int wave, int half, int hl) {
    const int H = a.hop, RL = q15_ring(15 * L, H);
    o.ring = reinterpret_cast<float*>(smem + Q15Lds::bufs) + (wave * Q15<L>::HALVES + half) * RL;
    o.H = H;
    o.RM = RL - 1;
    o.ring_blocks = a.ring_blocks;
    o.f0 = w.f0;
    o.yo = w.yo;
    o.hl = hl;
    o.den = a.t.den;
    o.rd = dev::make_rsrc(a.t.den, uint32_t(a.ring_blocks * H) * 4u);
    o.ry = q15_rsrc<L>(a.y, w.s0, a.ld_y, a.out_len, a.n_streams);
    o.ry_null = dev::make_rsrc(a.y, 0u);
    o.clear();
}

// ------------------------------------------------------------------ K_pair_stft
template <int L>
__global__ __launch_bounds__(64 * kQW, 2) void k_p15_stft(const PairSpecArgs pa) {
    using G = Q15<L>;
    const FusedArgs& a = pa.f;
    constexpr int E = kQE, P2 = G::P2;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, hl = lane % L, half = lane / L;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    dev::pc* buf = reinterpret_cast<dev::pc*>(smem) + wave * dev::kPairXbuf;
    Q15Walk<L> w;
    if (!q15_walk<L>(a, blockIdx.x * kQW + wave, 1, half, w)) return;
    const int H = a.hop;
    const __amdgpu_buffer_rsrc_t rx = q15_rsrc<L>(a.x, w.s0, a.ld_x, a.T, a.n_streams);
    float* so = pa.spec + int64_t(w.s) * pa.ld_spec;
    typename G::Tw tw;
    G::tw_load(tw, a.t.ptw, hl);
    float wa[E];
#pragma unroll
    for (int m = 0; m < E; ++m) wa[m] = a.t.wa[hl + L * m];
    const bool live = G::k1(hl) != 15, store = live && w.have;
    const int partner_lane = G::partner(hl) + L * half;
    const float xlo = a.t.px_lo, xhi = a.t.px_hi;
    float fa[E], fb[E];
    auto load = [&](float (&f)[E], int k) { q15_load<L>(f, rx, hl, w.xo, k * H - a.pad, a.T, a.pad_mode); };
    load(fa, w.f0);
    load(fb, w.f0 + 1);
    // bins k <= N/2 of this lane: registers d < 8 (bin lanes), d = 8 in half-lane 0 (k = N/2)
    auto store_bins = [&](float* row, auto valfn) {
        float2* r2 = reinterpret_cast<float2*>(row);
#pragma unroll
        for (int d = 0; d < 8; ++d) {
            const dev::pc o = valfn(d);
            if (store) r2[G::bin(lane, d)] = make_float2(o.x, o.y);
        }
        if (hl == 0 && w.have) {
            const dev::pc o = valfn(8);
            r2[P2] = make_float2(o.x, o.y);
        }
    };
    for (int k = w.f0; k < w.f1; k += 2) {  // (M even: chunks start on even frames)
        const bool two = k + 1 < w.f1;
        float* ra = so + int64_t(k) * pa.ld_frame;
        float* rb = ra + pa.ld_frame;
        const bool paired = q15_ok(fa, xlo, xhi) && q15_ok(fb, xlo, xhi);
        dev::pc v[16];
        if (paired) {
#pragma unroll
            for (int m = 0; m < E; ++m) v[m] = dev::pc_mk(fa[m] * wa[m], fb[m] * wa[m]);
            v[15] = dev::pc_mk(0.0f, 0.0f);
            load(fa, k + 2);  // (in flight during the transform)
            load(fb, k + 3);
            dev::wave_lds_fence();
            G::fwd(v, buf, tw, lane);
            dev::pc zp[16];
            q15_partners(v, zp, hl == 0, partner_lane);
            store_bins(ra, [&](int d) {
                return dev::pc_mk(0.5f * (v[d].x + zp[d].x), 0.5f * (v[d].y - zp[d].y));
            });
            if (two)
                store_bins(rb, [&](int d) {
                    return dev::pc_mk(0.5f * (v[d].y + zp[d].y), 0.5f * (zp[d].x - v[d].x));
                });
        } else {  // each frame alone, full input sanitize
            auto pass = [&](const float (&f)[E], float* row) {
#pragma unroll
                for (int m = 0; m < E; ++m) v[m] = dev::pc_mk(dev::sanit(f[m] * wa[m]), 0.0f);
                v[15] = dev::pc_mk(0.0f, 0.0f);
                dev::wave_lds_fence();
                G::fwd(v, buf, tw, lane);
                store_bins(row, [&](int d) {  // (DC and Nyquist: imaginary part exactly 0, as kiss_fftr writes them)
                    return dev::pc_mk(v[d].x, (hl == 0 && (d == 0 || d == 8)) ? 0.0f : v[d].y);
                });
            };
            pass(fa, ra);
            if (two) pass(fb, rb);
            load(fa, k + 2);
            load(fb, k + 3);
        }
    }
}

// ------------------------------------------------------------------ K_pair_istft
// PF: the next pair's rows and both blocks' divisors fetched ahead (H <= 4 L;
// 2 waves/SIMD: +16 % at 960/240 in an interleaved A/B), else at use (3 waves/SIMD
// where the registers allow: +9 % at 960/480)
template <int L, bool MASK, bool PF>
__global__ __launch_bounds__(64 * kQW, 2) void k_p15_istft(const PairSpecArgs pa) {
    using G = Q15<L>;
    const FusedArgs& a = pa.f;
    constexpr int N = G::N, E = kQE, P2 = G::P2, OB = P2 + 1, MI = 8;
    static_assert(MI * L > P2, "rows");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, hl = lane % L, half = lane / L;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    dev::pc* buf = reinterpret_cast<dev::pc*>(smem) + wave * dev::kPairXbuf;
    dev::pc* sbuf = buf + half * G::SB;  // this half's staging
    const int H = a.hop, NB = (N + H - 1) / H;
    Q15Walk<L> w;
    if (!q15_walk<L>(a, blockIdx.x * kQW + wave, NB, half, w)) return;
    Q15Ola<L> ola;
    q15_ola_init<L>(ola, a, smem, w, wave, half, hl);
    typename G::Tw tw;
    G::tw_load(tw, a.t.ptw, hl);
    float wsg[E];
#pragma unroll
    for (int m = 0; m < E; ++m) wsg[m] = a.t.ws[hl + L * m] * a.gain;
    const bool live = G::k1(hl) != 15;
    const float* sb = pa.sin + int64_t(w.s) * pa.ld_spec;
    const float* mrow0 = MASK ? pa.mask.p + int64_t(w.s) * pa.mask.ld_stream : nullptr;
    // the pair's rows (and mask rows) by real bin kr = h + L i <= N/2, coalesced;
    // stepped -- (X g) m, re and im each; DC and Nyquist imaginary parts dropped --
    // and staged at sbuf[kr] (frame k) and sbuf[OB + kr] (frame k+1, zeros past the last)
    float2 ra_[MI], rb_[MI];
    float ma_[MASK ? MI : 1], mb_[MASK ? MI : 1];
    auto load_rows = [&](int k) {
        const float2* ra = reinterpret_cast<const float2*>(sb + int64_t(k) * pa.ld_frame);
        const float2* rb = reinterpret_cast<const float2*>(sb + int64_t(k + 1) * pa.ld_frame);
        const bool two = k + 1 < a.F;
        const float* m0 = MASK ? mrow0 + int64_t(k) * pa.mask.ld_frame : nullptr;
        const float* m1 = MASK && two ? m0 + pa.mask.ld_frame : m0;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            const int kr = hl + L * i;
            const bool on = kr <= P2;
            ra_[i] = on ? ra[kr] : make_float2(0.f, 0.f);
            rb_[i] = on && two ? rb[kr] : make_float2(0.f, 0.f);
            if constexpr (MASK) {
                ma_[i] = on ? m0[kr] : 0.f;
                mb_[i] = on ? m1[kr] : 0.f;
            }
        }
    };
    auto stage = [&]() -> bool {
        bool bad = false;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            const int kr = hl + L * i;
            if (kr <= P2) {
                const float g = a.t.gain ? a.t.gain[kr] : 1.0f;
                float ax = ra_[i].x * g, ay = ra_[i].y * g, bx = rb_[i].x * g, by = rb_[i].y * g;
                if constexpr (MASK) {
                    ax *= ma_[i];
                    ay *= ma_[i];
                    bx *= mb_[i];
                    by *= mb_[i];
                }
                if (kr == 0 || kr == P2) ay = by = 0.0f;
                const float mx = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(ax), __builtin_fabsf(ay)),
                                                 __builtin_fmaxf(__builtin_fabsf(bx), __builtin_fabsf(by)));
                bad |= !(mx <= 0x1p60f) | (ax != ax) | (ay != ay) | (bx != bx) | (by != by);  // (NaN, Inf, huge)
                sbuf[kr] = dev::pc_mk(ax, ay);
                sbuf[OB + kr] = dev::pc_mk(bx, by);
            }
        }
        dev::wave_lds_fence();
        return __builtin_amdgcn_ballot_w64(bad) == 0;
    };
    // bin kb of (lane, d): real bin kb (kb <= N/2) or N - kb conjugated; the zero row stays 0
    auto gather = [&](dev::pc (&v)[16], bool pair_form, int off) {
#pragma unroll
        for (int d = 0; d < 16; ++d) {
            const int kb = G::bin(lane, d);
            const bool lo = kb <= P2;
            const int j = lo ? kb : N - kb;
            const dev::pc A = sbuf[off + (live ? j : 0)];
            if (pair_form) {
                const dev::pc B = sbuf[OB + (live ? j : 0)];
                v[d] = lo ? dev::pc_mk(A.x - B.y, A.y + B.x) : dev::pc_mk(A.x + B.y, B.x - A.y);
            } else {
                v[d] = lo ? A : dev::pc_mk(A.x, -A.y);
            }
            if (!live) v[d] = dev::pc_mk(0.0f, 0.0f);
        }
        dev::wave_lds_fence();  // (the reads before the inverse's transpose rewrites buf)
    };
    if (PF) load_rows(w.fs);
    for (int k = w.fs; k < w.f1; k += 2) {
        dev::pc v[16];
        const bool more = k + 2 < w.f1;
        if (!PF) load_rows(k);
        if (stage()) {
            gather(v, true, 0);
            G::inv(v, buf, tw, lane);
            if (PF && more) load_rows(k + 2);  // (in flight during the OLA stage)
            ola.template pair<PF>(v, wsg, a.inv_n, k, w.f1);
        } else {  // each frame alone, full sanitize (staged again for frame k+1: the inverse used buf)
            gather(v, false, 0);
            G::inv(v, buf, tw, lane);
            ola.template push<false>(v, wsg, a.inv_n, k);
            ola.produce(k);
            if (k + 1 < w.f1) {
                (void)stage();
                gather(v, false, OB);
                G::inv(v, buf, tw, lane);
                ola.template push<false>(v, wsg, a.inv_n, k + 1);
                ola.produce(k + 1);
            }
            if (PF && more) load_rows(k + 2);
        }
    }
}

// ------------------------------------------------------------------ K_pair_mask
template <int L>
__global__ __launch_bounds__(64 * kQW, 2) void k_p15_mask(const PairSpecArgs pa) {
    using G = Q15<L>;
    const FusedArgs& a = pa.f;
    constexpr int N = G::N, E = kQE, P2 = G::P2, MI = 8;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, hl = lane % L, half = lane / L;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    dev::pc* buf = reinterpret_cast<dev::pc*>(smem) + wave * dev::kPairXbuf;
    dev::pc* cbuf = buf + half * G::SB;  // this half's (c1, c2) by real bin
    const int H = a.hop, NB = (N + H - 1) / H;
    Q15Walk<L> w;
    if (!q15_walk<L>(a, blockIdx.x * kQW + wave, NB, half, w)) return;
    Q15Ola<L> ola;
    q15_ola_init<L>(ola, a, smem, w, wave, half, hl);
    const __amdgpu_buffer_rsrc_t rx = q15_rsrc<L>(a.x, w.s0, a.ld_x, a.T, a.n_streams);
    typename G::Tw tw;
    G::tw_load(tw, a.t.ptw, hl);
    // (at N = 480 the analysis window is read from L2 at each pair: in registers it spills)
    constexpr bool WREG = L == 64;
    float war[WREG ? E : 1], wsg[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        if constexpr (WREG) war[m] = a.t.wa[hl + L * m];
        wsg[m] = a.t.ws[hl + L * m] * a.gain;
    }
    auto wa = [&](int m) { return WREG ? war[WREG ? m : 0] : a.t.wa[hl + L * m]; };
    const bool live = G::k1(hl) != 15;
    const int partner_lane = G::partner(hl) + L * half;
    const float xlo = a.t.px_lo, xhi = a.t.px_hi * 0x1p-20f;  // (mask values up to 2^20)
    const float* mrow0 = pa.mask.p + int64_t(w.s) * pa.mask.ld_stream;
    auto row_a = [&](int k) { return mrow0 + int64_t(k) * pa.mask.ld_frame; };
    auto row_b = [&](int k) { return k + 1 < a.F ? row_a(k) + pa.mask.ld_frame : row_a(k); };  // (past F: unused)
    float ma[MI], mb[MI];  // the pair's mask rows by real bin h + L i (<= N/2; 1 beyond)
    auto load_rows = [&](int k) {
        const float* r0 = row_a(k);
        const float* r1 = row_b(k);
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            const int kr = hl + L * i;
            ma[i] = kr <= P2 ? r0[kr] : 1.0f;
            mb[i] = kr <= P2 ? r1[kr] : 1.0f;
        }
    };
    auto rows_ok = [&]() {
        bool bad = false;
#pragma unroll
        for (int i = 0; i < MI; ++i)
            bad |= !(__builtin_fabsf(ma[i]) <= 0x1p20f) | !(__builtin_fabsf(mb[i]) <= 0x1p20f);  // (NaN too)
        return __builtin_amdgcn_ballot_w64(bad) == 0;
    };
    float fa[E], fb[E];
    auto load = [&](float (&f)[E], int k) { q15_load<L>(f, rx, hl, w.xo, k * H - a.pad, a.T, a.pad_mode); };
    load(fa, w.fs);
    load(fb, w.fs + 1);
    load_rows(w.fs);
    for (int k = w.fs; k < w.f1; k += 2) {
        const bool paired = q15_ok(fa, xlo, xhi) && q15_ok(fb, xlo, xhi) && rows_ok();
        const bool partner_frame = k + 1 < a.F;  // frame k+1 past the last: imaginary part 0
        dev::pc v[16];
        if (paired) {
#pragma unroll
            for (int m = 0; m < E; ++m) {
                const float wv = wa(m);
                v[m] = dev::pc_mk(fa[m] * wv, partner_frame ? fb[m] * wv : 0.0f);
            }
            v[15] = dev::pc_mk(0.0f, 0.0f);
            load(fa, k + 2);  // (in flight during the transforms)
            load(fb, k + 3);
            dev::wave_lds_fence();
            G::fwd(v, buf, tw, lane);
            // (c1, c2) by real bin in the (now free) transpose buffer
#pragma unroll
            for (int i = 0; i < MI; ++i) {
                const int kr = hl + L * i;
                if (kr <= P2) {
                    const float g = a.t.gain ? a.t.gain[kr] : 1.0f;
                    const float ga = g * ma[i], gb = g * mb[i];
                    cbuf[kr] = dev::pc_mk(0.5f * (ga + gb), 0.5f * (ga - gb));
                }
            }
            if (k + 2 < w.f1) load_rows(k + 2);
            dev::wave_lds_fence();
            dev::pc zp[16];
            q15_partners(v, zp, hl == 0, partner_lane);
#pragma unroll
            for (int d = 0; d < 16; ++d) {
                const int kb = G::bin(lane, d);
                const dev::pc cc = cbuf[live ? (kb <= P2 ? kb : N - kb) : 0];
                v[d] = live ? dev::pc_mk(__builtin_fmaf(cc.y, zp[d].x, cc.x * v[d].x),
                                         __builtin_fmaf(-cc.y, zp[d].y, cc.x * v[d].y))
                            : dev::pc_mk(0.0f, 0.0f);
            }
            dev::wave_lds_fence();  // (the coefficient reads before the inverse's transpose rewrites buf)
            G::inv(v, buf, tw, lane);
            ola.template pair<false>(v, wsg, a.inv_n, k, w.f1);  // (the divisors fetched ahead would spill here)
        } else {  // each frame alone, full sanitize, its own gain g m (rows from L2, scrambled)
            auto pass = [&](const float (&f)[E], const float* r, int kk) {
#pragma unroll
                for (int m = 0; m < E; ++m) v[m] = dev::pc_mk(dev::sanit(f[m] * wa(m)), 0.0f);
                v[15] = dev::pc_mk(0.0f, 0.0f);
                dev::wave_lds_fence();
                G::fwd(v, buf, tw, lane);
#pragma unroll
                for (int d = 0; d < 16; ++d) {
                    const int kb = G::bin(lane, d), kr = live ? (kb <= P2 ? kb : N - kb) : 0;
                    v[d] = live ? v[d] * ((a.t.gain ? a.t.gain[kr] : 1.0f) * r[kr]) : dev::pc_mk(0.0f, 0.0f);
                }
                G::inv(v, buf, tw, lane);
                ola.template push<false>(v, wsg, a.inv_n, kk);
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

template <typename K>
hipError_t q15_launch(K kernel, const PairSpecArgs& a, int n, int64_t waves, int32_t kind, bool ring,
                      hipStream_t stream) {
    const size_t lds = Q15Lds::bytes(n, a.f.hop, ring);
    hipError_t e = set_lds(kernel, lds);
    if (e != hipSuccess) return e;
    const int64_t grid = (waves + kQW - 1) / kQW;
    note_launch(kind, grid);
    hipLaunchKernelGGL(kernel, dim3(unsigned(grid)), dim3(64 * kQW), lds, stream, a);
    return hipGetLastError();
}

// chunks: about two resident rounds of walks, each >= `min_m` frames, an even
// length; returns the waves to launch (stream units x chunks)
int64_t q15_chunks(FusedArgs& f, int n, int64_t F, int n_streams, int64_t min_m) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    const int halves = n == 480 ? 2 : 1;
    const int64_t units = std::max(1, (n_streams + halves - 1) / halves);
    const int64_t resident = int64_t(cus) * 2 * kQW;
    int64_t c = std::max<int64_t>(1, std::min<int64_t>(F / min_m, (2 * resident + units - 1) / units));
    c = chunks_or(c, F);
    int64_t m = (F + c - 1) / c;
    m += m & 1;
    f.M = int(m);
    f.n_chunks = int((F + m - 1) / m);
    note_chunks(f.n_chunks);
    return units * f.n_chunks;
}

}  // namespace

}  // namespace fk

bool pair15_spec_supported(int n, int h, int ring_len) {
    return (n == 960 || n == 480) && h >= 32 && h <= n && ring_len % h == 0;
}

// leading dimensions and lengths the 32-bit buffer offsets of the pair walks cover
// (at N = 480 one descriptor spans two streams)
bool pair15_spec_fits(int n, int64_t ld, int64_t len) {
    return len < (int64_t(1) << 27) && (n != 480 || ld < (int64_t(1) << 27));
}

// crlot_stft at N = 960 / 480 as frame pairs
hipError_t launch_pair15_stft(const Geometry& g, const DevTables& t, const float* x, int n_streams, int64_t T,
                              int64_t ld_x, int64_t F, float* spec, int64_t ld_spec, int64_t ld_frame,
                              hipStream_t stream) {
    if (!pair15_spec_supported(g.n, g.h, g.ring_len) || F <= 0 || n_streams <= 0 || !t.ptw || !t.wa ||
        !pair15_spec_fits(g.n, ld_x, T))
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
    const int64_t waves = fk::q15_chunks(a.f, g.n, F, n_streams, 32);
    return g.n == 960 ? fk::q15_launch(fk::k_p15_stft<64>, a, g.n, waves, CRLOT_K_PAIR_STFT, false, stream)
                      : fk::q15_launch(fk::k_p15_stft<32>, a, g.n, waves, CRLOT_K_PAIR_STFT, false, stream);
}

// crlot_istft_ola at N = 960 / 480 as frame pairs (the plan's mask, if any, applied)
hipError_t launch_pair15_istft(const Geometry& g, const DevTables& t, const SpecMask& m, const float* spec,
                               int64_t ld_spec, int64_t ld_frame, float* y, int n_streams, int64_t F, int64_t ld_y,
                               hipStream_t stream) {
    if (!pair15_spec_supported(g.n, g.h, g.ring_len) || F <= 0 || n_streams <= 0 || !t.ptw || !t.ws || !t.den ||
        !pair15_spec_fits(g.n, ld_y, F * g.h + g.n))
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
    const int64_t waves = fk::q15_chunks(a.f, g.n, F, n_streams, 48);
    const int32_t K = CRLOT_K_PAIR_ISTFT;
    if (g.n == 480)
        return m.p ? fk::q15_launch(fk::k_p15_istft<32, true, false>, a, g.n, waves, K, true, stream)
                   : fk::q15_launch(fk::k_p15_istft<32, false, false>, a, g.n, waves, K, true, stream);
    if (g.h <= 256)
        return m.p ? fk::q15_launch(fk::k_p15_istft<64, true, true>, a, g.n, waves, K, true, stream)
                   : fk::q15_launch(fk::k_p15_istft<64, false, true>, a, g.n, waves, K, true, stream);
    return m.p ? fk::q15_launch(fk::k_p15_istft<64, true, false>, a, g.n, waves, K, true, stream)
               : fk::q15_launch(fk::k_p15_istft<64, false, false>, a, g.n, waves, K, true, stream);
}

// crlot_roundtrip at N = 960 / 480 with a per-frame mask, one walk
hipError_t launch_pair15_masked(const Geometry& g, const DevTables& t, const SpecMask& m, const float* x, float* y,
                                int n_streams, int64_t T, int64_t ld_x, int64_t ld_y, int64_t F, int64_t out_len,
                                hipStream_t stream) {
    if (!pair15_spec_supported(g.n, g.h, g.ring_len) || F <= 0 || n_streams <= 0 || !m.p || !t.ptw || !t.wa ||
        !t.ws || !t.den || !pair15_spec_fits(g.n, ld_x, T) || !pair15_spec_fits(g.n, ld_y, out_len + g.n))
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
    const int64_t waves = fk::q15_chunks(a.f, g.n, F, n_streams, 48);
    return g.n == 960 ? fk::q15_launch(fk::k_p15_mask<64>, a, g.n, waves, CRLOT_K_PAIR_MASK, true, stream)
                      : fk::q15_launch(fk::k_p15_mask<32>, a, g.n, waves, CRLOT_K_PAIR_MASK, true, stream);
}

}  // namespace crlot
