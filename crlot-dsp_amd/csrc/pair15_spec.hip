// pair15_spec.hip -- the spectral entries and the masked round trip as frame
// pairs at N = 960 (20 ms at 48 kHz), any hop H >= 32 whose ring the plan allows:
//   K_pair_stft   k_p15_stft        (crlot_stft)
//   K_pair_istft  k_p15_istft<MASK> (crlot_istft_ola)
//   K_pair_mask   k_p15_mask        (crlot_roundtrip with a per-frame mask)
// on K_pair15's transform (fft_pair15.h: Good-Thomas 15 over the registers, then
// K_pair's 64-lane stage), one walk per wave, frames loaded whole (H is not a
// lane multiple) and the overlap-add in a per-wave LDS ring, as K_pair15
// (pair_any.hip).
//
// Bin k = k1 + 15 k' sits in lane l, register d with k1 = (l & 3) + 4 (l >> 4)
// and k' = ((l >> 2) & 3) + 4 d (pair15_bin; k1 = 15 is the zero row: lanes 51,
// 55, 59, 63 hold no bins).  Its partner N - k is register 15 - d of lane
// p15_partner(l) (k1 -> 15 - k1, bits 2-3 -> 3 - j; for k1 = 0, j -> 4 - j),
// except in lane 0 (k = 15 * 4 d), whose partners are its own registers
// (16 - d) mod 16 -- the map tests/test_pair_bin_maps.py checks exhaustively.
// The real bins 0 .. N/2 are registers d < 8 of the other lanes plus register 8
// of lane 0 (bin 480), as at N = 1024, so the split / merge / step code is
// pair_stft.hip's and pair_mask.hip's with this map:
//   stft:  A[k] = (Z[k] + conj Z[-k]) / 2, B[k] = (Z[k] - conj Z[-k]) / 2i;
//   istft: the stepped rows staged by real bin in the wave's transpose buffer,
//          read back scrambled as Z = A' + i B';
//   mask:  Z' = c1 Z + c2 conj Z[-k], c1 = (Ga + Gb) / 2, c2 = (Ga - Gb) / 2.
// Regimes per pair, wave-uniform (one transform per wave): the pair when its
// samples keep px_lo <= |x| <= px_hi (/ 2^20 with a mask, whose values must be
// finite and within 2^20) and its stepped spectra are finite and below 2^60;
// otherwise each frame alone with the full sanitize.  The inverse output is
// scaled and sanitized as kissfft_adapter.cc:154-163 does (o = sanit(v / N)) and
// pushed with fma(o, ws g, ring); produce divides by the plan's den (IEEE; the
// divisors of both blocks fetched ahead when H <= 256).
// Results equal the per-frame kissfft formulation within float32 rounding.
#include <algorithm>
#include <type_traits>

#include "fft_pair15.h"
#include "fused_common.h"

namespace crlot {
namespace fk {

namespace {

constexpr int kQW = 4;     // walks (waves) per workgroup
constexpr int kQN = 960;   // frame size
constexpr int kQE = 15;    // samples per lane per frame
constexpr int kQP2 = 480;  // N / 2

// LDS: per wave the transpose buffer (also the staging between transforms), then
// per wave the OLA ring (synthesis kernels): the next power of two >= H ceil(N/H)
// floats (<= 2048), so a position wraps with one AND
__host__ __device__ inline int q15_ring(int h) {
    const int span = h * ((kQN + h - 1) / h);
    int r = 1;
    while (r < span) r <<= 1;
    return r;
}
struct Q15Lds {
    static constexpr size_t bufs = sizeof(dev::pc) * dev::kPairXbuf * kQW;
    static size_t bytes(int h, bool ring) { return bufs + (ring ? sizeof(float) * q15_ring(h) * kQW : 0); }
};
static_assert(2 * (kQP2 + 1) <= dev::kPairXbuf, "A' | B' staged in the transpose buffer");
__device__ __forceinline__ int q15_k1(int l) { return (l & 3) + 4 * (l >> 4); }
__device__ __forceinline__ int q15_partner(int l) {
    const int k1 = q15_k1(l), j = (l >> 2) & 3;
    if (k1 == 15) return l;  // (the zero row: no bins)
    if (k1 == 0) return j == 0 ? 0 : 4 * (4 - j);
    const int kp = 15 - k1;
    return (kp & 3) + 4 * (3 - j) + 16 * (kp >> 2);
}
// (both take the value as a scalar: a bit cast applied to an ext_vector element
// directly is miscompiled by this clang)
__device__ __forceinline__ float q_bperm(int src_lane, float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src_lane * 4, __builtin_bit_cast(int, v)));
}
__device__ __forceinline__ float q_lane0(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
}

// frame at `origin`: x[origin + lane + 64 m], the plan's padding outside [0, T)
__device__ __forceinline__ void q15_load(float (&f)[kQE], __amdgpu_buffer_rsrc_t rx, int lane, int origin, int T,
                                         int mode) {
    if (origin >= 0 && origin + kQN <= T) {
#pragma unroll
        for (int m = 0; m < kQE; ++m) f[m] = dev::bload1(rx, (origin + lane) * 4 + m * 256, 0);
    } else {
#pragma unroll
        for (int m = 0; m < kQE; ++m) f[m] = fetch_x(rx, origin + lane + 64 * m, T, mode);
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
// Z[-k] of registers d = 0 .. 15 (partner lane's register 15 - d; lane 0: its own (16 - d) mod 16)
__device__ __forceinline__ void q15_partners(const dev::pc (&v)[16], dev::pc (&zp)[16], int lane, int partner) {
#pragma unroll
    for (int d = 0; d < 16; ++d) {
        const float px = v[(15 - d) & 15].x, py = v[(15 - d) & 15].y;
        const float ox = v[(16 - d) & 15].x, oy = v[(16 - d) & 15].y;
        zp[d] = dev::pc_mk(q_bperm(partner, px), q_bperm(partner, py));
        if (lane == 0) zp[d] = dev::pc_mk(ox, oy);
    }
}

// The per-wave OLA ring: push frame k (o = sanit(v / N), fma(o, ws g, ring) in
// ascending k), produce block k (ring / den, clear; stored when k >= f0).
struct Q15Ola {
    float* ring;
    int H, RM, ring_blocks, f0;
    const float* den;
    __amdgpu_buffer_rsrc_t ry, ry_null, rd;  // (rd: den, ring_blocks H floats)
    __device__ __forceinline__ void clear(int lane) {
        for (int i = lane; i <= RM; i += 64) ring[i] = 0.0f;
        dev::wave_lds_fence();
    }
    template <bool IMAG>
    __device__ __forceinline__ void push(const dev::pc (&v)[16], const float (&wsg)[kQE], float inv_n, int k,
                                         int lane) {
        const int base = k * H + lane;  // k H < 2^27 (host-checked)
#pragma unroll
        for (int m = 0; m < kQE; ++m) {
            const int pos = (base + 64 * m) & RM;
            const float o = dev::sanit((IMAG ? v[m].y : v[m].x) * inv_n);
            ring[pos] = __builtin_fmaf(o, wsg[m], ring[pos]);
        }
        dev::wave_lds_fence();
    }
    // H <= 256: a block is at most 4 rows of the walk; its divisors are fetched
    // before the pushes (a divisor load waits on every earlier store too: one
    // vmcnt counter), as K_pair15's DPRE form does
    __device__ __forceinline__ void den4(int k, float (&d)[4], int lane) const {
        const int dbase = (k % ring_blocks) * H;
#pragma unroll
        for (int i = 0; i < 4; ++i) d[i] = dev::bload1(rd, (lane + 64 * i) * 4, dbase * 4);  // (past the table: 0, unused)
    }
    __device__ __forceinline__ void produce4(int k, const float (&d)[4], int lane) {
        const int base = k * H;
        const __amdgpu_buffer_rsrc_t rk = k >= f0 ? ry : ry_null;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int j = lane + 64 * i;
            if (j < H) {
                const int pos = (base + j) & RM;
                const float s = ring[pos];
                ring[pos] = 0.0f;
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, s / d[i]), rk, (base + j) * 4, 0, 0);
            }
        }
        dev::wave_lds_fence();
    }
    // a pair's two frames: push k, produce k, push k+1, produce k+1 (when k+1 < f1)
    __device__ __forceinline__ void pair(const dev::pc (&v)[16], const float (&wsg)[kQE], float inv_n, int k, int f1,
                                         int lane) {
        if (H <= 256) {
            float d0[4], d1[4];
            den4(k, d0, lane);
            den4(k + 1, d1, lane);
            push<false>(v, wsg, inv_n, k, lane);
            produce4(k, d0, lane);
            push<true>(v, wsg, inv_n, k + 1, lane);
            if (k + 1 < f1) produce4(k + 1, d1, lane);
        } else {
            push<false>(v, wsg, inv_n, k, lane);
            produce(k, lane);
            push<true>(v, wsg, inv_n, k + 1, lane);
            if (k + 1 < f1) produce(k + 1, lane);
        }
    }
    __device__ __forceinline__ void produce(int k, int lane) {
        const int base = k * H;
        const float* dk = den + (k % ring_blocks) * H;
        const __amdgpu_buffer_rsrc_t rk = k >= f0 ? ry : ry_null;
        for (int j = lane; j < H; j += 64) {
            const int pos = (base + j) & RM;
            const float s = ring[pos];
            ring[pos] = 0.0f;
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, s / dk[j]), rk, (base + j) * 4, 0, 0);
        }
        dev::wave_lds_fence();
    }
};

// ------------------------------------------------------------------ K_pair_stft
__global__ __launch_bounds__(64 * kQW, 2) void k_p15_stft(const PairSpecArgs pa) {
    const FusedArgs& a = pa.f;
    constexpr int E = kQE, P2 = kQP2;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    dev::pc* buf = reinterpret_cast<dev::pc*>(smem) + wave * dev::kPairXbuf;
    const int gw = blockIdx.x * kQW + wave;
    if (gw >= a.n_streams * a.n_chunks) return;
    const int s = gw / a.n_chunks, c = gw - s * a.n_chunks;
    const int f0 = c * a.M, f1 = min(a.F, f0 + a.M);  // (M even: chunks start on even frames)
    const int H = a.hop;
    const __amdgpu_buffer_rsrc_t rx = dev::make_rsrc(a.x + int64_t(s) * a.ld_x, span_bytes(a.T, 1));
    float* so = pa.spec + int64_t(s) * pa.ld_spec;
    dev::Pair15Tw tw;
    dev::pair15_tw_load(tw, reinterpret_cast<const dev::pc*>(a.t.ptw), lane);
    float wa[E];
#pragma unroll
    for (int m = 0; m < E; ++m) wa[m] = a.t.wa[lane + 64 * m];
    const bool live = q15_k1(lane) != 15;
    const int partner = q15_partner(lane);
    const float xlo = a.t.px_lo, xhi = a.t.px_hi;
    float fa[E], fb[E];
    q15_load(fa, rx, lane, f0 * H - a.pad, a.T, a.pad_mode);
    q15_load(fb, rx, lane, (f0 + 1) * H - a.pad, a.T, a.pad_mode);
    // bins k <= N/2 of this lane: registers d < 8 (not the zero row), d = 8 in lane 0 (k = 480)
    auto store_bins = [&](float* row, auto valfn) {
        float2* r2 = reinterpret_cast<float2*>(row);
#pragma unroll
        for (int d = 0; d < 8; ++d) {
            const dev::pc o = valfn(d);
            if (live) r2[dev::pair15_bin(lane, d)] = make_float2(o.x, o.y);
        }
        if (lane == 0) {
            const dev::pc o = valfn(8);
            r2[P2] = make_float2(o.x, o.y);
        }
    };
    for (int k = f0; k < f1; k += 2) {
        const bool two = k + 1 < f1;
        float* ra = so + int64_t(k) * pa.ld_frame;
        float* rb = ra + pa.ld_frame;
        const bool paired = q15_ok(fa, xlo, xhi) && q15_ok(fb, xlo, xhi);
        dev::pc v[16];
        if (paired) {
#pragma unroll
            for (int m = 0; m < E; ++m) v[m] = dev::pc_mk(fa[m] * wa[m], fb[m] * wa[m]);
            v[15] = dev::pc_mk(0.0f, 0.0f);
            q15_load(fa, rx, lane, (k + 2) * H - a.pad, a.T, a.pad_mode);  // (in flight during the transform)
            q15_load(fb, rx, lane, (k + 3) * H - a.pad, a.T, a.pad_mode);
            dev::wave_lds_fence();
            dev::pair15_fwd(v, buf, tw, lane);
            dev::pc zp[16];
            q15_partners(v, zp, lane, partner);
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
                dev::pair15_fwd(v, buf, tw, lane);
                store_bins(row, [&](int d) {  // (DC and Nyquist: imaginary part exactly 0, as kiss_fftr writes them)
                    return dev::pc_mk(v[d].x, (lane == 0 && (d == 0 || d == 8)) ? 0.0f : v[d].y);
                });
            };
            pass(fa, ra);
            if (two) pass(fb, rb);
            q15_load(fa, rx, lane, (k + 2) * H - a.pad, a.T, a.pad_mode);
            q15_load(fb, rx, lane, (k + 3) * H - a.pad, a.T, a.pad_mode);
        }
    }
}

// Common walk state of the two synthesis kernels.
struct Q15Walk {
    int s, f0, f1, fs;
};
__device__ __forceinline__ bool q15_walk(const FusedArgs& a, int gw, int NB, Q15Walk& w) {
    if (gw >= a.n_streams * a.n_chunks) return false;
    w.s = gw / a.n_chunks;
    const int c = gw - w.s * a.n_chunks;
    w.f0 = c * a.M;
    w.f1 = min(a.F, w.f0 + a.M);
    w.fs = max(0, w.f0 - (NB - 1)) & ~1;  // pairs start on even frames
    return true;
}

// ------------------------------------------------------------------ K_pair_istft
// PF: the next pair's rows and both blocks' divisors fetched ahead (H <= 256; 180-204
// VGPRs, 2 waves/SIMD: +16 % at 960/240), else at use (3 waves/SIMD: +9 % at 960/480)
template <bool MASK, bool PF>
__global__ __launch_bounds__(64 * kQW, 2) void k_p15_istft(const PairSpecArgs pa) {
    const FusedArgs& a = pa.f;
    constexpr int N = kQN, E = kQE, P2 = kQP2, OB = P2 + 1, MI = 8;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    dev::pc* buf = reinterpret_cast<dev::pc*>(smem) + wave * dev::kPairXbuf;
    const int H = a.hop, NB = (N + H - 1) / H;
    Q15Walk w;
    if (!q15_walk(a, blockIdx.x * kQW + wave, NB, w)) return;
    Q15Ola ola;
    ola.ring = reinterpret_cast<float*>(smem + Q15Lds::bufs) + wave * q15_ring(H);
    ola.H = H;
    ola.RM = q15_ring(H) - 1;
    ola.ring_blocks = a.ring_blocks;
    ola.f0 = w.f0;
    ola.den = a.t.den;
    ola.rd = dev::make_rsrc(a.t.den, uint32_t(a.ring_blocks * H) * 4u);
    ola.ry = dev::make_rsrc(a.y + int64_t(w.s) * a.ld_y, span_bytes(a.out_len, 1));
    ola.ry_null = dev::make_rsrc(a.y, 0u);
    ola.clear(lane);
    dev::Pair15Tw tw;
    dev::pair15_tw_load(tw, reinterpret_cast<const dev::pc*>(a.t.ptw), lane);
    float wsg[E];
#pragma unroll
    for (int m = 0; m < E; ++m) wsg[m] = a.t.ws[lane + 64 * m] * a.gain;
    const bool live = q15_k1(lane) != 15;
    const float* sb = pa.sin + int64_t(w.s) * pa.ld_spec;
    const float* mrow0 = MASK ? pa.mask.p + int64_t(w.s) * pa.mask.ld_stream : nullptr;
    // the pair's rows (and mask rows) by real bin kr = lane + 64 i <= N/2, coalesced,
    // loaded during the previous pair's OLA stage; stepped -- (X g) m, re and im
    // each; DC and Nyquist imaginary parts dropped -- and staged at buf[kr] (frame
    // k) and buf[OB + kr] (frame k+1, zeros past the last)
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
            const int kr = lane + 64 * i;
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
            const int kr = lane + 64 * i;
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
                buf[kr] = dev::pc_mk(ax, ay);
                buf[OB + kr] = dev::pc_mk(bx, by);
            }
        }
        dev::wave_lds_fence();
        return __builtin_amdgcn_ballot_w64(bad) == 0;
    };
    // bin kb of (lane, d): real bin kb (kb <= N/2) or N - kb conjugated; the zero row stays 0
    auto gather = [&](dev::pc (&v)[16], bool pair_form, int off) {
#pragma unroll
        for (int d = 0; d < 16; ++d) {
            const int kb = dev::pair15_bin(lane, d);
            const bool lo = kb <= P2;
            const int j = lo ? kb : N - kb;
            const dev::pc A = buf[off + (live ? j : 0)];
            if (pair_form) {
                const dev::pc B = buf[OB + (live ? j : 0)];
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
            dev::pair15_inv(v, buf, tw, lane);
            if constexpr (PF) {
                if (more) load_rows(k + 2);  // (in flight during the OLA stage)
                ola.pair(v, wsg, a.inv_n, k, w.f1, lane);
            } else {
                ola.push<false>(v, wsg, a.inv_n, k, lane);
                ola.produce(k, lane);
                ola.push<true>(v, wsg, a.inv_n, k + 1, lane);
                if (k + 1 < w.f1) ola.produce(k + 1, lane);
            }
        } else {  // each frame alone, full sanitize (staged again for frame k+1: the inverse used buf)
            gather(v, false, 0);
            dev::pair15_inv(v, buf, tw, lane);
            ola.push<false>(v, wsg, a.inv_n, k, lane);
            ola.produce(k, lane);
            if (k + 1 < w.f1) {
                (void)stage();
                gather(v, false, OB);
                dev::pair15_inv(v, buf, tw, lane);
                ola.push<false>(v, wsg, a.inv_n, k + 1, lane);
                ola.produce(k + 1, lane);
            }
            if (PF && more) load_rows(k + 2);
        }
    }
}

// ------------------------------------------------------------------ K_pair_mask
__global__ __launch_bounds__(64 * kQW, 2) void k_p15_mask(const PairSpecArgs pa) {
    const FusedArgs& a = pa.f;
    constexpr int N = kQN, E = kQE, P2 = kQP2, MI = 8;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    dev::pc* buf = reinterpret_cast<dev::pc*>(smem) + wave * dev::kPairXbuf;
    const int H = a.hop, NB = (N + H - 1) / H;
    Q15Walk w;
    if (!q15_walk(a, blockIdx.x * kQW + wave, NB, w)) return;
    Q15Ola ola;
    ola.ring = reinterpret_cast<float*>(smem + Q15Lds::bufs) + wave * q15_ring(H);
    ola.H = H;
    ola.RM = q15_ring(H) - 1;
    ola.ring_blocks = a.ring_blocks;
    ola.f0 = w.f0;
    ola.den = a.t.den;
    ola.rd = dev::make_rsrc(a.t.den, uint32_t(a.ring_blocks * H) * 4u);
    ola.ry = dev::make_rsrc(a.y + int64_t(w.s) * a.ld_y, span_bytes(a.out_len, 1));
    ola.ry_null = dev::make_rsrc(a.y, 0u);
    ola.clear(lane);
    const __amdgpu_buffer_rsrc_t rx = dev::make_rsrc(a.x + int64_t(w.s) * a.ld_x, span_bytes(a.T, 1));
    dev::Pair15Tw tw;
    dev::pair15_tw_load(tw, reinterpret_cast<const dev::pc*>(a.t.ptw), lane);
    float wa[E], wsg[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        wa[m] = a.t.wa[lane + 64 * m];
        wsg[m] = a.t.ws[lane + 64 * m] * a.gain;
    }
    const bool live = q15_k1(lane) != 15;
    const int partner = q15_partner(lane);
    const float xlo = a.t.px_lo, xhi = a.t.px_hi * 0x1p-20f;  // (mask values up to 2^20)
    const float* mrow0 = pa.mask.p + int64_t(w.s) * pa.mask.ld_stream;
    auto row_a = [&](int k) { return mrow0 + int64_t(k) * pa.mask.ld_frame; };
    auto row_b = [&](int k) { return k + 1 < a.F ? row_a(k) + pa.mask.ld_frame : row_a(k); };  // (past F: unused)
    float ma[MI], mb[MI];  // the pair's mask rows by real bin lane + 64 i (<= N/2; 1 beyond)
    auto load_rows = [&](int k) {
        const float* r0 = row_a(k);
        const float* r1 = row_b(k);
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            const int kr = lane + 64 * i;
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
    q15_load(fa, rx, lane, w.fs * H - a.pad, a.T, a.pad_mode);
    q15_load(fb, rx, lane, (w.fs + 1) * H - a.pad, a.T, a.pad_mode);
    load_rows(w.fs);
    for (int k = w.fs; k < w.f1; k += 2) {
        const bool paired = q15_ok(fa, xlo, xhi) && q15_ok(fb, xlo, xhi) && rows_ok();
        const bool partner_frame = k + 1 < a.F;  // frame k+1 past the last: imaginary part 0
        dev::pc v[16];
        if (paired) {
#pragma unroll
            for (int m = 0; m < E; ++m) v[m] = dev::pc_mk(fa[m] * wa[m], partner_frame ? fb[m] * wa[m] : 0.0f);
            v[15] = dev::pc_mk(0.0f, 0.0f);
            q15_load(fa, rx, lane, (k + 2) * H - a.pad, a.T, a.pad_mode);  // (in flight during the transforms)
            q15_load(fb, rx, lane, (k + 3) * H - a.pad, a.T, a.pad_mode);
            dev::wave_lds_fence();
            dev::pair15_fwd(v, buf, tw, lane);
            // (c1, c2) by real bin in the (now free) transpose buffer
#pragma unroll
            for (int i = 0; i < MI; ++i) {
                const int kr = lane + 64 * i;
                if (kr <= P2) {
                    const float g = a.t.gain ? a.t.gain[kr] : 1.0f;
                    const float ga = g * ma[i], gb = g * mb[i];
                    buf[kr] = dev::pc_mk(0.5f * (ga + gb), 0.5f * (ga - gb));
                }
            }
            if (k + 2 < w.f1) load_rows(k + 2);
            dev::wave_lds_fence();
            dev::pc zp[16];
            q15_partners(v, zp, lane, partner);
#pragma unroll
            for (int d = 0; d < 16; ++d) {
                const int kb = dev::pair15_bin(lane, d);
                const dev::pc cc = buf[live ? (kb <= P2 ? kb : N - kb) : 0];
                v[d] = live ? dev::pc_mk(__builtin_fmaf(cc.y, zp[d].x, cc.x * v[d].x),
                                         __builtin_fmaf(-cc.y, zp[d].y, cc.x * v[d].y))
                            : dev::pc_mk(0.0f, 0.0f);
            }
            dev::wave_lds_fence();  // (the coefficient reads before the inverse's transpose rewrites buf)
            dev::pair15_inv(v, buf, tw, lane);
            ola.push<false>(v, wsg, a.inv_n, k, lane);  // (the divisors fetched ahead would spill here)
            ola.produce(k, lane);
            ola.push<true>(v, wsg, a.inv_n, k + 1, lane);
            if (k + 1 < w.f1) ola.produce(k + 1, lane);
        } else {  // each frame alone, full sanitize, its own gain g m (rows from L2, scrambled)
            auto pass = [&](const float (&f)[E], const float* r, int kk) {
#pragma unroll
                for (int m = 0; m < E; ++m) v[m] = dev::pc_mk(dev::sanit(f[m] * wa[m]), 0.0f);
                v[15] = dev::pc_mk(0.0f, 0.0f);
                dev::wave_lds_fence();
                dev::pair15_fwd(v, buf, tw, lane);
#pragma unroll
                for (int d = 0; d < 16; ++d) {
                    const int kb = dev::pair15_bin(lane, d), kr = live ? (kb <= P2 ? kb : N - kb) : 0;
                    v[d] = live ? v[d] * ((a.t.gain ? a.t.gain[kr] : 1.0f) * r[kr]) : dev::pc_mk(0.0f, 0.0f);
                }
                dev::pair15_inv(v, buf, tw, lane);
                ola.push<false>(v, wsg, a.inv_n, kk, lane);
                ola.produce(kk, lane);
            };
            pass(fa, row_a(k), k);
            if (k + 1 < w.f1) pass(fb, row_b(k), k + 1);
            q15_load(fa, rx, lane, (k + 2) * H - a.pad, a.T, a.pad_mode);
            q15_load(fb, rx, lane, (k + 3) * H - a.pad, a.T, a.pad_mode);
            if (k + 2 < w.f1) load_rows(k + 2);
        }
    }
}

template <typename K>
hipError_t q15_launch(K kernel, const PairSpecArgs& a, int64_t walkers, int32_t kind, bool ring, hipStream_t stream) {
    const size_t lds = Q15Lds::bytes(a.f.hop, ring);
    hipError_t e = set_lds(kernel, lds);
    if (e != hipSuccess) return e;
    const int64_t grid = (walkers + kQW - 1) / kQW;
    note_launch(kind, grid);
    hipLaunchKernelGGL(kernel, dim3(unsigned(grid)), dim3(64 * kQW), lds, stream, a);
    return hipGetLastError();
}

// chunks: about two resident rounds of walks, each >= `min_m` frames, an even length
void q15_chunks(FusedArgs& f, int64_t F, int n_streams, int64_t min_m) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    const int64_t resident = int64_t(cus) * 2 * kQW, S = std::max(1, n_streams);
    int64_t n = std::max<int64_t>(1, std::min<int64_t>(F / min_m, (2 * resident + S - 1) / S));
    n = chunks_or(n, F);
    int64_t m = (F + n - 1) / n;
    m += m & 1;
    f.M = int(m);
    f.n_chunks = int((F + m - 1) / m);
    note_chunks(f.n_chunks);
}

}  // namespace

}  // namespace fk

bool pair15_spec_supported(int n, int h, int ring_len) {
    return n == fk::kQN && h >= 32 && h <= n && ring_len % h == 0;
}

// crlot_stft at N = 960 as frame pairs
hipError_t launch_pair15_stft(const Geometry& g, const DevTables& t, const float* x, int n_streams, int64_t T,
                              int64_t ld_x, int64_t F, float* spec, int64_t ld_spec, int64_t ld_frame,
                              hipStream_t stream) {
    if (!pair15_spec_supported(g.n, g.h, g.ring_len) || F <= 0 || n_streams <= 0 || !t.ptw || !t.wa ||
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
    fk::q15_chunks(a.f, F, n_streams, 32);
    return fk::q15_launch(fk::k_p15_stft, a, int64_t(n_streams) * a.f.n_chunks, CRLOT_K_PAIR_STFT, false, stream);
}

// crlot_istft_ola at N = 960 as frame pairs (the plan's mask, if any, applied)
hipError_t launch_pair15_istft(const Geometry& g, const DevTables& t, const SpecMask& m, const float* spec,
                               int64_t ld_spec, int64_t ld_frame, float* y, int n_streams, int64_t F, int64_t ld_y,
                               hipStream_t stream) {
    if (!pair15_spec_supported(g.n, g.h, g.ring_len) || F <= 0 || n_streams <= 0 || !t.ptw || !t.ws || !t.den ||
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
    fk::q15_chunks(a.f, F, n_streams, 48);
    const int64_t walkers = int64_t(n_streams) * a.f.n_chunks;
    if (g.h <= 256)
        return m.p ? fk::q15_launch(fk::k_p15_istft<true, true>, a, walkers, CRLOT_K_PAIR_ISTFT, true, stream)
                   : fk::q15_launch(fk::k_p15_istft<false, true>, a, walkers, CRLOT_K_PAIR_ISTFT, true, stream);
    return m.p ? fk::q15_launch(fk::k_p15_istft<true, false>, a, walkers, CRLOT_K_PAIR_ISTFT, true, stream)
               : fk::q15_launch(fk::k_p15_istft<false, false>, a, walkers, CRLOT_K_PAIR_ISTFT, true, stream);
}

// crlot_roundtrip at N = 960 with a per-frame mask, one walk
hipError_t launch_pair15_masked(const Geometry& g, const DevTables& t, const SpecMask& m, const float* x, float* y,
                                int n_streams, int64_t T, int64_t ld_x, int64_t ld_y, int64_t F, int64_t out_len,
                                hipStream_t stream) {
    if (!pair15_spec_supported(g.n, g.h, g.ring_len) || F <= 0 || n_streams <= 0 || !m.p || !t.ptw || !t.wa ||
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
    fk::q15_chunks(a.f, F, n_streams, 48);
    return fk::q15_launch(fk::k_p15_mask, a, int64_t(n_streams) * a.f.n_chunks, CRLOT_K_PAIR_MASK, true, stream);
}

}  // namespace crlot
