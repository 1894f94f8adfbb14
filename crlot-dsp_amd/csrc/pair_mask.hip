// pair_mask.hip -- K_pair_mask k_pair_mask<SH,NB>: the N = 1024 frame-pair walk
// (K_pair, pair1k.hip; its two-regime form) with a time-varying spectral step:
// frame k's spectrum scaled by the plan's per-bin gain and by row k of the
// per-frame mask (crlot_plan_set_spectral_mask), between the transforms.
//
// Frames a = 2j and b = 2j+1 share one complex transform z = a w + i b w, so
// Z[k] = A[k] + i B[k] with A[k] = (Z[k] + conj Z[-k]) / 2 and
// B[k] = (Z[k] - conj Z[-k]) / 2i.  Real gains Ga, Gb per frame (bin-symmetric:
// the mask row covers bins 0 .. N/2 of a real frame) give
//     Z'[k] = Ga A[k] + i Gb B[k] = c1 Z[k] + c2 conj Z[-k],
//     c1 = (Ga + Gb) / 2,  c2 = (Ga - Gb) / 2,
// so the step needs each bin's partner Z[-k].  In fft_pair.h's bin-scrambled
// layout bin k = pbl(l) + 64 d sits in lane l, register d; its partner
// N - k = (64 - pbl(l)) + 64 (15 - d) is register 15 - d of lane
// pbl(64 - pbl(l)) (pbl swaps lane bits 2-3 with 4-5: an involution), except
// for lane 0 (k = 64 d), whose partner is its own register (16 - d) mod 16: one
// ds_bpermute per float, no LDS.  With Ga = Gb (the time-invariant gain) this
// is K_pair's Z' = G Z.
//
// Regimes per pair, as k_stft_ola_pair_fix: paired when the pair's hops keep
// px_lo <= |x| <= px_hi / 2^20 (or 0) and every mask value of both rows is
// finite with |m| <= 2^20 -- then no transform overflows (|Z'| < 2^95, the
// inverse < 2^105) and the output sanitize is its threshold test; otherwise each
// frame is transformed alone (imaginary part zero, full sanitize on both sides)
// with its own gain G = g m, so a NaN, Inf or huge sample or mask value stays in
// its frame, as the reference transforms every frame alone.  The OLA stage and
// the division are k_stft_ola_pair_fix's.  Results equal the per-frame kiss_fftr
// formulation (crlot_istft_ola(crlot_stft(x))) within float32 rounding, not bit
// for bit, and do not depend on the chunking or the batch.
#include <type_traits>

#include "fft_pair.h"
#include "fft_pair512.h"
#include "fused_common.h"

namespace crlot {
namespace fk {

struct MaskWalkArgs {
    FusedArgs f;
    SpecMask mask;
};

namespace {

constexpr int kMW = 4;  // waves per workgroup, each walking its own chunk
#ifndef CRLOT_PAIR_MASK_WAVES
#define CRLOT_PAIR_MASK_WAVES 2  // waves per SIMD
#endif

// LDS: the twiddle tables (loaded into registers, then overlaid by the gain
// table [N], symmetric) | wa4 [1024] | ws4 [1024] | per-wave transpose buffers |
// per-wave step coefficients (c1, c2) [513] (69.7 KB: two workgroups per CU)
struct MaskLds {
    static constexpr size_t t1 = 0;
    static constexpr size_t t2 = t1 + sizeof(dev::pc) * 15 * 64;
    static constexpr size_t wa = t2 + sizeof(dev::pc) * 3 * 16;
    static constexpr size_t ws = wa + sizeof(float) * 1024;
    static constexpr size_t bufs = ws + sizeof(float) * 1024;
    static constexpr int kCst = 514;  // per wave: (c1, c2) of the staged pair by real bin 0 .. 512
    static constexpr size_t cst = bufs + sizeof(dev::pc) * dev::kPairXbuf * kMW;
    static constexpr size_t bytes = cst + sizeof(dev::pc) * kCst * kMW;
};
static_assert(sizeof(dev::pc) * (15 * 64 + 3 * 16) >= sizeof(float) * 1024, "the gain table overlays the twiddles");

// (both take the value as a scalar: a bit cast applied to an ext_vector element
// directly is miscompiled by this clang)
__device__ __forceinline__ float lane0(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
}
__device__ __forceinline__ float bperm(int src_lane, float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src_lane * 4, __builtin_bit_cast(int, v)));
}

template <int SH, int NB>
__global__ __launch_bounds__(64 * kMW, CRLOT_PAIR_MASK_WAVES) void k_pair_mask(const MaskWalkArgs ma) {
    const FusedArgs& a = ma.f;
    constexpr int E = 16, N = 1024, H = 64 * SH, P2 = N / 2;
    static_assert(NB * SH == E, "N = NB * H");
    static_assert(SH >= 2, "den rows are read 16 bytes at a time");
    constexpr bool kFold = SH != 2;  // K_pair's OLA form (pair1k.hip kPairFoldWs): ws g staged
    extern __shared__ __attribute__((aligned(16))) char smem[];
    dev::pc* t1 = reinterpret_cast<dev::pc*>(smem + MaskLds::t1);
    dev::pc* t2s = reinterpret_cast<dev::pc*>(smem + MaskLds::t2);
    float* wa4 = reinterpret_cast<float*>(smem + MaskLds::wa);
    float* ws4 = reinterpret_cast<float*>(smem + MaskLds::ws);
    {
        const dev::pc* g1 = reinterpret_cast<const dev::pc*>(a.t.ptw);
        for (int i = threadIdx.x; i < 15 * 64 + 3 * 16; i += 64 * kMW) t1[i] = g1[i];  // t1 | t2
        for (int i = threadIdx.x; i < N; i += 64 * kMW) {
            const int l = i & 63, m = i >> 6;  // tap n = l + 64 m, stored [m/4][lane][m%4]
            const int d = (m >> 2) * 256 + l * 4 + (m & 3);
            wa4[d] = a.t.wa[i];
            ws4[d] = kFold ? a.t.wsn[i] * a.gain : a.t.wsn[i];
        }
        __syncthreads();
    }
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    dev::pc* buf = reinterpret_cast<dev::pc*>(smem + MaskLds::bufs) + wave * dev::kPairXbuf;
    std::conditional_t<SH == 4, dev::PairTwReg, dev::PairTw> tw;  // K_pair's twiddle forms
    dev::pair_tw_load(tw, t1, t2s + (lane & 15), lane);
    // the gain table replaces the twiddles in LDS (ones without a gain: x * 1 == x)
    __syncthreads();
    {
        float* gw_ = reinterpret_cast<float*>(smem + MaskLds::t1);
        for (int i = threadIdx.x; i < N; i += 64 * kMW)
            gw_[i] = a.t.gain ? a.t.gain[i <= P2 ? i : N - i] : 1.0f;
        __syncthreads();
    }
    const float* gl = reinterpret_cast<const float*>(smem + MaskLds::t1);
    const int gw = blockIdx.x * kMW + wave;
    if (gw >= a.n_streams * a.n_chunks) return;
    const int s = gw / a.n_chunks, c = gw - s * a.n_chunks;
    const int f0 = c * a.M, f1 = min(a.F, f0 + a.M);
    const int fs = max(0, f0 - (NB - 1)) & ~1;  // pairs start on even frames
    const __amdgpu_buffer_rsrc_t rx = dev::make_rsrc(a.x + int64_t(s) * a.ld_x, span_bytes(a.T, 1));
    const __amdgpu_buffer_rsrc_t ry = dev::make_rsrc(a.y + int64_t(s) * a.ld_y, span_bytes(a.out_len, 1));
    const __amdgpu_buffer_rsrc_t rp = dev::make_rsrc(a.t.pden, uint32_t(a.ring_blocks * H) * 8u);
    const __amdgpu_buffer_rsrc_t ry_null = dev::make_rsrc(a.y, 0u);
    const float xlo = a.t.px_lo, xhi = a.t.px_hi * 0x1p-20f;  // (mask values up to 2^20)
    const float* mrow0 = ma.mask.p + int64_t(s) * ma.mask.ld_stream;
    // this lane's bins: kb = pbl + 64 d, their real-frame index min(kb, N - kb), and the partner lane
    const int pbl = dev::pair_bin_lane(lane);
    const int partner = dev::pair_bin_lane((64 - pbl) & 63);

    float xin[E + SH];
    auto load_hop = [&](float* dst, int origin) { load_hop1<SH>(dst, rx, lane, origin, a.T, a.pad_mode); };
    float acc[NB][SH];
    auto accumulate = [&](const dev::pc (&v)[E], bool imag, bool paired) {
#pragma unroll
        for (int m4 = 0; m4 < E / 4; ++m4) {
            const float4 w = *reinterpret_cast<const float4*>(ws4 + m4 * 256 + lane * 4);
            const float wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int m = 4 * m4 + u;
                const float x = imag ? v[m].y : v[m].x;
                const float o = paired ? dev::sanit_scaled_finite<N>(x) : dev::sanit_scaled<N>(x);
                float& r = acc[m / SH][m % SH];
                if constexpr (kFold)
                    r = __builtin_fmaf(o, wv[u], r);
                else
                    r = __builtin_fmaf(__builtin_fmaf(o, wv[u], 0.0f), a.gain, r);
            }
        }
    };
    auto emit = [&](int k, const float (&dr)[2 * SH]) {
        float mx = 0.0f, mn = 0x1p127f;
#pragma unroll
        for (int q = 0; q < SH; ++q) {
            const float t = __builtin_fabsf(acc[0][q]);
            mx = __builtin_fmaxf(mx, t);
            mn = __builtin_fminf(mn, t);
        }
        const bool ok = (mx <= 0x1p64f) & ((mn >= 0x1p-64f) | (mx == 0.0f));
        float o[SH];
#pragma unroll
        for (int q = 0; q < SH; ++q) o[q] = mk_div(acc[0][q], dr[q], dr[SH + q]);
        if (__builtin_amdgcn_ballot_w64(!ok) != 0) {
#pragma unroll
            for (int q = 0; q < SH; ++q) o[q] = acc[0][q] / dr[q];
        }
        const __amdgpu_buffer_rsrc_t rk = k >= f0 ? ry : ry_null;  // warm-up blocks: dropped
#pragma unroll
        for (int q = 0; q < SH; ++q)
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o[q]), rk, lane * 4,
                                                  k * (4 * H) + q * 256, 0);
#pragma unroll
        for (int j = 0; j < NB - 1; ++j)
#pragma unroll
            for (int q = 0; q < SH; ++q) acc[j][q] = acc[j + 1][q];
#pragma unroll
        for (int q = 0; q < SH; ++q) acc[NB - 1][q] = 0.f;
    };

    uint32_t hopok = 0;
#pragma unroll
    for (int h = 0; h <= NB; ++h) {
        load_hop(xin + h * SH, (fs + h) * H - a.pad);
        hopok |= hop_ok<SH>(xin + h * SH, xlo, xhi) << h;
    }
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int q = 0; q < SH; ++q) acc[j][q] = 0.f;

    constexpr uint32_t kPairHops = (1u << (NB + 1)) - 1;
    // The step's coefficients for a pair, staged one pair ahead: the mask rows load
    // coalesced (real bin kr = lane + 64 i; i = 8 is bin 512, lane 0's) while the
    // previous pair transforms, then c1 = (g ma + g mb) / 2, c2 = (g ma - g mb) / 2
    // go to this wave's LDS rows, read back by the step in the scrambled order
    // (in-order LDS: the writes follow the previous step's reads)
    dev::pc* cst = reinterpret_cast<dev::pc*>(smem + MaskLds::cst) + wave * MaskLds::kCst;
    constexpr int MI = 9;
    float mra[MI], mrb[MI];
    auto row_a = [&](int k) { return mrow0 + int64_t(k) * ma.mask.ld_frame; };
    auto row_b = [&](int k) { return k + 1 < a.F ? row_a(k) + ma.mask.ld_frame : row_a(k); };  // (past F: unused)
    auto load_rows = [&](int k) {
        const float* ra = row_a(k);
        const float* rb = row_b(k);
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            const int kr = i < 8 ? lane + 64 * i : P2;
            mra[i] = ra[kr];
            mrb[i] = rb[kr];
        }
    };
    auto stage_rows = [&]() -> bool {  // true: every value keeps the paired regime
        bool bad = false;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            const int kr = i < 8 ? lane + 64 * i : P2;
            bad |= !(__builtin_fabsf(mra[i]) <= 0x1p20f) | !(__builtin_fabsf(mrb[i]) <= 0x1p20f);  // (NaN too)
            const float g = gl[kr];
            const float ga = g * mra[i], gb = g * mrb[i];
            if (i < 8 || lane == 0) cst[kr] = dev::pc_mk(0.5f * (ga + gb), 0.5f * (ga - gb));
        }
        return __builtin_amdgcn_ballot_w64(bad) == 0;
    };
    // bin kb = pbl + 64 d: real bin kr = kb (d < 8), N - kb (d >= 8; d = 8, pbl = 0: 512 both ways)
    const dev::pc* const cb1 = cst + pbl;
    const dev::pc* const cb2 = cst - pbl;
    load_rows(fs);
    bool mok = stage_rows();
    for (int k = fs; k < f1; k += 2) {
        float nxt[2 * SH];
        load_hop(nxt, (k + NB + 1) * H - a.pad);
        load_hop(nxt + SH, (k + NB + 2) * H - a.pad);
        const bool more = k + 2 < f1;
        if (more) load_rows(k + 2);  // (in flight during this pair)
        const bool paired = mok && (hopok & kPairHops) == kPairHops;
        dev::pc v[E];
        if (paired) {
#pragma unroll
            for (int m4 = 0; m4 < E / 4; ++m4) {
                const float4 w = *reinterpret_cast<const float4*>(wa4 + m4 * 256 + lane * 4);
                const float wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int m = 4 * m4 + u;
                    v[m] = dev::pc_mk(xin[m] * wv[u], xin[m + SH] * wv[u]);
                }
            }
            dev::pair_fft_fwd(v, buf, tw, tw, lane);
            // the step, Z' = c1 Z + c2 conj Z[-k], registers d and 15 - d together so
            // both update in place; lane 0's partners are its own registers
            // (16 - d) mod 16, read into SGPRs before any update
            float own_r[E], own_i[E];
#pragma unroll
            for (int d = 0; d < E; ++d) {
                const float re = v[(16 - d) & 15].x, im = v[(16 - d) & 15].y;
                own_r[d] = lane0(re);
                own_i[d] = lane0(im);
            }
#pragma unroll
            for (int d = 0; d < E / 2; ++d) {
                const int e = 15 - d;
                dev::pc zd = dev::pc_mk(bperm(partner, v[e].x), bperm(partner, v[e].y));
                dev::pc ze = dev::pc_mk(bperm(partner, v[d].x), bperm(partner, v[d].y));
                if (lane == 0) {
                    zd = dev::pc_mk(own_r[d], own_i[d]);
                    ze = dev::pc_mk(own_r[e], own_i[e]);
                }
                const dev::pc cd = cb1[64 * d], ce = cb2[N - 64 * e];
                v[d] = dev::pc_mk(__builtin_fmaf(cd.y, zd.x, cd.x * v[d].x), __builtin_fmaf(-cd.y, zd.y, cd.x * v[d].y));
                v[e] = dev::pc_mk(__builtin_fmaf(ce.y, ze.x, ce.x * v[e].x), __builtin_fmaf(-ce.y, ze.y, ce.x * v[e].y));
            }
            dev::pair_fft_inv(v, buf, tw, tw, lane);
            float dr0[2 * SH], dr1[2 * SH];
            load_den<SH>(dr0, rp, lane, k % a.ring_blocks);
            load_den<SH>(dr1, rp, lane, (k + 1) % a.ring_blocks);
            accumulate(v, false, true);
            emit(k, dr0);
            if (k + 1 < f1) {
                accumulate(v, true, true);
                emit(k + 1, dr1);
            }
        } else {  // each frame alone, full sanitize, its own gain g m (rows read again)
            const int npass = min(2, f1 - k);
            for (int p = 0; p < npass; ++p) {
#pragma unroll
                for (int m4 = 0; m4 < E / 4; ++m4) {
                    const float4 w = *reinterpret_cast<const float4*>(wa4 + m4 * 256 + lane * 4);
                    const float wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int m = 4 * m4 + u;
                        v[m] = dev::pc_mk(dev::sanit((p ? xin[m + SH] : xin[m]) * wv[u]), 0.0f);
                    }
                }
                dev::pair_fft_fwd(v, buf, tw, tw, lane);
                const float* r = p ? row_b(k) : row_a(k);
#pragma unroll
                for (int d = 0; d < E; ++d) {
                    const int kb = pbl + 64 * d, kr = kb <= P2 ? kb : N - kb;
                    v[d] = v[d] * (gl[kb] * r[kr]);
                }
                dev::pair_fft_inv(v, buf, tw, tw, lane);
                float dr[2 * SH];
                load_den<SH>(dr, rp, lane, (k + p) % a.ring_blocks);
                accumulate(v, false, false);
                emit(k + p, dr);
            }
        }
        if (more) mok = stage_rows();
        hopok = (hopok | hop_ok<SH>(nxt, xlo, xhi) << (NB + 1) | hop_ok<SH>(nxt + SH, xlo, xhi) << (NB + 2)) >> 2;
#pragma unroll
        for (int m = 0; m < E + SH - 2 * SH; ++m) xin[m] = xin[m + 2 * SH];
#pragma unroll
        for (int q = 0; q < 2 * SH; ++q) xin[E - SH + q] = nxt[q];
    }
}

// ------------------------------------------------------------------ N = 512
// The same walk on K_pair512's transform (fft_pair512.h): bins q(l) + 64 d with
// q(l) = (l >> 3) + 8 (l & 7), the partner of (l, d) register 7 - d of lane
// q(64 - q(l)) (lane 0: its own register (8 - d) mod 8); windows, twiddles in
// registers, the gain from L2; per wave the exchange buffer and the staged
// (c1, c2) of bins 0 .. 256.
struct Mask512Lds {
    static constexpr int kCst = 258;
    static constexpr int per_wave = dev::kP512Buf + kCst;  // complex elements
    static constexpr size_t bytes = sizeof(dev::pc) * per_wave * kMW;
};
__device__ __forceinline__ int m512_q(int l) { return (l >> 3) + 8 * (l & 7); }

template <int SH, int NB>
__global__ __launch_bounds__(64 * kMW) void k_pair512_mask(const MaskWalkArgs ma) {
    const FusedArgs& a = ma.f;
    constexpr int E = 8, N = 512, H = 64 * SH, P2 = N / 2;
    static_assert(NB * SH == E, "N = NB * H");
    static_assert(SH >= 2, "den rows are read 16 bytes at a time");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    dev::pc* buf = reinterpret_cast<dev::pc*>(smem) + wave * Mask512Lds::per_wave;
    dev::pc* cst = buf + dev::kP512Buf;
    const int gw = blockIdx.x * kMW + wave;
    if (gw >= a.n_streams * a.n_chunks) return;
    const int s = gw / a.n_chunks, c = gw - s * a.n_chunks;
    const int f0 = c * a.M, f1 = min(a.F, f0 + a.M);
    const int fs = max(0, f0 - (NB - 1)) & ~1;
    const __amdgpu_buffer_rsrc_t rx = dev::make_rsrc(a.x + int64_t(s) * a.ld_x, span_bytes(a.T, 1));
    const __amdgpu_buffer_rsrc_t ry = dev::make_rsrc(a.y + int64_t(s) * a.ld_y, span_bytes(a.out_len, 1));
    const __amdgpu_buffer_rsrc_t rp = dev::make_rsrc(a.t.pden, uint32_t(a.ring_blocks * H) * 8u);
    const __amdgpu_buffer_rsrc_t ry_null = dev::make_rsrc(a.y, 0u);
    const float xlo = a.t.px_lo, xhi = a.t.px_hi * 0x1p-20f;  // (mask values up to 2^20)
    const float* mrow0 = ma.mask.p + int64_t(s) * ma.mask.ld_stream;
    const int q = m512_q(lane);
    const int partner = m512_q((64 - q) & 63);
    dev::Pair512TwReg tw;
    dev::pair512_tw_load(tw, reinterpret_cast<const dev::pc*>(a.t.ptw), lane);
    float wa[E], ws[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        wa[m] = a.t.wa[lane + 64 * m];
        ws[m] = a.t.wsn[lane + 64 * m] * a.gain;  // (ws g: K_pair512's OLA form)
    }
    auto gain_at = [&](int kr) { return a.t.gain ? a.t.gain[kr] : 1.0f; };
    float xin[E + SH];
    auto load_hop = [&](float* dst, int origin) { load_hop1<SH>(dst, rx, lane, origin, a.T, a.pad_mode); };
    float acc[NB][SH];
    auto accumulate = [&](const dev::pc (&v)[E], bool imag, bool paired) {
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const float x = imag ? v[m].y : v[m].x;
            const float o = paired ? dev::sanit_scaled_finite<N>(x) : dev::sanit_scaled<N>(x);
            float& r = acc[m / SH][m % SH];
            r = __builtin_fmaf(o, ws[m], r);
        }
    };
    auto emit = [&](int k, const float (&dr)[2 * SH]) {
        float mx = 0.0f, mn = 0x1p127f;
#pragma unroll
        for (int qq = 0; qq < SH; ++qq) {
            const float t = __builtin_fabsf(acc[0][qq]);
            mx = __builtin_fmaxf(mx, t);
            mn = __builtin_fminf(mn, t);
        }
        const bool ok = (mx <= 0x1p64f) & ((mn >= 0x1p-64f) | (mx == 0.0f));
        float o[SH];
#pragma unroll
        for (int qq = 0; qq < SH; ++qq) o[qq] = mk_div(acc[0][qq], dr[qq], dr[SH + qq]);
        if (__builtin_amdgcn_ballot_w64(!ok) != 0) {
#pragma unroll
            for (int qq = 0; qq < SH; ++qq) o[qq] = acc[0][qq] / dr[qq];
        }
        const __amdgpu_buffer_rsrc_t rk = k >= f0 ? ry : ry_null;
#pragma unroll
        for (int qq = 0; qq < SH; ++qq)
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o[qq]), rk, lane * 4,
                                                  k * (4 * H) + qq * 256, 0);
#pragma unroll
        for (int j = 0; j < NB - 1; ++j)
#pragma unroll
            for (int qq = 0; qq < SH; ++qq) acc[j][qq] = acc[j + 1][qq];
#pragma unroll
        for (int qq = 0; qq < SH; ++qq) acc[NB - 1][qq] = 0.f;
    };
    uint32_t hopok = 0;
#pragma unroll
    for (int h = 0; h <= NB; ++h) {
        load_hop(xin + h * SH, (fs + h) * H - a.pad);
        hopok |= hop_ok<SH>(xin + h * SH, xlo, xhi) << h;
    }
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int qq = 0; qq < SH; ++qq) acc[j][qq] = 0.f;

    constexpr uint32_t kPairHops = (1u << (NB + 1)) - 1;
    constexpr int MI = 5;  // real bins lane + 64 i (i = 4: bin 256, lane 0's)
    float mra[MI], mrb[MI];
    auto row_a = [&](int k) { return mrow0 + int64_t(k) * ma.mask.ld_frame; };
    auto row_b = [&](int k) { return k + 1 < a.F ? row_a(k) + ma.mask.ld_frame : row_a(k); };
    auto load_rows = [&](int k) {
        const float* ra = row_a(k);
        const float* rb = row_b(k);
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            const int kr = i < 4 ? lane + 64 * i : P2;
            mra[i] = ra[kr];
            mrb[i] = rb[kr];
        }
    };
    auto stage_rows = [&]() -> bool {
        bool bad = false;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            const int kr = i < 4 ? lane + 64 * i : P2;
            bad |= !(__builtin_fabsf(mra[i]) <= 0x1p20f) | !(__builtin_fabsf(mrb[i]) <= 0x1p20f);  // (NaN too)
            const float g = gain_at(kr);
            const float ga = g * mra[i], gb = g * mrb[i];
            if (i < 4 || lane == 0) cst[kr] = dev::pc_mk(0.5f * (ga + gb), 0.5f * (ga - gb));
        }
        return __builtin_amdgcn_ballot_w64(bad) == 0;
    };
    const dev::pc* const cb1 = cst + q;
    const dev::pc* const cb2 = cst - q;
    load_rows(fs);
    bool mok = stage_rows();
    for (int k = fs; k < f1; k += 2) {
        float nxt[2 * SH];
        load_hop(nxt, (k + NB + 1) * H - a.pad);
        load_hop(nxt + SH, (k + NB + 2) * H - a.pad);
        const bool more = k + 2 < f1;
        if (more) load_rows(k + 2);
        const bool paired = mok && (hopok & kPairHops) == kPairHops;
        dev::pc v[E];
        if (paired) {
#pragma unroll
            for (int m = 0; m < E; ++m) v[m] = dev::pc_mk(xin[m] * wa[m], xin[m + SH] * wa[m]);
            dev::wave_lds_fence();
            dev::pair512_fwd(v, buf, tw, lane);
            float own_r[E], own_i[E];
#pragma unroll
            for (int d = 0; d < E; ++d) {
                const float re = v[(8 - d) & 7].x, im = v[(8 - d) & 7].y;
                own_r[d] = lane0(re);
                own_i[d] = lane0(im);
            }
#pragma unroll
            for (int d = 0; d < E / 2; ++d) {
                const int e = 7 - d;
                dev::pc zd = dev::pc_mk(bperm(partner, v[e].x), bperm(partner, v[e].y));
                dev::pc ze = dev::pc_mk(bperm(partner, v[d].x), bperm(partner, v[d].y));
                if (lane == 0) {
                    zd = dev::pc_mk(own_r[d], own_i[d]);
                    ze = dev::pc_mk(own_r[e], own_i[e]);
                }
                const dev::pc cd = cb1[64 * d], ce = cb2[N - 64 * e];
                v[d] = dev::pc_mk(__builtin_fmaf(cd.y, zd.x, cd.x * v[d].x), __builtin_fmaf(-cd.y, zd.y, cd.x * v[d].y));
                v[e] = dev::pc_mk(__builtin_fmaf(ce.y, ze.x, ce.x * v[e].x), __builtin_fmaf(-ce.y, ze.y, ce.x * v[e].y));
            }
            dev::pair512_inv(v, buf, tw, lane);
            float dr0[2 * SH], dr1[2 * SH];
            load_den<SH>(dr0, rp, lane, k % a.ring_blocks);
            load_den<SH>(dr1, rp, lane, (k + 1) % a.ring_blocks);
            accumulate(v, false, true);
            emit(k, dr0);
            if (k + 1 < f1) {
                accumulate(v, true, true);
                emit(k + 1, dr1);
            }
        } else {  // each frame alone, full sanitize, its own gain g m
            const int npass = min(2, f1 - k);
            for (int p = 0; p < npass; ++p) {
#pragma unroll
                for (int m = 0; m < E; ++m) v[m] = dev::pc_mk(dev::sanit((p ? xin[m + SH] : xin[m]) * wa[m]), 0.0f);
                dev::wave_lds_fence();
                dev::pair512_fwd(v, buf, tw, lane);
                const float* r = p ? row_b(k) : row_a(k);
#pragma unroll
                for (int d = 0; d < E; ++d) {
                    const int kb = q + 64 * d, kr = kb <= P2 ? kb : N - kb;
                    v[d] = v[d] * (gain_at(kr) * r[kr]);
                }
                dev::pair512_inv(v, buf, tw, lane);
                float dr[2 * SH];
                load_den<SH>(dr, rp, lane, (k + p) % a.ring_blocks);
                accumulate(v, false, false);
                emit(k + p, dr);
            }
        }
        if (more) mok = stage_rows();
        hopok = (hopok | hop_ok<SH>(nxt, xlo, xhi) << (NB + 1) | hop_ok<SH>(nxt + SH, xlo, xhi) << (NB + 2)) >> 2;
#pragma unroll
        for (int m = 0; m < E + SH - 2 * SH; ++m) xin[m] = xin[m + 2 * SH];
#pragma unroll
        for (int qq = 0; qq < 2 * SH; ++qq) xin[E - SH + qq] = nxt[qq];
    }
}

template <int SH>
hipError_t pair512_mask_sh(const MaskWalkArgs& a, int64_t grid, hipStream_t stream) {
    constexpr int NB = 8 / SH;
    hipLaunchKernelGGL((k_pair512_mask<SH, NB>), dim3(unsigned(grid)), dim3(64 * kMW), Mask512Lds::bytes, stream, a);
    return hipGetLastError();
}

template <int SH>
hipError_t pair_mask_sh(const MaskWalkArgs& a, int64_t grid, hipStream_t stream) {
    constexpr int NB = 16 / SH;
    auto k = k_pair_mask<SH, NB>;
    hipError_t e = set_lds(k, MaskLds::bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3(unsigned(grid)), dim3(64 * kMW), MaskLds::bytes, stream, a);
    return hipGetLastError();
}

}  // namespace

int pair_mask_walkers_per_cu(int n) {
    if (n >= 2048) return pair_wg_walkers_per_cu(n);
    static const int v1k = [] {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void*>(k_pair_mask<4, 4>),
                                                         64 * kMW, MaskLds::bytes) != hipSuccess ||
            nb <= 0)
            nb = 1;
        return nb * kMW;
    }();
    static const int v512 = [] {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void*>(k_pair512_mask<2, 4>),
                                                         64 * kMW, Mask512Lds::bytes) != hipSuccess ||
            nb <= 0)
            nb = 1;
        return nb * kMW;
    }();
    return n == 512 ? v512 : v1k;
}

hipError_t launch_pair_mask(int n, int h, const FusedArgs& f, const SpecMask& m, int64_t walkers,
                            hipStream_t stream) {
    if (n >= 2048) {  // one workgroup per walk (pair_wg_spec.hip)
        PairSpecArgs pa{};
        pa.f = f;
        pa.mask = m;
        return launch_pairwg_mask(n, h, pa, walkers, stream);
    }
    MaskWalkArgs a;
    a.f = f;
    a.mask = m;
    const int64_t grid = (walkers + kMW - 1) / kMW;
    note_launch(CRLOT_K_PAIR_MASK, grid);
    if (n == 512) {
        switch (h) {
            case 128: return pair512_mask_sh<2>(a, grid, stream);
            case 256: return pair512_mask_sh<4>(a, grid, stream);
            default: return hipErrorInvalidValue;
        }
    }
    switch (h) {
        case 128: return pair_mask_sh<2>(a, grid, stream);
        case 256: return pair_mask_sh<4>(a, grid, stream);
        case 512: return pair_mask_sh<8>(a, grid, stream);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace fk
}  // namespace crlot
