// pair_stft.hip -- the spectral entries as frame pairs at N = 1024 (frame
// pairing on, the default): K_pair_stft k_pair_stft<SH> (crlot_stft) and
// K_pair_istft k_pair_istft<SH,NB> (crlot_istft_ola), H = 64 SH, SH = 2, 4, 8.
//
// Frames a = 2j and b = 2j+1 of a stream share one 1024-point complex transform
// (fft_pair.h, K_pair's).  Forward: z = a w + i b w, Z = FFT(z), and the two
// real spectra come out of the bin-scrambled Z with their partners Z[-k]
// (register 15 - d of lane pbl(64 - pbl(l)), one ds_bpermute per float; lane
// 0's partners are its own registers (16 - d) mod 16, pair_mask.hip):
//     A[k] = (Z[k] + conj Z[-k]) / 2,   B[k] = (Z[k] - conj Z[-k]) / 2i,
// stored for k = 0 .. N/2 (DC and Nyquist come out with exactly zero imaginary
// parts, as kiss_fftr writes them).  Inverse: the two stepped half spectra,
// extended by conjugate symmetry (imaginary parts of DC and Nyquist ignored, as
// kiss_fftri ignores them), form Z = A' + i B' and ONE inverse gives both frames'
// push_frame_AoS inputs, then K_pair's OLA stage and division.
//
// Regimes, as the other pair walkers: the forward pairs frames whose samples
// keep px_lo <= |x| <= px_hi (or 0) -- sanitize(x w) = x w there -- and
// transforms any other frame alone with the full input sanitize; the inverse
// pairs spectra whose stepped values are all finite and below 2^60 (no
// overflow, output sanitize reduced to its threshold test) and otherwise inverts
// each frame alone with the full sanitize.  Pairs start on even frames whatever
// the chunking, so every value depends only on its stream.  The results equal
// the per-frame kiss_fftr / kiss_fftri formulation within float32 rounding, not
// bit for bit (frame pairing off keeps K_stft / K_istft: bit-identical to
// crlot_rfft_batched / crlot_irfft_batched + crlot_ola_gather).
#include <algorithm>
#include <type_traits>

#include "fft_pair.h"
#include "fft_pair512.h"
#include "fused_common.h"

namespace crlot {
namespace fk {

namespace {

constexpr int kSW = 4;  // waves per workgroup, each walking its own chunk
#ifndef CRLOT_PAIR_SPEC_NT
#define CRLOT_PAIR_SPEC_NT 0  // A/B: nontemporal spectrum stores / row loads (measured: stft -7 to -11 %, istft +1 %)
#endif
__device__ __forceinline__ void st2(float2* p, float x, float y) {
#if CRLOT_PAIR_SPEC_NT
    __builtin_nontemporal_store(x, &p->x);
    __builtin_nontemporal_store(y, &p->y);
#else
    *p = make_float2(x, y);
#endif
}
__device__ __forceinline__ float2 ld2(const float2* p) {
#if CRLOT_PAIR_SPEC_NT
    return make_float2(__builtin_nontemporal_load(&p->x), __builtin_nontemporal_load(&p->y));
#else
    return *p;
#endif
}

// (float arguments: a bit cast applied to an ext_vector element directly is
// miscompiled by this clang)
__device__ __forceinline__ float bperm_f(int src_lane, float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src_lane * 4, __builtin_bit_cast(int, v)));
}

// LDS: twiddle tables t1 | t2 (loaded into registers; the istft then overlays
// its gain table on them) | window [1024] stored [m/4][lane][m%4] | per-wave
// transpose buffers
struct SpecLds {
    static constexpr size_t t1 = 0;
    static constexpr size_t t2 = t1 + sizeof(dev::pc) * 15 * 64;
    static constexpr size_t win = t2 + sizeof(dev::pc) * 3 * 16;
    static constexpr size_t bufs = win + sizeof(float) * 1024;
    static constexpr size_t bytes = bufs + sizeof(dev::pc) * dev::kPairXbuf * kSW;
};

template <typename TW>
__device__ __forceinline__ void spec_lds_setup(const FusedArgs& a, char* smem, const float* wtab, float wscale,
                                               TW& tw, int lane) {
    dev::pc* t1 = reinterpret_cast<dev::pc*>(smem + SpecLds::t1);
    dev::pc* t2s = reinterpret_cast<dev::pc*>(smem + SpecLds::t2);
    float* w4 = reinterpret_cast<float*>(smem + SpecLds::win);
    const dev::pc* g1 = reinterpret_cast<const dev::pc*>(a.t.ptw);
    for (int i = threadIdx.x; i < 15 * 64 + 3 * 16; i += 64 * kSW) t1[i] = g1[i];  // t1 | t2
    for (int i = threadIdx.x; i < 1024; i += 64 * kSW) {
        const int l = i & 63, m = i >> 6;  // tap n = l + 64 m
        w4[(m >> 2) * 256 + l * 4 + (m & 3)] = wtab[i] * wscale;
    }
    __syncthreads();
    dev::pair_tw_load(tw, t1, t2s + (lane & 15), lane);
}

// ------------------------------------------------------------------ K_pair_stft
template <int SH>
__global__ __launch_bounds__(64 * kSW, 3) void k_pair_stft(const PairSpecArgs pa) {
    const FusedArgs& a = pa.f;
    constexpr int E = 16, N = 1024, H = 64 * SH, NB = 16 / SH, P2 = N / 2;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    std::conditional_t<SH == 4, dev::PairTwReg, dev::PairTw> tw;  // K_pair's twiddle forms
    spec_lds_setup(a, smem, a.t.wa, 1.0f, tw, lane);
    const float* wa4 = reinterpret_cast<const float*>(smem + SpecLds::win);
    dev::pc* buf = reinterpret_cast<dev::pc*>(smem + SpecLds::bufs) + wave * dev::kPairXbuf;
    const int gw = blockIdx.x * kSW + wave;
    if (gw >= a.n_streams * a.n_chunks) return;
    const int s = gw / a.n_chunks, c = gw - s * a.n_chunks;
    const int f0 = c * a.M, f1 = min(a.F, f0 + a.M);  // (M even: chunks start on even frames)
    const __amdgpu_buffer_rsrc_t rx = dev::make_rsrc(a.x + int64_t(s) * a.ld_x, span_bytes(a.T, 1));
    float* so = pa.spec + int64_t(s) * pa.ld_spec;
    const float xlo = a.t.px_lo, xhi = a.t.px_hi;
    const int pbl = dev::pair_bin_lane(lane);
    const int partner = dev::pair_bin_lane((64 - pbl) & 63);
    auto load_hop = [&](float* dst, int origin) { load_hop1<SH>(dst, rx, lane, origin, a.T, a.pad_mode); };

    float xin[E + SH];  // hops k .. k+NB of the pair at k
    uint32_t hopok = 0;
#pragma unroll
    for (int h = 0; h <= NB; ++h) {
        load_hop(xin + h * SH, (f0 + h) * H - a.pad);
        hopok |= hop_ok<SH>(xin + h * SH, xlo, xhi) << h;
    }
    // bins k = pbl + 64 d <= N/2 of a frame: d < 8 in every lane, d = 8 in lane 0 (k = N/2)
    auto store_bins = [&](float* row, auto valfn) {
        float2* r2 = reinterpret_cast<float2*>(row);
#pragma unroll
        for (int d = 0; d < 8; ++d) {
            const dev::pc o = valfn(d);
            st2(r2 + pbl + 64 * d, o.x, o.y);
        }
        if (lane == 0) {
            const dev::pc o = valfn(8);
            st2(r2 + P2, o.x, o.y);
        }
    };
    constexpr uint32_t kPairHops = (1u << (NB + 1)) - 1;
    for (int k = f0; k < f1; k += 2) {
        float nxt[2 * SH];
        load_hop(nxt, (k + NB + 1) * H - a.pad);
        load_hop(nxt + SH, (k + NB + 2) * H - a.pad);
        const bool two = k + 1 < f1;
        float* ra = so + int64_t(k) * pa.ld_frame;
        float* rb = ra + pa.ld_frame;
        dev::pc v[E];
        if ((hopok & kPairHops) == kPairHops) {
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
            // Z[-k] of registers 0 .. 8 (the partners: registers 15 .. 7 of the partner lane)
            dev::pc zp[9];
#pragma unroll
            for (int d = 0; d < 9; ++d) {
                const float px = v[(15 - d) & 15].x, py = v[(15 - d) & 15].y;
                zp[d] = dev::pc_mk(bperm_f(partner, px), bperm_f(partner, py));
                if (lane == 0) zp[d] = v[(16 - d) & 15];
            }
            store_bins(ra, [&](int d) {
                return dev::pc_mk(0.5f * (v[d].x + zp[d].x), 0.5f * (v[d].y - zp[d].y));
            });
            if (two)
                store_bins(rb, [&](int d) {
                    return dev::pc_mk(0.5f * (v[d].y + zp[d].y), 0.5f * (zp[d].x - v[d].x));
                });
        } else {  // each frame alone, full input sanitize
            for (int p = 0; p < (two ? 2 : 1); ++p) {
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
                store_bins(p ? rb : ra, [&](int d) {  // (DC and Nyquist: imaginary part exactly 0)
                    return dev::pc_mk(v[d].x, (lane == 0 && (d == 0 || d == 8)) ? 0.0f : v[d].y);
                });
            }
        }
        hopok = (hopok | hop_ok<SH>(nxt, xlo, xhi) << (NB + 1) | hop_ok<SH>(nxt + SH, xlo, xhi) << (NB + 2)) >> 2;
#pragma unroll
        for (int m = 0; m < E + SH - 2 * SH; ++m) xin[m] = xin[m + 2 * SH];
#pragma unroll
        for (int q = 0; q < 2 * SH; ++q) xin[E - SH + q] = nxt[q];
    }
}

// ------------------------------------------------------------------ K_pair_istft
#ifndef CRLOT_PAIR_ISTFT_WAVES
#define CRLOT_PAIR_ISTFT_WAVES 3  // waves per SIMD without a mask (the mask rows' registers: 2)
#endif
template <int SH, bool MASK>
struct PairIstftOcc {  // (H = 512 at 3 waves spills: 2 measured 7 % faster)
    static constexpr int value = (MASK || SH == 8) ? 2 : CRLOT_PAIR_ISTFT_WAVES;
};
template <int SH, int NB, bool MASK>
__global__ __launch_bounds__(64 * kSW, (PairIstftOcc<SH, MASK>::value)) void k_pair_istft(const PairSpecArgs pa) {
    const FusedArgs& a = pa.f;
    constexpr int E = 16, N = 1024, H = 64 * SH, P2 = N / 2;
    static_assert(NB * SH == E, "N = NB * H");
    constexpr bool kFold = SH != 2;  // K_pair's OLA form (pair1k.hip kPairFoldWs): ws g staged
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    std::conditional_t<SH == 4, dev::PairTwReg, dev::PairTw> tw;
    spec_lds_setup(a, smem, a.t.wsn, kFold ? a.gain : 1.0f, tw, lane);
    const float* ws4 = reinterpret_cast<const float*>(smem + SpecLds::win);
    // the spectral gain by real bin (ones without one: x * 1 == x) over the twiddle tables
    __syncthreads();
    {
        float* gw_ = reinterpret_cast<float*>(smem + SpecLds::t1);
        for (int i = threadIdx.x; i <= P2; i += 64 * kSW) gw_[i] = a.t.gain ? a.t.gain[i] : 1.0f;
        __syncthreads();
    }
    const float* gl = reinterpret_cast<const float*>(smem + SpecLds::t1);
    dev::pc* buf = reinterpret_cast<dev::pc*>(smem + SpecLds::bufs) + wave * dev::kPairXbuf;
    const int gw = blockIdx.x * kSW + wave;
    if (gw >= a.n_streams * a.n_chunks) return;
    const int s = gw / a.n_chunks, c = gw - s * a.n_chunks;
    const int f0 = c * a.M, f1 = min(a.F, f0 + a.M);
    const int fs = max(0, f0 - (NB - 1)) & ~1;  // pairs start on even frames
    const __amdgpu_buffer_rsrc_t ry = dev::make_rsrc(a.y + int64_t(s) * a.ld_y, span_bytes(a.out_len, 1));
    const __amdgpu_buffer_rsrc_t rp = dev::make_rsrc(a.t.pden, uint32_t(a.ring_blocks * H) * 8u);
    const __amdgpu_buffer_rsrc_t ry_null = dev::make_rsrc(a.y, 0u);
    const float* sb = pa.sin + int64_t(s) * pa.ld_spec;
    const int pbl = dev::pair_bin_lane(lane);

    float acc[NB][SH];
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int q = 0; q < SH; ++q) acc[j][q] = 0.f;
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

    // The pair's rows (and mask rows) load one pair ahead in natural order (real bin
    // kr = lane + 64 i, i = 8: bin N/2, lane 0's), coalesced.  At the pair they are
    // stepped there -- (X g) m, re and im each, as K_istft / the oracle; DC and
    // Nyquist imaginary parts dropped -- checked for the paired regime, and put
    // in this wave's transpose buffer (free between transforms), from which each
    // lane reads its scrambled bins; frame k+1 past the last frame is zeros.
    constexpr int MI = 9;
    float2 ra_[MI], rb_[MI];
    float ma_[MASK ? MI : 1], mb_[MASK ? MI : 1];
    constexpr bool has_mask = MASK;
    const float* mrow0 = has_mask ? pa.mask.p + int64_t(s) * pa.mask.ld_stream : nullptr;
    auto load_rows = [&](int k) {
        const float2* ra = reinterpret_cast<const float2*>(sb + int64_t(k) * pa.ld_frame);
        const float2* rb = reinterpret_cast<const float2*>(sb + int64_t(k + 1) * pa.ld_frame);
        const bool two = k + 1 < a.F;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            const int kr = i < 8 ? lane + 64 * i : P2;
            ra_[i] = ld2(ra + kr);
            rb_[i] = two ? ld2(rb + kr) : make_float2(0.f, 0.f);
        }
        if constexpr (has_mask) {
            const float* m0 = mrow0 + int64_t(k) * pa.mask.ld_frame;
            const float* m1 = two ? m0 + pa.mask.ld_frame : m0;
#pragma unroll
            for (int i = 0; i < MI; ++i) {
                const int kr = i < 8 ? lane + 64 * i : P2;
                ma_[i] = m0[kr];
                mb_[i] = m1[kr];
            }
        }
    };
    // (A', B') of real bin kr at buf[kr] = A', buf[513 + kr] = B'; true when the pair keeps the paired regime
    auto stage = [&]() -> bool {
        bool bad = false;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            const int kr = i < 8 ? lane + 64 * i : P2;
            const float g = gl[kr];
            float ax = ra_[i].x * g, ay = ra_[i].y * g, bx = rb_[i].x * g, by = rb_[i].y * g;
            if constexpr (has_mask) {
                ax *= ma_[i];
                ay *= ma_[i];
                bx *= mb_[i];
                by *= mb_[i];
            }
            if (kr == 0 || kr == P2) ay = by = 0.0f;
            const float m = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(ax), __builtin_fabsf(ay)),
                                            __builtin_fmaxf(__builtin_fabsf(bx), __builtin_fabsf(by)));
            bad |= !(m <= 0x1p60f) | (ax != ax) | (ay != ay) | (bx != bx) | (by != by);  // (NaN, Inf, huge)
            if (i < 8 || lane == 0) {
                buf[kr] = dev::pc_mk(ax, ay);
                buf[P2 + 1 + kr] = dev::pc_mk(bx, by);
            }
        }
        return __builtin_amdgcn_ballot_w64(bad) == 0;
    };
    // bin kb = pbl + 64 d: real bin kb (d < 8) or N - kb (d >= 8, conjugated; d = 8 in
    // lane 0 is bin N/2 itself, whose imaginary part is zero either way)
    const dev::pc* const ca = buf + pbl;
    const dev::pc* const cb = buf - pbl;
    load_rows(fs);
    for (int k = fs; k < f1; k += 2) {
        const bool paired = stage();
        dev::wave_lds_fence();
        const bool more = k + 2 < f1;
        dev::pc v[E];
        if (paired) {
#pragma unroll
            for (int d = 0; d < E; ++d) {
                const dev::pc A = d < 8 ? ca[64 * d] : cb[N - 64 * d];
                const dev::pc B = d < 8 ? ca[P2 + 1 + 64 * d] : cb[P2 + 1 + N - 64 * d];
                v[d] = d < 8 ? dev::pc_mk(A.x - B.y, A.y + B.x) : dev::pc_mk(A.x + B.y, B.x - A.y);
            }
            dev::wave_lds_fence();  // (the bins read before the inverse's exchange rewrites buf)
            if (more) load_rows(k + 2);  // (in flight during the inverse and the OLA)
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
        } else {  // each frame alone, full sanitize (frame k+1's bins staged again after frame k's inverse)
            const int npass = min(2, f1 - k);
            for (int p = 0; p < npass; ++p) {
                if (p) {
                    dev::wave_lds_fence();
                    (void)stage();
                    dev::wave_lds_fence();
                }
#pragma unroll
                for (int d = 0; d < E; ++d) {
                    const dev::pc X = d < 8 ? ca[(p ? P2 + 1 : 0) + 64 * d] : cb[(p ? P2 + 1 : 0) + N - 64 * d];
                    v[d] = d < 8 ? X : dev::pc_mk(X.x, -X.y);
                }
                dev::wave_lds_fence();
                dev::pair_fft_inv(v, buf, tw, tw, lane);
                float dr[2 * SH];
                load_den<SH>(dr, rp, lane, (k + p) % a.ring_blocks);
                accumulate(v, false, false);
                emit(k + p, dr);
            }
            if (more) load_rows(k + 2);
        }
        dev::wave_lds_fence();  // (the inverse's last reads of buf before the next staging writes)
    }
}

// ------------------------------------------------------------------ N = 512 (fft_pair512.h)
// The same two kernels on K_pair512's transform: lane l holds z[l + 64 m], m < 8;
// the spectrum sits at bin q(l) + 64 d, q(l) = (l >> 3) + 8 (l & 7) (pair512_bin:
// an involution), so the partner of (l, d) is register 7 - d of lane
// q(64 - q(l)) and lane 0's partners its own registers (8 - d) mod 8.  Windows,
// twiddles in registers; LDS only the per-wave exchange buffer (576 complex),
// which also stages the inverse's rows (2 x 257 complex).
__device__ __forceinline__ int p512_q(int l) { return (l >> 3) + 8 * (l & 7); }
struct Spec512Lds {
    static constexpr size_t bytes = sizeof(dev::pc) * dev::kP512Buf * kSW;
};

template <int SH>
__global__ __launch_bounds__(64 * kSW) void k_pair512_stft(const PairSpecArgs pa) {
    const FusedArgs& a = pa.f;
    constexpr int E = 8, H = 64 * SH, NB = 8 / SH, P2 = 256;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    dev::pc* buf = reinterpret_cast<dev::pc*>(smem) + wave * dev::kP512Buf;
    const int gw = blockIdx.x * kSW + wave;
    if (gw >= a.n_streams * a.n_chunks) return;
    const int s = gw / a.n_chunks, c = gw - s * a.n_chunks;
    const int f0 = c * a.M, f1 = min(a.F, f0 + a.M);  // (M even)
    const __amdgpu_buffer_rsrc_t rx = dev::make_rsrc(a.x + int64_t(s) * a.ld_x, span_bytes(a.T, 1));
    float* so = pa.spec + int64_t(s) * pa.ld_spec;
    const float xlo = a.t.px_lo, xhi = a.t.px_hi;
    const int q = p512_q(lane);
    const int partner = p512_q((64 - q) & 63);
    dev::Pair512TwReg tw;
    dev::pair512_tw_load(tw, reinterpret_cast<const dev::pc*>(a.t.ptw), lane);
    float wa[E];
#pragma unroll
    for (int m = 0; m < E; ++m) wa[m] = a.t.wa[lane + 64 * m];
    auto load_hop = [&](float* dst, int origin) { load_hop1<SH>(dst, rx, lane, origin, a.T, a.pad_mode); };
    float xin[E + SH];
    uint32_t hopok = 0;
#pragma unroll
    for (int h = 0; h <= NB; ++h) {
        load_hop(xin + h * SH, (f0 + h) * H - a.pad);
        hopok |= hop_ok<SH>(xin + h * SH, xlo, xhi) << h;
    }
    auto store_bins = [&](float* row, auto valfn) {  // bins q + 64 d <= N/2: d < 4, and d = 4 in lane 0
        float2* r2 = reinterpret_cast<float2*>(row);
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const dev::pc o = valfn(d);
            st2(r2 + q + 64 * d, o.x, o.y);
        }
        if (lane == 0) {
            const dev::pc o = valfn(4);
            st2(r2 + P2, o.x, o.y);
        }
    };
    constexpr uint32_t kPairHops = (1u << (NB + 1)) - 1;
    for (int k = f0; k < f1; k += 2) {
        float nxt[2 * SH];
        load_hop(nxt, (k + NB + 1) * H - a.pad);
        load_hop(nxt + SH, (k + NB + 2) * H - a.pad);
        const bool two = k + 1 < f1;
        float* ra = so + int64_t(k) * pa.ld_frame;
        float* rb = ra + pa.ld_frame;
        dev::pc v[E];
        if ((hopok & kPairHops) == kPairHops) {
#pragma unroll
            for (int m = 0; m < E; ++m) v[m] = dev::pc_mk(xin[m] * wa[m], xin[m + SH] * wa[m]);
            dev::wave_lds_fence();
            dev::pair512_fwd(v, buf, tw, lane);
            dev::pc zp[5];
#pragma unroll
            for (int d = 0; d < 5; ++d) {
                const float px = v[(7 - d) & 7].x, py = v[(7 - d) & 7].y;
                zp[d] = dev::pc_mk(bperm_f(partner, px), bperm_f(partner, py));
                if (lane == 0) zp[d] = v[(8 - d) & 7];
            }
            store_bins(ra, [&](int d) {
                return dev::pc_mk(0.5f * (v[d].x + zp[d].x), 0.5f * (v[d].y - zp[d].y));
            });
            if (two)
                store_bins(rb, [&](int d) {
                    return dev::pc_mk(0.5f * (v[d].y + zp[d].y), 0.5f * (zp[d].x - v[d].x));
                });
        } else {  // each frame alone, full input sanitize
            for (int p = 0; p < (two ? 2 : 1); ++p) {
#pragma unroll
                for (int m = 0; m < E; ++m) v[m] = dev::pc_mk(dev::sanit((p ? xin[m + SH] : xin[m]) * wa[m]), 0.0f);
                dev::wave_lds_fence();
                dev::pair512_fwd(v, buf, tw, lane);
                store_bins(p ? rb : ra, [&](int d) {
                    return dev::pc_mk(v[d].x, (lane == 0 && (d == 0 || d == 4)) ? 0.0f : v[d].y);
                });
            }
        }
        hopok = (hopok | hop_ok<SH>(nxt, xlo, xhi) << (NB + 1) | hop_ok<SH>(nxt + SH, xlo, xhi) << (NB + 2)) >> 2;
#pragma unroll
        for (int m = 0; m < E + SH - 2 * SH; ++m) xin[m] = xin[m + 2 * SH];
#pragma unroll
        for (int qq = 0; qq < 2 * SH; ++qq) xin[E - SH + qq] = nxt[qq];
    }
}

template <int SH, int NB, bool MASK>
__global__ __launch_bounds__(64 * kSW) void k_pair512_istft(const PairSpecArgs pa) {
    const FusedArgs& a = pa.f;
    constexpr int E = 8, N = 512, H = 64 * SH, P2 = 256;
    static_assert(NB * SH == E, "N = NB * H");
    static_assert(SH >= 2, "den rows are read 16 bytes at a time");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    dev::pc* buf = reinterpret_cast<dev::pc*>(smem) + wave * dev::kP512Buf;
    const int gw = blockIdx.x * kSW + wave;
    if (gw >= a.n_streams * a.n_chunks) return;
    const int s = gw / a.n_chunks, c = gw - s * a.n_chunks;
    const int f0 = c * a.M, f1 = min(a.F, f0 + a.M);
    const int fs = max(0, f0 - (NB - 1)) & ~1;
    const __amdgpu_buffer_rsrc_t ry = dev::make_rsrc(a.y + int64_t(s) * a.ld_y, span_bytes(a.out_len, 1));
    const __amdgpu_buffer_rsrc_t rp = dev::make_rsrc(a.t.pden, uint32_t(a.ring_blocks * H) * 8u);
    const __amdgpu_buffer_rsrc_t ry_null = dev::make_rsrc(a.y, 0u);
    const float* sb = pa.sin + int64_t(s) * pa.ld_spec;
    const int q = p512_q(lane);
    dev::Pair512TwReg tw;
    dev::pair512_tw_load(tw, reinterpret_cast<const dev::pc*>(a.t.ptw), lane);
    float ws[E];
#pragma unroll
    for (int m = 0; m < E; ++m) ws[m] = a.t.wsn[lane + 64 * m] * a.gain;  // (ws g: K_pair512's OLA form)
    float acc[NB][SH];
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int qq = 0; qq < SH; ++qq) acc[j][qq] = 0.f;
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
    constexpr int MI = 5;  // natural-order bins lane + 64 i (i = 4: bin N/2, lane 0's)
    float2 ra_[MI], rb_[MI];
    float ma_[MASK ? MI : 1], mb_[MASK ? MI : 1];
    const float* mrow0 = MASK ? pa.mask.p + int64_t(s) * pa.mask.ld_stream : nullptr;
    auto load_rows = [&](int k) {
        const float2* ra = reinterpret_cast<const float2*>(sb + int64_t(k) * pa.ld_frame);
        const float2* rb = reinterpret_cast<const float2*>(sb + int64_t(k + 1) * pa.ld_frame);
        const bool two = k + 1 < a.F;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            const int kr = i < 4 ? lane + 64 * i : P2;
            ra_[i] = ld2(ra + kr);
            rb_[i] = two ? ld2(rb + kr) : make_float2(0.f, 0.f);
        }
        if constexpr (MASK) {
            const float* m0 = mrow0 + int64_t(k) * pa.mask.ld_frame;
            const float* m1 = two ? m0 + pa.mask.ld_frame : m0;
#pragma unroll
            for (int i = 0; i < MI; ++i) {
                const int kr = i < 4 ? lane + 64 * i : P2;
                ma_[i] = m0[kr];
                mb_[i] = m1[kr];
            }
        }
    };
    auto stage = [&]() -> bool {
        bool bad = false;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            const int kr = i < 4 ? lane + 64 * i : P2;
            const float g = a.t.gain ? a.t.gain[kr] : 1.0f;
            float ax = ra_[i].x * g, ay = ra_[i].y * g, bx = rb_[i].x * g, by = rb_[i].y * g;
            if constexpr (MASK) {
                ax *= ma_[i];
                ay *= ma_[i];
                bx *= mb_[i];
                by *= mb_[i];
            }
            if (kr == 0 || kr == P2) ay = by = 0.0f;
            const float m = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(ax), __builtin_fabsf(ay)),
                                            __builtin_fmaxf(__builtin_fabsf(bx), __builtin_fabsf(by)));
            bad |= !(m <= 0x1p60f) | (ax != ax) | (ay != ay) | (bx != bx) | (by != by);
            if (i < 4 || lane == 0) {
                buf[kr] = dev::pc_mk(ax, ay);
                buf[P2 + 1 + kr] = dev::pc_mk(bx, by);
            }
        }
        return __builtin_amdgcn_ballot_w64(bad) == 0;
    };
    const dev::pc* const ca = buf + q;
    const dev::pc* const cb = buf - q;
    load_rows(fs);
    for (int k = fs; k < f1; k += 2) {
        const bool paired = stage();
        dev::wave_lds_fence();
        const bool more = k + 2 < f1;
        dev::pc v[E];
        if (paired) {
#pragma unroll
            for (int d = 0; d < E; ++d) {
                const dev::pc A = d < 4 ? ca[64 * d] : cb[N - 64 * d];
                const dev::pc B = d < 4 ? ca[P2 + 1 + 64 * d] : cb[P2 + 1 + N - 64 * d];
                v[d] = d < 4 ? dev::pc_mk(A.x - B.y, A.y + B.x) : dev::pc_mk(A.x + B.y, B.x - A.y);
            }
            dev::wave_lds_fence();
            if (more) load_rows(k + 2);
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
        } else {
            const int npass = min(2, f1 - k);
            for (int p = 0; p < npass; ++p) {
                if (p) {
                    dev::wave_lds_fence();
                    (void)stage();
                    dev::wave_lds_fence();
                }
#pragma unroll
                for (int d = 0; d < E; ++d) {
                    const dev::pc X = d < 4 ? ca[(p ? P2 + 1 : 0) + 64 * d] : cb[(p ? P2 + 1 : 0) + N - 64 * d];
                    v[d] = d < 4 ? X : dev::pc_mk(X.x, -X.y);
                }
                dev::wave_lds_fence();
                dev::pair512_inv(v, buf, tw, lane);
                float dr[2 * SH];
                load_den<SH>(dr, rp, lane, (k + p) % a.ring_blocks);
                accumulate(v, false, false);
                emit(k + p, dr);
            }
            if (more) load_rows(k + 2);
        }
        dev::wave_lds_fence();
    }
}

template <typename K>
hipError_t launch_spec(K kernel, const PairSpecArgs& a, int64_t walkers, hipStream_t stream) {
    hipError_t e = set_lds(kernel, SpecLds::bytes);
    if (e != hipSuccess) return e;
    const int64_t grid = (walkers + kSW - 1) / kSW;
    hipLaunchKernelGGL(kernel, dim3(unsigned(grid)), dim3(64 * kSW), SpecLds::bytes, stream, a);
    return hipGetLastError();
}

}  // namespace

int pair_spec_walkers_per_cu(int n) {
    if (n >= 2048) return pair_wg_walkers_per_cu(n);
    static const int v = [] {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void*>(k_pair_istft<4, 4, false>),
                                                         64 * kSW, SpecLds::bytes) != hipSuccess ||
            nb <= 0)
            nb = 1;
        return nb * kSW;
    }();
    return v;
}

template <typename K>
hipError_t launch_spec512(K kernel, const PairSpecArgs& a, int64_t walkers, hipStream_t stream) {
    const int64_t grid = (walkers + kSW - 1) / kSW;
    hipLaunchKernelGGL(kernel, dim3(unsigned(grid)), dim3(64 * kSW), Spec512Lds::bytes, stream, a);
    return hipGetLastError();
}

hipError_t launch_pair_stft(int n, int h, const PairSpecArgs& a, int64_t walkers, hipStream_t stream) {
    if (n >= 2048) return launch_pairwg_stft(n, h, a, walkers, stream);
    note_launch(CRLOT_K_PAIR_STFT, (walkers + kSW - 1) / kSW);
    if (n == 512) {
        switch (h) {
            case 128: return launch_spec512(k_pair512_stft<2>, a, walkers, stream);
            case 256: return launch_spec512(k_pair512_stft<4>, a, walkers, stream);
            default: return hipErrorInvalidValue;
        }
    }
    switch (h) {
        case 128: return launch_spec(k_pair_stft<2>, a, walkers, stream);
        case 256: return launch_spec(k_pair_stft<4>, a, walkers, stream);
        case 512: return launch_spec(k_pair_stft<8>, a, walkers, stream);
        default: return hipErrorInvalidValue;
    }
}

template <bool MASK>
hipError_t pair_istft_m(int h, const PairSpecArgs& a, int64_t walkers, hipStream_t stream) {
    switch (h) {
        case 128: return launch_spec(k_pair_istft<2, 8, MASK>, a, walkers, stream);
        case 256: return launch_spec(k_pair_istft<4, 4, MASK>, a, walkers, stream);
        case 512: return launch_spec(k_pair_istft<8, 2, MASK>, a, walkers, stream);
        default: return hipErrorInvalidValue;
    }
}

template <bool MASK>
hipError_t pair512_istft_m(int h, const PairSpecArgs& a, int64_t walkers, hipStream_t stream) {
    switch (h) {
        case 128: return launch_spec512(k_pair512_istft<2, 4, MASK>, a, walkers, stream);
        case 256: return launch_spec512(k_pair512_istft<4, 2, MASK>, a, walkers, stream);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_pair_istft(int n, int h, const PairSpecArgs& a, int64_t walkers, hipStream_t stream) {
    if (n >= 2048) return launch_pairwg_istft(n, h, a, walkers, stream);
    note_launch(CRLOT_K_PAIR_ISTFT, (walkers + kSW - 1) / kSW);
    if (n == 512)
        return a.mask.p ? pair512_istft_m<true>(h, a, walkers, stream) : pair512_istft_m<false>(h, a, walkers, stream);
    return a.mask.p ? pair_istft_m<true>(h, a, walkers, stream) : pair_istft_m<false>(h, a, walkers, stream);
}

}  // namespace fk
}  // namespace crlot
