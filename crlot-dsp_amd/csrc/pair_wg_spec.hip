// pair_wg_spec.hip -- the spectral entries and the masked round trip as frame
// pairs at N = 4096 and 2048, one workgroup per chunk (the transforms of
// K_pair4k / K_pair2k: fft_pair4k.h, 256 lanes; fft_pair2k.h, 128 lanes):
//   K_pair_stft   k_pairwg_stft<G,SH>        (crlot_stft)
//   K_pair_istft  k_pairwg_istft<G,SH,NB,MASK> (crlot_istft_ola)
//   K_pair_mask   k_pairwg_mask<G,SH,NB,GAIN>  (crlot_roundtrip with a per-frame mask)
//
// Frames a = 2j and b = 2j+1 of a stream share one complex transform
// z = a w + i b w, as in pair_stft.hip / pair_mask.hip (N = 1024, 512), but the
// bins of these transforms are spread over the workgroup's waves, so every step
// that needs a bin's partner Z[N-k] goes through LDS: the spectrum is staged in
// natural bin order (padded: bin k at k + k/16, which keeps the 16-lane groups of
// a b64 access on distinct banks for both the scrambled and the natural side),
// and each lane works on its own natural bins k = t + L i (and N/2 in lane 0):
//   stft:  A[k] = (Z[k] + conj Z[-k]) / 2,  B[k] = (Z[k] - conj Z[-k]) / 2i,
//          stored coalesced (rows of N/2+1 complex);
//   istft: the stepped half spectra A' = X_a g m_a, B' = X_b g m_b staged by real
//          bin, read back in the transform's scrambled order as Z = A' + i B'
//          (conjugated above N/2), ONE inverse for both frames, then K_pair4k's
//          OLA stage and division;
//   mask:  Z'[k] = c1 Z[k] + c2 conj Z[-k] with c1 = (Ga + Gb)/2, c2 = (Ga - Gb)/2
//          (Ga = g m_a, Gb = g m_b), computed in place for the pair {k, N-k} by the
//          one lane that owns it: under a mask of ones c1 = g and c2 = 0, so the
//          walk is K_pair4k / K_pair2k's own (same twiddle forms, same OLA form:
//          bit for bit).
// Regimes as the per-wave pair kernels (pair_stft.hip, pair_mask.hip), agreed by
// the whole workgroup (its transforms exchange data across the waves): each wave
// posts its verdict in LDS before a barrier the walk needs anyway, and every lane
// reads the four (or two) verdicts after it.
#include <algorithm>
#include <type_traits>

#include "fft_pair2k.h"
#include "fft_pair4k.h"
#include "fused_common.h"

namespace crlot {
namespace fk {

namespace {

// Twiddle stages in the two forms the walkers use (fft_pair.h): explicit
// products (Tw15C) or the FMA form fused into the inverse's radix-16 (Tw15F).
struct Tw15C {
    dev::pc w[15];
};
__device__ __forceinline__ void tw_fwd(dev::pc (&v)[16], const Tw15C& w) {
#pragma unroll
    for (int k = 1; k < 16; ++k) v[k] = dev::pc_mul(v[k], w.w[k - 1]);
}
__device__ __forceinline__ void tw_fwd(dev::pc (&v)[16], const dev::Tw15F& w) { dev::tw15_apply_fwd(v, w); }
// conjugate twiddles, then the inverse radix-16
__device__ __forceinline__ void tw_inv16(dev::pc (&v)[16], const Tw15C& w) {
#pragma unroll
    for (int k = 1; k < 16; ++k) v[k] = dev::pc_mulc(v[k], w.w[k - 1]);
    dev::pdft16<true>(v);
}
__device__ __forceinline__ void tw_inv16(dev::pc (&v)[16], const dev::Tw15F& w) { dev::tw15_pdft16_inv(v, w); }
template <typename WF>
__device__ __forceinline__ void tw_load15(Tw15C& tw, WF w) {
#pragma unroll
    for (int k = 1; k < 16; ++k) tw.w[k - 1] = w(k);
}
template <typename WF>
__device__ __forceinline__ void tw_load15(dev::Tw15F& tw, WF w) {
    dev::tw15_load(tw, w);
}

// The two workgroup transforms with their self-synchronised exchanges (the
// two-regime walkers' forms -- fft_pair4k.h pair4k_fwd / _inv, fft_pair2k.h
// pair2k_fwd / _inv, step for step -- every exchange bracketed by barriers, so
// the exchange buffer is free for the staging between transforms).  The
// first-stage twiddles (per lane) stay in registers; the second-stage ones
// depend on the lane's low bits only (16 / 8 sets) and are read from LDS.
// T1 / T2: the forms of K_pair4k / K_pair2k for (SH, GAIN), or the explicit
// products (CLASSIC) where no bit-identity with those walkers is at stake.
struct W4k {
    static constexpr int N = 4096, L = 256, XB = dev::kP4Xbuf, TB = dev::kPairXbuf, X2 = 16;
    template <int SH, bool GAIN>
    using T1 = std::conditional_t<SH == 4 && !GAIN, dev::Tw15F, Tw15C>;  // (Pair4kTwFor)
    template <int SH, bool GAIN>
    using T2 = T1<SH, GAIN>;
    static __device__ __forceinline__ int bin(int t, int d) { return dev::pair4k_bin(t, d); }
    template <typename A, typename B>
    static __device__ __forceinline__ void tw_load(A& w1, B* w2s, const float* g, int t) {
        const dev::pc* gp = reinterpret_cast<const dev::pc*>(g);
        tw_load15(w1, [&](int k) { return gp[(k - 1) * 256 + t]; });
        if (t < X2) {
            B w2;
            tw_load15(w2, [&](int k) { return gp[15 * 256 + (k - 1) * 16 + t]; });
            w2s[t] = w2;
        }
    }
    static __device__ __forceinline__ int x2(int t) { return t & 15; }
    template <typename A, typename B>
    static __device__ __forceinline__ void fwd(dev::pc (&v)[16], dev::pc* xb, dev::pc* tb, const A& w1, const B& w2,
                                               int t) {
        dev::pdft16<false>(v);
        tw_fwd(v, w1);
        dev::pair4k_xchg_fwd(v, xb, t);
        dev::pdft16<false>(v);
        tw_fwd(v, w2);
        dev::transpose16(v, tb, t & 63);
        dev::pdft16<false>(v);
    }
    template <typename A, typename B>
    static __device__ __forceinline__ void inv(dev::pc (&v)[16], dev::pc* xb, dev::pc* tb, const A& w1, const B& w2,
                                               int t) {
        dev::pdft16<true>(v);
        dev::transpose16(v, tb, t & 63);
        tw_inv16(v, w2);
        dev::pair4k_xchg_inv(v, xb, t);
        tw_inv16(v, w1);
    }
};
struct W2k {
    static constexpr int N = 2048, L = 128, XB = dev::kP2Xbuf, TB = dev::kP2Tbuf, X2 = 8;
    template <int SH, bool GAIN>
    using T1 = std::conditional_t<SH == 4, dev::Tw15F, Tw15C>;  // (Pair2kTwFor: the gain does not matter)
    template <int SH, bool GAIN>
    using T2 = Tw15C;
    static __device__ __forceinline__ int bin(int t, int d) { return dev::pair2k_bin(t, d); }
    template <typename A, typename B>
    static __device__ __forceinline__ void tw_load(A& w1, B* w2s, const float* g, int t) {
        const dev::pc* gp = reinterpret_cast<const dev::pc*>(g);
        tw_load15(w1, [&](int k) { return gp[(k - 1) * 128 + t]; });
        if (t < X2) {
            B w2;
            tw_load15(w2, [&](int k) { return gp[15 * 128 + (k - 1) * 8 + t]; });
            w2s[t] = w2;
        }
    }
    static __device__ __forceinline__ int x2(int t) { return t & 7; }
    template <typename A, typename B>
    static __device__ __forceinline__ void fwd(dev::pc (&v)[16], dev::pc* xb, dev::pc* tb, const A& w1, const B& w2,
                                               int t) {
        dev::pdft16<false>(v);
        tw_fwd(v, w1);
        dev::pair2k_xchg_fwd(v, xb, t);
        dev::pdft16<false>(v);
        tw_fwd(v, w2);
        dev::pair2k_t8(v, tb, t & 63);
        dev::pdft8_halves<false>(v);
    }
    template <typename A, typename B>
    static __device__ __forceinline__ void inv(dev::pc (&v)[16], dev::pc* xb, dev::pc* tb, const A& w1, const B& w2,
                                               int t) {
        dev::pdft8_halves<true>(v);
        dev::pair2k_t8(v, tb, t & 63);
        tw_inv16(v, w2);
        dev::pair2k_xchg_inv(v, xb, t);
        tw_inv16(v, w1);
    }
};
// The twiddles of one walker: first stage in registers, second stage in LDS.
template <typename G, typename A, typename B>
struct WgTw {
    A w1;
    const B* w2;
    __device__ WgTw(B* w2s, const float* g, int t) : w2(w2s + G::x2(t)) { G::tw_load(w1, w2s, g, t); }
    __device__ __forceinline__ void fwd(dev::pc (&v)[16], dev::pc* xb, dev::pc* tb, int t) const {
        G::fwd(v, xb, tb, w1, *w2, t);
    }
    __device__ __forceinline__ void inv(dev::pc (&v)[16], dev::pc* xb, dev::pc* tb, int t) const {
        G::inv(v, xb, tb, w1, *w2, t);
    }
};
// staged bin k at k + k/16 (complex units)
__device__ __forceinline__ constexpr int spad(int k) { return k + (k >> 4); }

// LDS: the exchange buffer, grown to hold the staging (the spectrum of a pair, or
// the two stepped half spectra A' | B'), the per-wave transpose buffers, the verdicts.
template <typename G>
struct WgLds {
    static constexpr int half = spad(G::N / 2) + 1;  // A' of bins 0 .. N/2, then B'
    static constexpr int xs = std::max(std::max(G::XB, spad(G::N - 1) + 1), 2 * half);
    static constexpr size_t tb = sizeof(dev::pc) * xs;
    static constexpr size_t votes = tb + sizeof(dev::pc) * G::TB * (G::L / 64);
    static constexpr size_t w2 = votes + 32;  // (two sets of verdicts)
    static constexpr size_t bytes = w2 + sizeof(dev::Tw15F) * G::X2;  // (>= a Tw15C)
};
static_assert(sizeof(dev::Tw15F) >= sizeof(Tw15C), "w2 table");

template <typename G>
struct WgSmem {
    dev::pc* xb;
    dev::pc* tb;
    uint32_t* votes;
    char* w2;
    __device__ WgSmem(char* smem, int wave)
        : xb(reinterpret_cast<dev::pc*>(smem)),
          tb(reinterpret_cast<dev::pc*>(smem + WgLds<G>::tb) + wave * G::TB),
          votes(reinterpret_cast<uint32_t*>(smem + WgLds<G>::votes)),
          w2(smem + WgLds<G>::w2) {}
    // post this wave's verdict (wave-uniform) in set `set`, before a barrier
    __device__ __forceinline__ void post(int wave, int lane, bool ok, int set = 0) {
        if (lane == 0) votes[4 * set + wave] = ok ? 1u : 0u;
    }
    // after that barrier: every wave's verdict was ok
    __device__ __forceinline__ bool all(int set = 0) const {
        uint32_t v = 1u;
#pragma unroll
        for (int w = 0; w < G::L / 64; ++w) v &= votes[4 * set + w];
        return v != 0u;
    }
};

// hop of H = L SH samples at `origin`, lane t holding samples origin + t + L q,
// with the plan's padding outside [0, T)
template <int L, int SH>
__device__ __forceinline__ void load_hop_wg(float* dst, __amdgpu_buffer_rsrc_t rx, int t, int origin, int T,
                                            int mode) {
    constexpr int H = L * SH;
    if (origin >= 0 && origin + H <= T) {
#pragma unroll
        for (int q = 0; q < SH; ++q) dst[q] = dev::bload1(rx, t * 4, origin * 4 + q * (4 * L));
    } else {
#pragma unroll
        for (int q = 0; q < SH; ++q) dst[q] = fetch_x(rx, origin + t + L * q, T, mode);
    }
}
// den | rden of block b for lane t (DevTables::pden4: [block][L][den SH | rden SH])
template <int L, int SH>
__device__ __forceinline__ void den_wg(float (&dr)[2 * SH], __amdgpu_buffer_rsrc_t rp, int t, int b) {
#pragma unroll
    for (int j = 0; j < 2 * SH / 4; ++j) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rp, t * (8 * SH), b * (8 * L * SH) + 16 * j, 0);
        const unsigned u0 = v[0], u1 = v[1], u2 = v[2], u3 = v[3];  // (see bload2)
        dr[4 * j] = __builtin_bit_cast(float, u0);
        dr[4 * j + 1] = __builtin_bit_cast(float, u1);
        dr[4 * j + 2] = __builtin_bit_cast(float, u2);
        dr[4 * j + 3] = __builtin_bit_cast(float, u3);
    }
}

// The OLA stage of the two-regime walkers (k_stft_ola_pair4k / _pair2k): ws g
// folded, ascending k, Markstein's division with the per-wave IEEE fallback,
// warm-up blocks dropped.
template <typename G, int SH, int NB>
struct WgOla {
    static constexpr int E = 16, L = G::L, H = L * SH;
    float acc[NB][SH];
    __device__ __forceinline__ void clear() {
#pragma unroll
        for (int j = 0; j < NB; ++j)
#pragma unroll
            for (int q = 0; q < SH; ++q) acc[j][q] = 0.f;
    }
    __device__ __forceinline__ void add(const dev::pc (&v)[E], const float (&ws)[E], bool imag, bool paired) {
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const float x = imag ? v[m].y : v[m].x;
            const float o = paired ? dev::sanit_scaled_finite<G::N>(x) : dev::sanit_scaled<G::N>(x);
            float& r = acc[m / SH][m % SH];
            r = __builtin_fmaf(o, ws[m], r);
        }
    }
    __device__ __forceinline__ void emit(int k, int f0, const float (&dr)[2 * SH], __amdgpu_buffer_rsrc_t ry,
                                         __amdgpu_buffer_rsrc_t ry_null, int t) {
        float mx = 0.0f, mn = 0x1p127f;
#pragma unroll
        for (int q = 0; q < SH; ++q) {
            const float u = __builtin_fabsf(acc[0][q]);
            mx = __builtin_fmaxf(mx, u);
            mn = __builtin_fminf(mn, u);
        }
        const bool ok = (mx <= 0x1p64f) & ((mn >= 0x1p-64f) | (mx == 0.0f));
        float o[SH];
#pragma unroll
        for (int q = 0; q < SH; ++q) o[q] = mk_div(acc[0][q], dr[q], dr[SH + q]);
        if (__builtin_amdgcn_ballot_w64(!ok) != 0) {
#pragma unroll
            for (int q = 0; q < SH; ++q) o[q] = acc[0][q] / dr[q];
        }
        const __amdgpu_buffer_rsrc_t rk = k >= f0 ? ry : ry_null;
#pragma unroll
        for (int q = 0; q < SH; ++q)
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o[q]), rk, t * 4,
                                                  k * (4 * H) + q * (4 * L), 0);
#pragma unroll
        for (int j = 0; j < NB - 1; ++j)
#pragma unroll
            for (int q = 0; q < SH; ++q) acc[j][q] = acc[j + 1][q];
#pragma unroll
        for (int q = 0; q < SH; ++q) acc[NB - 1][q] = 0.f;
    }
};

// ------------------------------------------------------------------ K_pair_stft
template <typename G, int SH>
__global__ __launch_bounds__(G::L, 2) void k_pairwg_stft(const PairSpecArgs pa) {
    const FusedArgs& a = pa.f;
    constexpr int E = 16, N = G::N, L = G::L, H = L * SH, NB = E / SH, P2 = N / 2, NI = P2 / L;
    static_assert(NB * SH == E && NI * L == P2, "geometry");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    WgSmem<G> sm(smem, wave);
    const int s = blockIdx.x / a.n_chunks, c = blockIdx.x - s * a.n_chunks;
    const int f0 = c * a.M, f1 = min(a.F, f0 + a.M);  // (M even: chunks start on even frames)
    const __amdgpu_buffer_rsrc_t rx = dev::make_rsrc(a.x + int64_t(s) * a.ld_x, span_bytes(a.T, 1));
    float* so = pa.spec + int64_t(s) * pa.ld_spec;
    const WgTw<G, Tw15C, Tw15C> tw(reinterpret_cast<Tw15C*>(sm.w2), a.t.ptw4, t);  // (explicit products)
    float wa[E];
#pragma unroll
    for (int m = 0; m < E; ++m) wa[m] = a.t.wa[t + L * m];
    const float xlo = a.t.px_lo, xhi = a.t.px_hi;
    auto load_hop = [&](float* dst, int origin) { load_hop_wg<L, SH>(dst, rx, t, origin, a.T, a.pad_mode); };

    float xin[E + SH];  // hops k .. k+NB of the pair at k
    uint32_t hopok = 0;
#pragma unroll
    for (int h = 0; h <= NB; ++h) {
        load_hop(xin + h * SH, (f0 + h) * H - a.pad);
        hopok |= hop_ok<SH>(xin + h * SH, xlo, xhi) << h;
    }
    constexpr uint32_t kPairHops = (1u << (NB + 1)) - 1;
    sm.post(wave, lane, (hopok & kPairHops) == kPairHops);
    __syncthreads();
    bool paired = sm.all();
    for (int k = f0; k < f1; k += 2) {
        float nxt[2 * SH];
        load_hop(nxt, (k + NB + 1) * H - a.pad);
        load_hop(nxt + SH, (k + NB + 2) * H - a.pad);
        const bool two = k + 1 < f1;
        float2* ra = reinterpret_cast<float2*>(so + int64_t(k) * pa.ld_frame);
        float2* rb = reinterpret_cast<float2*>(so + int64_t(k + 1) * pa.ld_frame);
        auto pass = [&](auto pc_) {  // P = 0 / 1: frame k / k+1 alone; paired: both (P = 0)
            constexpr int P = decltype(pc_)::value;
            dev::pc v[E];
#pragma unroll
            for (int m = 0; m < E; ++m)
                v[m] = paired ? dev::pc_mk(xin[m] * wa[m], xin[m + SH] * wa[m])
                              : dev::pc_mk(dev::sanit(xin[m + P * SH] * wa[m]), 0.0f);
            tw.fwd(v, sm.xb, sm.tb, t);
#pragma unroll
            for (int d = 0; d < E; ++d) sm.xb[spad(G::bin(t, d))] = v[d];
            __syncthreads();
#pragma unroll
            for (int i = 0; i <= NI; ++i) {
                const int kr = i < NI ? t + L * i : P2;
                const bool on = i < NI || t == 0;
                const dev::pc z = sm.xb[spad(kr)];
                if (paired) {
                    const dev::pc zp = sm.xb[spad((N - kr) & (N - 1))];
                    if (on) ra[kr] = make_float2(0.5f * (z.x + zp.x), 0.5f * (z.y - zp.y));
                    if (on && two) rb[kr] = make_float2(0.5f * (z.y + zp.y), 0.5f * (zp.x - z.x));
                } else if (on) {  // (DC and Nyquist: imaginary part exactly 0, as kiss_fftr writes them)
                    (P ? rb : ra)[kr] = make_float2(z.x, (kr == 0 || kr == P2) ? 0.0f : z.y);
                }
            }
        };
        pass(std::integral_constant<int, 0>());
        if (!paired && two) {
            __syncthreads();  // (pass 0's staged reads before pass 1's exchange rewrites xb)
            pass(std::integral_constant<int, 1>());
        }
        // the next pair's regime; the barrier also keeps the staged reads ahead of
        // the next exchange's writes
        hopok = (hopok | hop_ok<SH>(nxt, xlo, xhi) << (NB + 1) | hop_ok<SH>(nxt + SH, xlo, xhi) << (NB + 2)) >> 2;
        sm.post(wave, lane, (hopok & kPairHops) == kPairHops);
        __syncthreads();
        paired = sm.all();
#pragma unroll
        for (int m = 0; m < E + SH - 2 * SH; ++m) xin[m] = xin[m + 2 * SH];
#pragma unroll
        for (int q = 0; q < 2 * SH; ++q) xin[E - SH + q] = nxt[q];
    }
}

// ------------------------------------------------------------------ K_pair_istft
template <typename G, int SH, int NB, bool MASK>
__global__ __launch_bounds__(G::L, 2) void k_pairwg_istft(const PairSpecArgs pa) {
    const FusedArgs& a = pa.f;
    constexpr int E = 16, N = G::N, L = G::L, P2 = N / 2, NI = P2 / L, OB = WgLds<G>::half;
    static_assert(NB * SH == E && NI * L == P2, "geometry");
    static_assert(SH >= 2, "den rows are read 16 bytes at a time");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    WgSmem<G> sm(smem, wave);
    const int s = blockIdx.x / a.n_chunks, c = blockIdx.x - s * a.n_chunks;
    const int f0 = c * a.M, f1 = min(a.F, f0 + a.M);
    const int fs = max(0, f0 - (NB - 1)) & ~1;  // pairs start on even frames
    const __amdgpu_buffer_rsrc_t ry = dev::make_rsrc(a.y + int64_t(s) * a.ld_y, span_bytes(a.out_len, 1));
    const __amdgpu_buffer_rsrc_t ry_null = dev::make_rsrc(a.y, 0u);
    const __amdgpu_buffer_rsrc_t rp = dev::make_rsrc(a.t.pden4, uint32_t(a.ring_blocks * L * SH) * 8u);
    const float* sb = pa.sin + int64_t(s) * pa.ld_spec;
    const WgTw<G, Tw15C, Tw15C> tw(reinterpret_cast<Tw15C*>(sm.w2), a.t.ptw4, t);  // (explicit products)
    float ws[E];
#pragma unroll
    for (int m = 0; m < E; ++m) ws[m] = a.t.wsn[t + L * m] * a.gain;  // (ws g: the two-regime walkers' OLA form)
    WgOla<G, SH, NB> ola;
    ola.clear();

    // The pair's rows (and mask rows), natural bins kr = t + L i (i = NI: bin N/2,
    // lane 0's), loaded coalesced at the pair (not prefetched: registers; the other
    // workgroup of the CU covers the wait), stepped when staged -- (X g) m,
    // re and im each, as K_istft / the oracle; DC and Nyquist imaginary parts
    // dropped -- and checked for the paired regime; frame k+1 past the last: zeros.
    float2 ra_[NI + 1], rb_[NI + 1];
    float ma_[MASK ? NI + 1 : 1], mb_[MASK ? NI + 1 : 1];
    const float* mrow0 = MASK ? pa.mask.p + int64_t(s) * pa.mask.ld_stream : nullptr;
    auto load_rows = [&](int k) {
        const float2* ra = reinterpret_cast<const float2*>(sb + int64_t(k) * pa.ld_frame);
        const float2* rb = reinterpret_cast<const float2*>(sb + int64_t(k + 1) * pa.ld_frame);
        const bool two = k + 1 < a.F;
#pragma unroll
        for (int i = 0; i <= NI; ++i) {
            const int kr = i < NI ? t + L * i : P2;
            const bool on = i < NI || t == 0;
            ra_[i] = on ? ra[kr] : make_float2(0.f, 0.f);
            rb_[i] = on && two ? rb[kr] : make_float2(0.f, 0.f);
        }
        if constexpr (MASK) {
            const float* m0 = mrow0 + int64_t(k) * pa.mask.ld_frame;
            const float* m1 = two ? m0 + pa.mask.ld_frame : m0;
#pragma unroll
            for (int i = 0; i <= NI; ++i) {
                const int kr = i < NI ? t + L * i : P2;
                const bool on = i < NI || t == 0;
                ma_[i] = on ? m0[kr] : 0.f;
                mb_[i] = on ? m1[kr] : 0.f;
            }
        }
    };
    // (A', B') of real bin kr at xb[spad(kr)], xb[OB + spad(kr)]; true when this lane keeps the paired regime
    auto stage = [&]() -> bool {
        bool bad = false;
#pragma unroll
        for (int i = 0; i <= NI; ++i) {
            const int kr = i < NI ? t + L * i : P2;
            const bool on = i < NI || t == 0;  // (the others hold zeros)
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
            bad |= !(m <= 0x1p60f) | (ax != ax) | (ay != ay) | (bx != bx) | (by != by);  // (NaN, Inf, huge)
            if (on) {
                sm.xb[spad(kr)] = dev::pc_mk(ax, ay);
                sm.xb[OB + spad(kr)] = dev::pc_mk(bx, by);
            }
        }
        return !bad;
    };
    for (int k = fs; k < f1; k += 2) {
        load_rows(k);
        sm.post(wave, lane, __builtin_amdgcn_ballot_w64(!stage()) == 0);
        __syncthreads();
        const bool paired = sm.all();
        dev::pc v[E];
        if (paired) {
#pragma unroll
            for (int d = 0; d < E; ++d) {  // bin kb: real bin kb (kb <= N/2) or N - kb, conjugated
                const int kb = G::bin(t, d);
                const bool lo = kb <= P2;
                const int j = spad(lo ? kb : N - kb);
                const dev::pc A = sm.xb[j], B = sm.xb[OB + j];
                v[d] = lo ? dev::pc_mk(A.x - B.y, A.y + B.x) : dev::pc_mk(A.x + B.y, B.x - A.y);
            }
            __syncthreads();  // (the staged reads before the inverse's exchange rewrites xb)
            tw.inv(v, sm.xb, sm.tb, t);
            float dr0[2 * SH], dr1[2 * SH];
            den_wg<L, SH>(dr0, rp, t, k % a.ring_blocks);
            den_wg<L, SH>(dr1, rp, t, (k + 1) % a.ring_blocks);
            ola.add(v, ws, false, true);
            ola.emit(k, f0, dr0, ry, ry_null, t);
            if (k + 1 < f1) {
                ola.add(v, ws, true, true);
                ola.emit(k + 1, f0, dr1, ry, ry_null, t);
            }
        } else {  // each frame alone, full sanitize (frame k+1's bins staged again after frame k's inverse)
            const int npass = min(2, f1 - k);
            for (int p = 0; p < npass; ++p) {
                if (p) {
                    (void)stage();
                    __syncthreads();
                }
#pragma unroll
                for (int d = 0; d < E; ++d) {
                    const int kb = G::bin(t, d);
                    const bool lo = kb <= P2;
                    const dev::pc X = sm.xb[(p ? OB : 0) + spad(lo ? kb : N - kb)];
                    v[d] = lo ? X : dev::pc_mk(X.x, -X.y);
                }
                __syncthreads();
                tw.inv(v, sm.xb, sm.tb, t);
                float dr[2 * SH];
                den_wg<L, SH>(dr, rp, t, (k + p) % a.ring_blocks);
                ola.add(v, ws, false, false);
                ola.emit(k + p, f0, dr, ry, ry_null, t);
            }
        }
        // (the next staging writes xb behind the inverse's last barrier)
    }
}

// ------------------------------------------------------------------ K_pair_mask
template <typename G, int SH, int NB, bool GAIN>
__global__ __launch_bounds__(G::L, 2) void k_pairwg_mask(const PairSpecArgs pa) {
    const FusedArgs& a = pa.f;
    constexpr int E = 16, N = G::N, L = G::L, H = L * SH, P2 = N / 2, NI = P2 / L;
    static_assert(NB * SH == E && NI * L == P2, "geometry");
    static_assert(SH >= 2, "den rows are read 16 bytes at a time");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    WgSmem<G> sm(smem, wave);
    const int s = blockIdx.x / a.n_chunks, c = blockIdx.x - s * a.n_chunks;
    const int f0 = c * a.M, f1 = min(a.F, f0 + a.M);
    const int fs = max(0, f0 - (NB - 1)) & ~1;  // pairs start on even frames
    const __amdgpu_buffer_rsrc_t rx = dev::make_rsrc(a.x + int64_t(s) * a.ld_x, span_bytes(a.T, 1));
    const __amdgpu_buffer_rsrc_t ry = dev::make_rsrc(a.y + int64_t(s) * a.ld_y, span_bytes(a.out_len, 1));
    const __amdgpu_buffer_rsrc_t ry_null = dev::make_rsrc(a.y, 0u);
    const __amdgpu_buffer_rsrc_t rp = dev::make_rsrc(a.t.pden4, uint32_t(a.ring_blocks * H) * 8u);
    const float xlo = a.t.px_lo, xhi = a.t.px_hi * 0x1p-20f;  // (mask values up to 2^20)
    using T2 = typename G::template T2<SH, GAIN>;  // (the two-regime walker's twiddle forms for this plan)
    const WgTw<G, typename G::template T1<SH, GAIN>, T2> tw(reinterpret_cast<T2*>(sm.w2), a.t.ptw4, t);
    float ws[E];  // (the analysis window is read from L2 at each pair: registers)
#pragma unroll
    for (int m = 0; m < E; ++m) ws[m] = a.t.wsn[t + L * m] * a.gain;
    const float* wag = a.t.wa + t;
    WgOla<G, SH, NB> ola;
    ola.clear();
    auto load_hop = [&](float* dst, int origin) { load_hop_wg<L, SH>(dst, rx, t, origin, a.T, a.pad_mode); };
    const float* mrow0 = pa.mask.p + int64_t(s) * pa.mask.ld_stream;
    auto row_a = [&](int k) { return mrow0 + int64_t(k) * pa.mask.ld_frame; };
    auto row_b = [&](int k) { return k + 1 < a.F ? row_a(k) + pa.mask.ld_frame : row_a(k); };  // (past F: unused)
    float ma_[NI + 1], mb_[NI + 1];  // the pair's mask rows, natural bins t + L i (i = NI: N/2, lane 0)
    auto load_rows = [&](int k) {
        const float* r0 = row_a(k);
        const float* r1 = row_b(k);
#pragma unroll
        for (int i = 0; i <= NI; ++i) {
            const int kr = i < NI ? t + L * i : P2;
            const bool on = i < NI || t == 0;
            ma_[i] = on ? r0[kr] : 1.0f;
            mb_[i] = on ? r1[kr] : 1.0f;
        }
    };
    auto rows_ok = [&]() {
        bool bad = false;
#pragma unroll
        for (int i = 0; i <= NI; ++i)
            bad |= !(__builtin_fabsf(ma_[i]) <= 0x1p20f) | !(__builtin_fabsf(mb_[i]) <= 0x1p20f);  // (NaN too)
        return __builtin_amdgcn_ballot_w64(bad) == 0;
    };

    float xin[E + SH];
    uint32_t hopok = 0;
#pragma unroll
    for (int h = 0; h <= NB; ++h) {
        load_hop(xin + h * SH, (fs + h) * H - a.pad);
        hopok |= hop_ok<SH>(xin + h * SH, xlo, xhi) << h;
    }
    constexpr uint32_t kPairHops = (1u << (NB + 1)) - 1;
    // verdict set 0: the pair's hops (posted one pair ahead); set 1: its mask rows
    // (loaded after the forward, so they are live across no transform, and
    // checked at the step: a row that leaves the paired regime drops the pair's
    // paired forward and the pair is done frame by frame)
    sm.post(wave, lane, (hopok & kPairHops) == kPairHops);
    __syncthreads();
    bool hops_paired = sm.all();
    for (int k = fs; k < f1; k += 2) {
        float nxt[2 * SH];
        load_hop(nxt, (k + NB + 1) * H - a.pad);
        load_hop(nxt + SH, (k + NB + 2) * H - a.pad);
        hopok = (hopok | hop_ok<SH>(nxt, xlo, xhi) << (NB + 1) | hop_ok<SH>(nxt + SH, xlo, xhi) << (NB + 2)) >> 2;
        const bool next_hops = (hopok & kPairHops) == kPairHops;
        dev::pc v[E];
        bool done = false;
        if (hops_paired) {
            const bool partner = k + 1 < a.F;  // frame k+1 past the last: imaginary part 0 (as the two-regime walker)
#pragma unroll
            for (int m = 0; m < E; ++m) {
                const float w = wag[L * m];
                v[m] = dev::pc_mk(xin[m] * w, partner ? xin[m + SH] * w : 0.0f);
            }
            tw.fwd(v, sm.xb, sm.tb, t);
#pragma unroll
            for (int d = 0; d < E; ++d) sm.xb[spad(G::bin(t, d))] = v[d];
            load_rows(k);
            __syncthreads();
            sm.post(wave, lane, rows_ok(), 1);
            // the step on this lane's bin pairs {kr, N - kr}, in place
#pragma unroll
            for (int i = 0; i <= NI; ++i) {
                const int kr = i < NI ? t + L * i : P2;
                const bool on = i < NI || t == 0;
                const int jr = (N - kr) & (N - 1);
                const float g = a.t.gain ? a.t.gain[kr] : 1.0f;
                const float ga = g * ma_[i], gb = g * mb_[i];
                const float c1 = 0.5f * (ga + gb), c2 = 0.5f * (ga - gb);
                const dev::pc z = sm.xb[spad(kr)], zp = sm.xb[spad(jr)];
                if (on) sm.xb[spad(kr)] = dev::pc_mk(__builtin_fmaf(c2, zp.x, c1 * z.x), __builtin_fmaf(-c2, zp.y, c1 * z.y));
                if (on && jr != kr)
                    sm.xb[spad(jr)] =
                        dev::pc_mk(__builtin_fmaf(c2, z.x, c1 * zp.x), __builtin_fmaf(-c2, z.y, c1 * zp.y));
            }
            __syncthreads();
            if (sm.all(1)) {  // (uniform: otherwise no wave reads xb again before the frame-by-frame pass)
#pragma unroll
                for (int d = 0; d < E; ++d) v[d] = sm.xb[spad(G::bin(t, d))];
                // the next pair's hop verdict; the barrier also keeps these reads ahead
                // of the inverse's exchange writes
                sm.post(wave, lane, next_hops);
                __syncthreads();
                tw.inv(v, sm.xb, sm.tb, t);
                float dr0[2 * SH], dr1[2 * SH];
                den_wg<L, SH>(dr0, rp, t, k % a.ring_blocks);
                den_wg<L, SH>(dr1, rp, t, (k + 1) % a.ring_blocks);
                ola.add(v, ws, false, true);
                ola.emit(k, f0, dr0, ry, ry_null, t);
                if (k + 1 < f1) {
                    ola.add(v, ws, true, true);
                    ola.emit(k + 1, f0, dr1, ry, ry_null, t);
                }
                done = true;
            }
        }
        if (!done) {  // each frame alone, full sanitize, its own gain g m
            auto pass = [&](auto pc_) {
                constexpr int P = decltype(pc_)::value;
#pragma unroll
                for (int m = 0; m < E; ++m) v[m] = dev::pc_mk(dev::sanit(xin[m + P * SH] * wag[L * m]), 0.0f);
                tw.fwd(v, sm.xb, sm.tb, t);
                // the frame's multipliers g m by real bin, staged in the (free) exchange buffer
                float* gm = reinterpret_cast<float*>(sm.xb);
                const float* r = P ? row_b(k) : row_a(k);
#pragma unroll
                for (int i = 0; i <= NI; ++i) {
                    const int kr = i < NI ? t + L * i : P2;
                    if (i < NI || t == 0) gm[kr] = (a.t.gain ? a.t.gain[kr] : 1.0f) * r[kr];
                }
                __syncthreads();
#pragma unroll
                for (int d = 0; d < E; ++d) {
                    const int kb = G::bin(t, d);
                    v[d] = v[d] * gm[kb <= P2 ? kb : N - kb];
                }
                __syncthreads();  // (the reads before the inverse's exchange rewrites xb)
                tw.inv(v, sm.xb, sm.tb, t);
                float dr[2 * SH];
                den_wg<L, SH>(dr, rp, t, (k + P) % a.ring_blocks);
                ola.add(v, ws, false, false);
                ola.emit(k + P, f0, dr, ry, ry_null, t);
            };
            pass(std::integral_constant<int, 0>());
            if (k + 1 < f1) pass(std::integral_constant<int, 1>());
            sm.post(wave, lane, next_hops);
            __syncthreads();
        }
        hops_paired = sm.all();
#pragma unroll
        for (int m = 0; m < E + SH - 2 * SH; ++m) xin[m] = xin[m + 2 * SH];
#pragma unroll
        for (int q = 0; q < 2 * SH; ++q) xin[E - SH + q] = nxt[q];
    }
}

template <typename G, typename K>
hipError_t launch_wg(K kernel, const PairSpecArgs& a, int64_t walkers, hipStream_t stream) {
    constexpr size_t lds = WgLds<G>::bytes;
    hipError_t e = set_lds(kernel, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kernel, dim3(unsigned(walkers)), dim3(G::L), lds, stream, a);
    return hipGetLastError();
}

template <typename G, typename K>
int wg_per_cu(K kernel) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void*>(kernel), G::L,
                                                     WgLds<G>::bytes) != hipSuccess ||
        nb <= 0)
        nb = 1;
    return nb;
}

}  // namespace

// N = 4096: H 512, 1024, 2048; N = 2048: H 256, 512, 1024 (SH = H / L = 2, 4, 8)
bool pair_wg_supported(int n, int h) {
    return (n == 4096 && (h == 512 || h == 1024 || h == 2048)) || (n == 2048 && (h == 256 || h == 512 || h == 1024));
}

int pair_wg_walkers_per_cu(int n) {
    static const int v4 = wg_per_cu<W4k>(k_pairwg_mask<W4k, 4, 4, false>);
    static const int v2 = wg_per_cu<W2k>(k_pairwg_mask<W2k, 4, 4, false>);
    return n == 4096 ? v4 : v2;
}

hipError_t launch_pairwg_stft(int n, int h, const PairSpecArgs& a, int64_t walkers, hipStream_t stream) {
    if (!pair_wg_supported(n, h) || !a.f.t.ptw4 || !a.f.t.wa) return hipErrorInvalidValue;
    note_launch(CRLOT_K_PAIR_STFT, walkers);
    auto go = [&](auto g) {
        using G = decltype(g);
        const int sh = h / G::L;
        return sh == 2 ? launch_wg<G>(k_pairwg_stft<G, 2>, a, walkers, stream)
                       : sh == 4 ? launch_wg<G>(k_pairwg_stft<G, 4>, a, walkers, stream)
                                 : launch_wg<G>(k_pairwg_stft<G, 8>, a, walkers, stream);
    };
    return n == 4096 ? go(W4k{}) : go(W2k{});
}

template <typename G, bool MASK>
hipError_t pairwg_istft_m(int sh, const PairSpecArgs& a, int64_t walkers, hipStream_t stream) {
    return sh == 2   ? launch_wg<G>(k_pairwg_istft<G, 2, 8, MASK>, a, walkers, stream)
           : sh == 4 ? launch_wg<G>(k_pairwg_istft<G, 4, 4, MASK>, a, walkers, stream)
                     : launch_wg<G>(k_pairwg_istft<G, 8, 2, MASK>, a, walkers, stream);
}

hipError_t launch_pairwg_istft(int n, int h, const PairSpecArgs& a, int64_t walkers, hipStream_t stream) {
    if (!pair_wg_supported(n, h) || !a.f.t.ptw4 || !a.f.t.pden4 || !a.f.t.wsn) return hipErrorInvalidValue;
    note_launch(CRLOT_K_PAIR_ISTFT, walkers);
    const bool mask = a.mask.p != nullptr;
    if (n == 4096) {
        const int sh = h / 256;
        return mask ? pairwg_istft_m<W4k, true>(sh, a, walkers, stream)
                    : pairwg_istft_m<W4k, false>(sh, a, walkers, stream);
    }
    const int sh = h / 128;
    return mask ? pairwg_istft_m<W2k, true>(sh, a, walkers, stream) : pairwg_istft_m<W2k, false>(sh, a, walkers, stream);
}

template <typename G, bool GAIN>
hipError_t pairwg_mask_g(int sh, const PairSpecArgs& a, int64_t walkers, hipStream_t stream) {
    return sh == 2   ? launch_wg<G>(k_pairwg_mask<G, 2, 8, GAIN>, a, walkers, stream)
           : sh == 4 ? launch_wg<G>(k_pairwg_mask<G, 4, 4, GAIN>, a, walkers, stream)
                     : launch_wg<G>(k_pairwg_mask<G, 8, 2, GAIN>, a, walkers, stream);
}

hipError_t launch_pairwg_mask(int n, int h, const PairSpecArgs& a, int64_t walkers, hipStream_t stream) {
    if (!pair_wg_supported(n, h) || !a.mask.p || !a.f.t.ptw4 || !a.f.t.pden4 || !a.f.t.wsn)
        return hipErrorInvalidValue;
    note_launch(CRLOT_K_PAIR_MASK, walkers);
    const bool gain = a.f.t.gain != nullptr;
    if (n == 4096) {
        const int sh = h / 256;
        return gain ? pairwg_mask_g<W4k, true>(sh, a, walkers, stream) : pairwg_mask_g<W4k, false>(sh, a, walkers, stream);
    }
    const int sh = h / 128;
    return gain ? pairwg_mask_g<W2k, true>(sh, a, walkers, stream) : pairwg_mask_g<W2k, false>(sh, a, walkers, stream);
}

}  // namespace fk
}  // namespace crlot
