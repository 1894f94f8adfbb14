// pair_hot.hip -- paired-only hot walkers of the frame-pair kernels other than
// K_pair (pair1k.hip): k_pair_wg_hot<Geo4k> (N = 4096, config 3) and <Geo2k>
// (N = 2048), one workgroup per chunk; k_pair512_hot (N = 512, the config-4
// shape batched), one wave per chunk.
//
// The same walk, transform and arithmetic as k_stft_ola_pair4k / _pair2k /
// _pair512 (kernels.hip),
// restructured the way K_pair's hot walker is (pair1k.hip):
//   * paired regime only: a hop outside the paired range, an output below the
//     sanitize threshold or a block outside Markstein's exact range flags the
//     workgroup's chunk, and k_stft_ola_pair4k (the two-regime walker, run after
//     it with the flags) redoes exactly those chunks -- so the per-pair
//     __syncthreads_or regime votes and the per-sample sanitize selects leave the
//     loop;
//   * the two workgroup exchanges of a pair use two buffers (A forward, B
//     inverse), so each costs one barrier instead of two: between a buffer's
//     reads and its next writes every wave passes the other buffer's barrier;
//   * each wave's quarter-wave transposes run in the exchange rows it alone
//     reads (forward, A) or writes (inverse, B), so the double buffer costs no
//     extra LDS: two 78 KB workgroups per CU at N = 4096, four 39 KB ones at 2048;
//   * hops and OLA blocks rotate through registers (compile-time slots), no
//     shifting.
// Outputs are bit-identical to the two-regime walkers: every paired pair runs
// the same operations in the same order.
#include <type_traits>

#include "fft_pair2k.h"
#include "fft_pair4k.h"
#include "fft_pair512.h"
#include "fused_common.h"
#include "ola_pair.h"

namespace crlot {
namespace fk {

namespace {

// Cache policy of the hot walkers' hop loads and output stores (2 = nt, streaming).
// Default policy kept: nt measured 4096/1024 +1.6 / -2.5 %, 512/128 -1.6 / -1.8 %,
// 2048/512 +2.0 / +0.9 % in interleaved A/Bs (scripts/ab_bench.py).
#ifndef CRLOT_HOT_AUX
#define CRLOT_HOT_AUX 0
#endif
// The OLA stage on block pairs (ola_pair.h) and the screened output-sanitize test
// (fft_pair.h out_min_exp_screened), as K_pair's hot walker (pair1k.hip).
#ifndef CRLOT_HOT_PK
#define CRLOT_HOT_PK 1
#endif

// 2^e as a float (e a normal exponent)
constexpr float pow2f(int e) { return __builtin_bit_cast(float, uint32_t(127 + e) << 23); }

// Exchange rows: a wave's own rows hold its 1152-element transpose buffer, and
// the row stride keeps the lane groups of a 32-lane b64 access on distinct
// banks (4k: 16-lane groups 2432 B = 128 B mod 256 B apart, as kP4Stride;
// 2k: 8-lane groups 1216 B = 192 B mod 256 B apart, as kP2Stride).
template <int SIDE>  // lanes t = x + SIDE r
struct XchgRows {
    // (lane t, reg k1) -> (lane SIDE k1 + x, reg r) through buffer A
    template <int KS>
    static __device__ __forceinline__ void fwd(dev::pc (&v)[16], dev::pc* A, int t) {
#pragma unroll
        for (int k1 = 0; k1 < 16; ++k1) A[KS * k1 + t] = v[k1];
        __syncthreads();
        const dev::pc* rb = A + KS * (t / SIDE) + (t % SIDE);
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = rb[SIDE * r];
    }
    // the inverse mapping through buffer B
    template <int KS>
    static __device__ __forceinline__ void inv(dev::pc (&v)[16], dev::pc* B, int t) {
        dev::pc* wb = B + KS * (t / SIDE) + (t % SIDE);
#pragma unroll
        for (int r = 0; r < 16; ++r) wb[SIDE * r] = v[r];
        __syncthreads();
#pragma unroll
        for (int k1 = 0; k1 < 16; ++k1) v[k1] = B[KS * k1 + t];
    }
};

template <bool INV, typename TW>
__device__ __forceinline__ void tw_all(dev::pc (&v)[16], const TW& w) {
    constexpr int idx[15] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
    dev::pc_tw_run<INV>(v, idx, [&](int i) { return w[i]; });
}
// a twiddle stage, explicit (pc[15]) or in the FMA form (Tw15F), then for the
// inverse the radix-16 that follows it (fused with the twiddles in the FMA form)
__device__ __forceinline__ void tw_fwd(dev::pc (&v)[16], const dev::pc (&w)[15]) { tw_all<false>(v, w); }
__device__ __forceinline__ void tw_fwd(dev::pc (&v)[16], const dev::Tw15F& w) { dev::tw15_apply_fwd(v, w); }
__device__ __forceinline__ void tw_pdft16_inv(dev::pc (&v)[16], const dev::pc (&w)[15]) {
    tw_all<true>(v, w);
    dev::pdft16<true>(v);
}
__device__ __forceinline__ void tw_pdft16_inv(dev::pc (&v)[16], const dev::Tw15F& w) { dev::tw15_pdft16_inv(v, w); }

// N = 4096: 256 lanes (fft_pair4k.h), rows of 304, a wave's own rows 4w .. 4w+3
struct Geo4k {
    static constexpr int N = 4096, L = 256, KS = 304, ROWS_PER_WAVE = 4, SIDE = 16, MIN_EXP = -87;  // 1e-30 N = 2^-87.66
    template <int SH, bool GAIN>
    using Tw = dev::Pair4kTwFor<SH, GAIN>;
    using X = XchgRows<SIDE>;
    template <typename TW>
    static __device__ __forceinline__ void tw_load(TW& tw, const float* g, int t) {
        dev::pair4k_tw_load(tw, reinterpret_cast<const dev::pc*>(g), t);
    }
    static constexpr __device__ int bin(int t, int d) { return dev::pair4k_bin(t, d); }
    template <typename TW>
    static __device__ __forceinline__ void fwd(dev::pc (&v)[16], dev::pc* A, const TW& tw, int t, int wave) {
        dev::pdft16<false>(v);
        tw_fwd(v, tw.w1);
        X::fwd<KS>(v, A, t);
        dev::pdft16<false>(v);
        tw_fwd(v, tw.w2);
        dev::transpose16(v, A + KS * ROWS_PER_WAVE * wave, t & 63);
        dev::pdft16<false>(v);
    }
    template <typename TW>
    static __device__ __forceinline__ void inv(dev::pc (&v)[16], dev::pc* B, const TW& tw, int t, int wave) {
        dev::pdft16<true>(v);
        dev::transpose16(v, B + KS * ROWS_PER_WAVE * wave, t & 63);
        tw_pdft16_inv(v, tw.w2);
        X::inv<KS>(v, B, t);
        tw_pdft16_inv(v, tw.w1);
    }
    // the wave-local parts of fwd / inv (after / before the workgroup exchange),
    // second-stage twiddles from a getter
    template <typename WF>
    static __device__ __forceinline__ void fwd_tail(dev::pc (&v)[16], dev::pc* own, WF w2, int lane) {
        constexpr int idx[15] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
        dev::pdft16<false>(v);
        dev::pc_tw_run<false>(v, idx, w2);
        dev::transpose16(v, own, lane);
        dev::pdft16<false>(v);
    }
    template <typename WF>
    static __device__ __forceinline__ void inv_head(dev::pc (&v)[16], dev::pc* own, WF w2, int lane) {
        constexpr int idx[15] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
        dev::pdft16<true>(v);
        dev::transpose16(v, own, lane);
        dev::pc_tw_run<true>(v, idx, w2);
        dev::pdft16<true>(v);
    }
};

// N = 2048: 128 lanes (fft_pair2k.h), rows of 152, a wave's own rows 8w .. 8w+7
struct Geo2k {
    static constexpr int N = 2048, L = 128, KS = 152, ROWS_PER_WAVE = 8, SIDE = 8, MIN_EXP = -88;  // 1e-30 N = 2^-88.66
    template <int SH, bool GAIN>
    using Tw = dev::Pair2kTwFor<SH, GAIN>;
    using X = XchgRows<SIDE>;
    template <typename TW>
    static __device__ __forceinline__ void tw_load(TW& tw, const float* g, int t) {
        dev::pair2k_tw_load(tw, reinterpret_cast<const dev::pc*>(g), t);
    }
    template <typename TW>
    static __device__ __forceinline__ void fwd(dev::pc (&v)[16], dev::pc* A, const TW& tw, int t, int wave) {
        dev::pdft16<false>(v);
        tw_fwd(v, tw.w1);
        X::fwd<KS>(v, A, t);
        dev::pdft16<false>(v);
        tw_fwd(v, tw.w2);
        dev::pair2k_t8(v, A + KS * ROWS_PER_WAVE * wave, t & 63);
        dev::pdft8_halves<false>(v);
    }
    template <typename TW>
    static __device__ __forceinline__ void inv(dev::pc (&v)[16], dev::pc* B, const TW& tw, int t, int wave) {
        dev::pdft8_halves<true>(v);
        dev::pair2k_t8(v, B + KS * ROWS_PER_WAVE * wave, t & 63);
        tw_pdft16_inv(v, tw.w2);
        X::inv<KS>(v, B, t);
        tw_pdft16_inv(v, tw.w1);
    }
    template <typename WF>
    static __device__ __forceinline__ void fwd_tail(dev::pc (&v)[16], dev::pc* own, WF w2, int lane) {
        constexpr int idx[15] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
        dev::pdft16<false>(v);
        dev::pc_tw_run<false>(v, idx, w2);
        dev::pair2k_t8(v, own, lane);
        dev::pdft8_halves<false>(v);
    }
    template <typename WF>
    static __device__ __forceinline__ void inv_head(dev::pc (&v)[16], dev::pc* own, WF w2, int lane) {
        constexpr int idx[15] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
        dev::pdft8_halves<true>(v);
        dev::pair2k_t8(v, own, lane);
        dev::pc_tw_run<true>(v, idx, w2);
        dev::pdft16<true>(v);
    }
};
static_assert(Geo4k::KS * Geo4k::ROWS_PER_WAVE >= dev::kPairXbuf, "4k transpose in own rows");
static_assert(Geo2k::KS * Geo2k::ROWS_PER_WAVE >= dev::kP2Tbuf, "2k transpose in own rows");

template <int NB>
struct RotWg {
    static constexpr int R = NB == 2 ? 8 : NB == 4 ? 8 : 16;
    static constexpr int U = R / 2;
    static_assert(R >= NB + 3 && (2 * U) % NB == 0, "ring");
};

template <int L, int SH>
__device__ __forceinline__ void load_hop_wg0(float* dst, __amdgpu_buffer_rsrc_t rx, int t, int origin) {
    const int v = (origin + t) * 4;  // out-of-range lanes (either side) read 0: see load_hop0
#pragma unroll
    for (int q = 0; q < SH; ++q)
        dst[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, v + q * (4 * L), 0, CRLOT_HOT_AUX));
}
// ... for one wave (lane l holds samples l + 64 q)
template <int SH>
__device__ __forceinline__ void load_hop_w(float* dst, __amdgpu_buffer_rsrc_t rx, int lane, int origin) {
    load_hop_wg0<64, SH>(dst, rx, lane, origin);
}

// den | rden of block b (DevTables::pden4: [block][L][den SH | rden SH])
template <int L, int SH>
__device__ __forceinline__ void load_den_wg(float (&dr)[2 * SH], __amdgpu_buffer_rsrc_t rp, int t, int b) {
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

}  // namespace

// Both geometries: two waves per SIMD (<= 256 VGPRs), two 4k / four 2k workgroups per CU.
template <typename G>
constexpr size_t hot_lds() {
    return sizeof(dev::pc) * 2 * 16 * G::KS;  // exchange buffers A | B
}

// One workgroup (G::L lanes) walks one chunk; lane t holds samples t + L m.
template <typename G, int SH, int NB, bool HAS_GAIN = false>
__global__ __launch_bounds__(G::L) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_pair_wg_hot(const FusedArgs a) {
    constexpr int E = 16, L = G::L, H = L * SH;
    constexpr int R = RotWg<NB>::R, U = RotWg<NB>::U;
    static_assert(NB * SH == E, "N = NB * H");
    static_assert(SH >= 2, "den rows are read 16 bytes at a time");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    dev::pc* A = reinterpret_cast<dev::pc*>(smem);
    dev::pc* B = A + 16 * G::KS;
    const int t = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);

    const int s = blockIdx.x / a.n_chunks, c = blockIdx.x - s * a.n_chunks;
    const int f0 = c * a.M;
    const int f1 = min(a.F, f0 + a.M);
    const int fs = max(0, f0 - (NB - 1)) & ~1;  // pairs start on even frames
    const __amdgpu_buffer_rsrc_t rx = dev::make_rsrc(a.x + int64_t(s) * a.ld_x, uint32_t(a.T) * 4u);
    const __amdgpu_buffer_rsrc_t ry = dev::make_rsrc(a.y + int64_t(s) * a.ld_y, uint32_t(a.out_len) * 4u);
    const __amdgpu_buffer_rsrc_t ry_null = dev::make_rsrc(a.y, 0u);
#if CRLOT_HOT_PK
    const __amdgpu_buffer_rsrc_t rp2 = dev::make_rsrc(a.t.pden2, uint32_t(a.ring_blocks * H) * 16u);
#else
    const __amdgpu_buffer_rsrc_t rp = dev::make_rsrc(a.t.pden4, uint32_t(a.ring_blocks * H) * 8u);
#endif
    const uint32_t xlo_b = __builtin_bit_cast(uint32_t, a.t.px_lo), xhi_b = __builtin_bit_cast(uint32_t, a.t.px_hi);

    typename G::template Tw<SH, HAS_GAIN> tw;
    G::tw_load(tw, a.t.ptw4, t);
    float wa[E], ws[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        wa[m] = a.t.wa[t + L * m];
        ws[m] = a.t.wsn[t + L * m] * a.gain;  // (ws g: ola_pair.h ola_pair_push_w)
    }
    // spectral gain of this lane's bins (the two-regime walker's operation), in registers
    float gr[HAS_GAIN ? E : 1];
    if constexpr (HAS_GAIN) {
#pragma unroll
        for (int d = 0; d < E; ++d) {
            const int kb = G::bin(t, d);
            gr[d] = a.t.gain[kb <= G::N / 2 ? kb : G::N - kb];
        }
    }

    // a hop keeps the paired regime iff every sample is 0 or in [px_lo, px_hi]
    // (hop_ok_bits on this lane's samples; the workgroup's verdict is the OR at the end)
    bool bad = false;
    auto hop_check = [&](const float (&h)[SH]) {
        uint32_t mx = 0u, mn = ~0u;
#pragma unroll
        for (int q = 0; q < SH; ++q) {
            const uint32_t u = __builtin_bit_cast(uint32_t, h[q]) & 0x7fffffffu;
            mx = max(mx, u);
            mn = min(mn, u - 1u);
        }
        bad |= (mx > xhi_b) | (mn < xlo_b - 1u);
    };
    float xr[R][SH];
#pragma unroll
    for (int h = 0; h <= NB; ++h) {
        load_hop_wg0<L, SH>(xr[h], rx, t, (fs + h) * H - a.pad);
        hop_check(xr[h]);
    }
    auto store_block = [&](int k, const float (&o)[SH]) {  // (k = -1: dropped)
        const __amdgpu_buffer_rsrc_t rk = k >= f0 ? ry : ry_null;
#pragma unroll
        for (int q = 0; q < SH; ++q)
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o[q]), rk, t * 4,
                                                  k * (4 * H) + q * (4 * L), CRLOT_HOT_AUX);
    };
#if CRLOT_HOT_PK
    dev::pc acc2[NB / 2][SH];
#pragma unroll
    for (int j = 0; j < NB / 2; ++j)
#pragma unroll
        for (int q = 0; q < SH; ++q) acc2[j][q] = dev::pc{0.f, 0.f};
#else
    float acc[NB][SH];
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int q = 0; q < SH; ++q) acc[j][q] = 0.f;

    // produce(H) of block k: Markstein division, exact for sums 0 or |acc| in
    // [2^-64, 2^64]; anything else flags the chunk for the IEEE division
    auto emit = [&](const float (&av)[SH], int k, const float (&dr)[2 * SH]) {
        int ex_lo = 0, ex_hi = 0;
#pragma unroll
        for (int q = 0; q < SH; ++q) {
            const int e = __builtin_amdgcn_frexp_expf(av[q]);
            ex_lo = min(ex_lo, e);
            ex_hi = max(ex_hi, e);
        }
        bad |= !((ex_lo >= -63) & (ex_hi <= 65));
        float o[SH];
#pragma unroll
        for (int q = 0; q < SH; ++q) o[q] = mk_div(av[q], dr[q], dr[SH + q]);
        store_block(k, o);
    };
#endif

    auto step = [&](auto phc, int k) {
        constexpr int PH = decltype(phc)::value;
        constexpr int S0 = (2 * PH) % R, B0 = (2 * PH) % NB;
        load_hop_wg0<L, SH>(xr[(S0 + NB + 1) % R], rx, t, (k + NB + 1) * H - a.pad);
        load_hop_wg0<L, SH>(xr[(S0 + NB + 2) % R], rx, t, (k + NB + 2) * H - a.pad);
        const bool partner = k + 1 < a.F;  // frame k+1 past the last: imaginary part 0 (as the two-regime walker)
        dev::pc v[E];
#pragma unroll
        for (int m = 0; m < E; ++m)
            v[m] = dev::pc_mk(xr[(S0 + m / SH) % R][m % SH] * wa[m],
                              partner ? xr[(S0 + 1 + m / SH) % R][m % SH] * wa[m] : 0.0f);
        G::fwd(v, A, tw, t, wave);
        if constexpr (HAS_GAIN) {
#pragma unroll
            for (int d = 0; d < E; ++d) v[d] = v[d] * gr[d];
        }
#if CRLOT_HOT_PK
        dev::pc d2[SH], r2[SH];
        load_den_pair<L, SH>(d2, r2, rp2, t, k % a.ring_blocks);
#else
        float dr0[2 * SH], dr1[2 * SH];
        load_den_wg<L, SH>(dr0, rp, t, k % a.ring_blocks);
        load_den_wg<L, SH>(dr1, rp, t, (k + 1) % a.ring_blocks);
#endif
        G::inv(v, B, tw, t, wave);
        // output sanitize: finite here, so only its threshold |v| < 1e-30 N can
        // act; frexp exponents <= G::MIN_EXP flag the chunk
#if CRLOT_HOT_PK
        bad |= dev::out_min_exp_screened<E>(v, pow2f(G::MIN_EXP)) <= G::MIN_EXP;
#else
        {
            int e[4] = {0, 0, 0, 0};
#pragma unroll
            for (int m = 0; m < E; ++m)
                e[m & 3] = min(e[m & 3], min(__builtin_amdgcn_frexp_expf(v[m].x), __builtin_amdgcn_frexp_expf(v[m].y)));
            bad |= min(min(e[0], e[1]), min(e[2], e[3])) <= G::MIN_EXP;
        }
#endif
        // push_frame_AoS of both frames, window and gain folded into the adds
#if CRLOT_HOT_PK
        ola_pair_push_w<E, SH, NB, B0>(acc2, v, ws);
        {
            float o0[SH], o1[SH];
            bad |= !mk_div_pair<SH>(acc2[B0 / 2], d2, r2, o0, o1);
            store_block(k, o0);
            store_block(k + 1 < f1 ? k + 1 : -1, o1);
        }
        ola_pair_open_w<E, SH, NB, B0>(acc2, v, ws);
#else
#pragma unroll
        for (int m = 0; m < E; ++m) {
            float& r = acc[(B0 + m / SH) % NB][m % SH];
            r = __builtin_fmaf(v[m].x, ws[m], m / SH == NB - 1 ? 0.0f : r);
        }
        emit(acc[B0], k, dr0);
#pragma unroll
        for (int m = 0; m < E; ++m) {
            float& r = acc[(B0 + 1 + m / SH) % NB][m % SH];
            r = __builtin_fmaf(v[m].y, ws[m], m / SH == NB - 1 ? 0.0f : r);
        }
        emit(acc[(B0 + 1) % NB], k + 1 < f1 ? k + 1 : -1, dr1);
#endif
        hop_check(xr[(S0 + NB + 1) % R]);
        hop_check(xr[(S0 + NB + 2) % R]);
    };
    for (int k = fs; k < f1; k += 2 * U) {
        step(std::integral_constant<int, 0>(), k);
        if (k + 2 >= f1) break;
        step(std::integral_constant<int, 1>(), k + 2);
        if (k + 4 >= f1) break;
        step(std::integral_constant<int, 2>(), k + 4);
        if (k + 6 >= f1) break;
        step(std::integral_constant<int, 3>(), k + 6);
        if constexpr (U > 4) {
            if (k + 8 >= f1) break;
            step(std::integral_constant<int, 4>(), k + 8);
            if (k + 10 >= f1) break;
            step(std::integral_constant<int, 5>(), k + 10);
            if (k + 12 >= f1) break;
            step(std::integral_constant<int, 6>(), k + 12);
            if (k + 14 >= f1) break;
            step(std::integral_constant<int, 7>(), k + 14);
        }
    }
    // every wave leaves the loop at the same k (f1 is per workgroup): one vote
    const bool any_bad = __syncthreads_or(bad);
    if (t == 0) a.t.pflags[blockIdx.x] = any_bad ? 1u : 0u;
}

template <typename G>
hipError_t launch_wg_hot(int sh, const FusedArgs& a, int64_t grid, hipStream_t stream) {
    constexpr size_t lds = hot_lds<G>();
    if (CRLOT_HOT_PK && !a.t.pden2) return hipErrorInvalidValue;  // the block-pair divisor rows
    auto go = [&](auto k) {
        hipError_t e = set_lds(k, lds);
        if (e != hipSuccess) return e;
        note_launch(G::N == 4096 ? CRLOT_K_PAIR4K_HOT : CRLOT_K_PAIR2K_HOT, grid);
        hipLaunchKernelGGL(k, dim3(unsigned(grid)), dim3(G::L), lds, stream, a);
        return hipGetLastError();
    };
    if constexpr (G::N == 2048) {  // H = 256 / 1024 spill at N = 2048: the two-regime walker runs those
        return sh == 4 && !a.t.gain ? go(k_pair_wg_hot<G, 4, 4>) : hipErrorInvalidValue;
    } else {
        if (a.t.gain) {  // the gain's 16 registers fit beside H = 1024's walk only
            auto kg = k_pair_wg_hot<G, 4, 4, true>;
            return sh == 4 ? go(kg) : hipErrorInvalidValue;
        }
        switch (sh) {
            case 2: return go(k_pair_wg_hot<G, 2, 8>);
            case 4: return go(k_pair_wg_hot<G, 4, 4>);
            case 8: return go(k_pair_wg_hot<G, 8, 2>);
            default: return hipErrorInvalidValue;
        }
    }
}

// ---- N = 4096 / 2048 at three waves per SIMD: a measured negative result kept
// outside the release library (tools/experiments/pair_wg_hot3.inc, on the include
// path of `make experiments` only); stubs here.
#ifdef CRLOT_PAIR_WG_HOT3_EXPERIMENT
#include "pair_wg_hot3.inc"
#else
hipError_t launch_pair4k_hot3(int, const FusedArgs&, int64_t, hipStream_t) { return hipErrorInvalidValue; }
hipError_t launch_pair2k_hot3(int, const FusedArgs&, int64_t, hipStream_t) { return hipErrorInvalidValue; }
#endif  // CRLOT_PAIR_WG_HOT3_EXPERIMENT

// ---- N = 512: one wave per chunk (W per workgroup, independent), lane l holds
// samples l + 64 m (m < 8); flags per wave.
template <int SH, int NB, int W>
__global__ __launch_bounds__(64 * W, 4) void k_pair512_hot(const FusedArgs a) {  // (4 waves per SIMD)
    constexpr int E = 8, N = 512, H = 64 * SH;
    constexpr int R = RotWg<NB>::R, U = RotWg<NB>::U;
    static_assert(NB * SH == E, "N = NB * H");
    static_assert(SH >= 2, "den rows are read 16 bytes at a time");
    static_assert(N == 512, "threshold exponent");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    dev::pc* buf = reinterpret_cast<dev::pc*>(smem) + wave * dev::kP512Buf;
    const int gw = blockIdx.x * W + wave;
    if (gw >= a.n_streams * a.n_chunks) return;
    const int s = gw / a.n_chunks, c = gw - s * a.n_chunks;
    const int f0 = c * a.M;
    const int f1 = min(a.F, f0 + a.M);
    const int fs = max(0, f0 - (NB - 1)) & ~1;  // pairs start on even frames
    const __amdgpu_buffer_rsrc_t rx = dev::make_rsrc(a.x + int64_t(s) * a.ld_x, uint32_t(a.T) * 4u);
    const __amdgpu_buffer_rsrc_t ry = dev::make_rsrc(a.y + int64_t(s) * a.ld_y, uint32_t(a.out_len) * 4u);
    const __amdgpu_buffer_rsrc_t ry_null = dev::make_rsrc(a.y, 0u);
#if CRLOT_HOT_PK
    const __amdgpu_buffer_rsrc_t rp2 = dev::make_rsrc(a.t.pden2, uint32_t(a.ring_blocks * H) * 16u);
#else
    const __amdgpu_buffer_rsrc_t rp = dev::make_rsrc(a.t.pden, uint32_t(a.ring_blocks * H) * 8u);
#endif
    const uint32_t xlo_b = __builtin_bit_cast(uint32_t, a.t.px_lo), xhi_b = __builtin_bit_cast(uint32_t, a.t.px_hi);

    dev::Pair512TwReg tw;
    dev::pair512_tw_load(tw, reinterpret_cast<const dev::pc*>(a.t.ptw), lane);
    float wa[E], ws[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        wa[m] = a.t.wa[lane + 64 * m];
        ws[m] = a.t.wsn[lane + 64 * m] * a.gain;  // (ws g: ola_pair.h ola_pair_push_w)
    }
    bool bad = false;
    auto hop_check = [&](const float (&h)[SH]) {
        uint32_t mx = 0u, mn = ~0u;
#pragma unroll
        for (int q = 0; q < SH; ++q) {
            const uint32_t u = __builtin_bit_cast(uint32_t, h[q]) & 0x7fffffffu;
            mx = max(mx, u);
            mn = min(mn, u - 1u);
        }
        bad |= (mx > xhi_b) | (mn < xlo_b - 1u);
    };
    float xr[R][SH];
#pragma unroll
    for (int h = 0; h <= NB; ++h) {
        load_hop_w<SH>(xr[h], rx, lane, (fs + h) * H - a.pad);
        hop_check(xr[h]);
    }
    auto store_block = [&](int k, const float (&o)[SH]) {  // (k = -1: dropped)
        const __amdgpu_buffer_rsrc_t rk = k >= f0 ? ry : ry_null;
#pragma unroll
        for (int q = 0; q < SH; ++q)
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o[q]), rk, lane * 4,
                                                  k * (4 * H) + q * 256, CRLOT_HOT_AUX);
    };
#if CRLOT_HOT_PK
    dev::pc acc2[NB / 2][SH];
#pragma unroll
    for (int j = 0; j < NB / 2; ++j)
#pragma unroll
        for (int q = 0; q < SH; ++q) acc2[j][q] = dev::pc{0.f, 0.f};
#else
    float acc[NB][SH];
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int q = 0; q < SH; ++q) acc[j][q] = 0.f;
    auto emit = [&](const float (&av)[SH], int k, const float (&dr)[2 * SH]) {
        int ex_lo = 0, ex_hi = 0;
#pragma unroll
        for (int q = 0; q < SH; ++q) {
            const int e = __builtin_amdgcn_frexp_expf(av[q]);
            ex_lo = min(ex_lo, e);
            ex_hi = max(ex_hi, e);
        }
        bad |= !((ex_lo >= -63) & (ex_hi <= 65));
        float o[SH];
#pragma unroll
        for (int q = 0; q < SH; ++q) o[q] = mk_div(av[q], dr[q], dr[SH + q]);
        store_block(k, o);
    };
#endif
    auto step = [&](auto phc, int k) {
        constexpr int PH = decltype(phc)::value;
        constexpr int S0 = (2 * PH) % R, B0 = (2 * PH) % NB;
        load_hop_w<SH>(xr[(S0 + NB + 1) % R], rx, lane, (k + NB + 1) * H - a.pad);
        load_hop_w<SH>(xr[(S0 + NB + 2) % R], rx, lane, (k + NB + 2) * H - a.pad);
        const bool partner = k + 1 < a.F;  // as the two-regime walker
        dev::pc v[E];
#pragma unroll
        for (int m = 0; m < E; ++m)
            v[m] = dev::pc_mk(xr[(S0 + m / SH) % R][m % SH] * wa[m],
                              partner ? xr[(S0 + 1 + m / SH) % R][m % SH] * wa[m] : 0.0f);
        dev::pair512_fwd(v, buf, tw, lane);
#if CRLOT_HOT_PK
        dev::pc d2[SH], r2[SH];
        load_den_pair<64, SH>(d2, r2, rp2, lane, k % a.ring_blocks);
#else
        float dr0[2 * SH], dr1[2 * SH];
        load_den<SH>(dr0, rp, lane, k % a.ring_blocks);
        load_den<SH>(dr1, rp, lane, (k + 1) % a.ring_blocks);
#endif
        dev::pair512_inv(v, buf, tw, lane);
        // output sanitize threshold 1e-30 N = 2^-90.66: frexp exponents <= -90 flag the chunk
#if CRLOT_HOT_PK
        bad |= dev::out_min_exp_screened<E>(v, pow2f(-90)) <= -90;
#else
        {
            int e[4] = {0, 0, 0, 0};
#pragma unroll
            for (int m = 0; m < E; ++m)
                e[m & 3] = min(e[m & 3], min(__builtin_amdgcn_frexp_expf(v[m].x), __builtin_amdgcn_frexp_expf(v[m].y)));
            bad |= min(min(e[0], e[1]), min(e[2], e[3])) <= -90;
        }
#endif
        // push_frame_AoS of both frames, window and gain folded into the adds
#if CRLOT_HOT_PK
        ola_pair_push_w<E, SH, NB, B0>(acc2, v, ws);
        {
            float o0[SH], o1[SH];
            bad |= !mk_div_pair<SH>(acc2[B0 / 2], d2, r2, o0, o1);
            store_block(k, o0);
            store_block(k + 1 < f1 ? k + 1 : -1, o1);
        }
        ola_pair_open_w<E, SH, NB, B0>(acc2, v, ws);
#else
#pragma unroll
        for (int m = 0; m < E; ++m) {
            float& r = acc[(B0 + m / SH) % NB][m % SH];
            r = __builtin_fmaf(v[m].x, ws[m], m / SH == NB - 1 ? 0.0f : r);
        }
        emit(acc[B0], k, dr0);
#pragma unroll
        for (int m = 0; m < E; ++m) {
            float& r = acc[(B0 + 1 + m / SH) % NB][m % SH];
            r = __builtin_fmaf(v[m].y, ws[m], m / SH == NB - 1 ? 0.0f : r);
        }
        emit(acc[(B0 + 1) % NB], k + 1 < f1 ? k + 1 : -1, dr1);
#endif
        hop_check(xr[(S0 + NB + 1) % R]);
        hop_check(xr[(S0 + NB + 2) % R]);
    };
    for (int k = fs; k < f1; k += 2 * U) {
        step(std::integral_constant<int, 0>(), k);
        if (k + 2 >= f1) break;
        step(std::integral_constant<int, 1>(), k + 2);
        if (k + 4 >= f1) break;
        step(std::integral_constant<int, 2>(), k + 4);
        if (k + 6 >= f1) break;
        step(std::integral_constant<int, 3>(), k + 6);
        if constexpr (U > 4) {
            if (k + 8 >= f1) break;
            step(std::integral_constant<int, 4>(), k + 8);
            if (k + 10 >= f1) break;
            step(std::integral_constant<int, 5>(), k + 10);
            if (k + 12 >= f1) break;
            step(std::integral_constant<int, 6>(), k + 12);
            if (k + 14 >= f1) break;
            step(std::integral_constant<int, 7>(), k + 14);
        }
    }
    const bool any_bad = __builtin_amdgcn_ballot_w64(bad) != 0;
    if (lane == 0) a.t.pflags[gw] = any_bad ? 1u : 0u;
}

hipError_t launch_pair512_hot(int sh, const FusedArgs& a, int64_t waves, int w, hipStream_t stream) {
    constexpr int W = 4;
    if (w != W || (CRLOT_HOT_PK && !a.t.pden2)) return hipErrorInvalidValue;
    const size_t lds = sizeof(dev::pc) * dev::kP512Buf * W;
    const int64_t grid = (waves + W - 1) / W;
    auto go = [&](auto k) {
        hipError_t e = set_lds(k, lds);
        if (e != hipSuccess) return e;
        note_launch(CRLOT_K_PAIR512_HOT, grid);
        hipLaunchKernelGGL(k, dim3(unsigned(grid)), dim3(64 * W), lds, stream, a);
        return hipGetLastError();
    };
    switch (sh) {
        case 2: return go(k_pair512_hot<2, 4, W>);
        case 4: return go(k_pair512_hot<4, 2, W>);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_pair4k_hot(int sh, const FusedArgs& a, int64_t grid, hipStream_t stream) {
    return launch_wg_hot<Geo4k>(sh, a, grid, stream);
}
hipError_t launch_pair2k_hot(int sh, const FusedArgs& a, int64_t grid, hipStream_t stream) {
    return launch_wg_hot<Geo2k>(sh, a, grid, stream);
}

}  // namespace fk
}  // namespace crlot
