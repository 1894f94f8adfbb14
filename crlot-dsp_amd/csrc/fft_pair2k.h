// fft_pair2k.h -- 2048-point complex FFT of one 128-lane workgroup (two waves),
// for the two-frames-per-transform round trip at N = 2048 (K_pair2k, kernels.hip).
//
// Lane t (0..127) holds z[t + 128 m], m = 0..15.  With t = x + 8 r (x < 8,
// r < 16) and k = k1 + 16 k2 + 256 k3 (k1, k2 < 16, k3 < 8):
//   X[k] = sum_x W8^{x k3} W128^{x k2} sum_r W16^{r k2} [W2048^{t k1} sum_m W16^{m k1} z[t + 128 m]]
// Forward: radix-16 over the registers, twiddle W2048^{t k1}, one
// workgroup-wide LDS exchange (lane t, reg k1) -> (lane 8 k1 + x, reg r),
// radix-16 over r, twiddle W128^{x k2}, an 8x8 transpose inside every 8-lane
// group for each half of the registers, then radix-8 over x on both halves.
// The spectrum is left bin-scrambled (lane 8 k1 + (k2 & 7), register
// k3 + 8 (k2 >> 3): pair2k_bin()); the inverse runs the steps backwards.
#pragma once

#include "fft_pair512.h"

namespace crlot {
namespace dev {

__host__ __device__ constexpr int pair2k_bin(int t, int d) {
    return (t >> 3) + 16 * ((t & 7) + 8 * (d >> 3)) + 256 * (d & 7);
}

// Exchange buffer: sequence k1 at 136 k1 + t.  Writes: 64 consecutive
// elements per wave-instruction; b64 reads: 8-lane groups of 8 consecutive
// elements, four groups per 32-lane read 136 elements (1088 B = 64 B mod 256 B)
// apart -- distinct banks.
constexpr int kP2Stride = 136;
constexpr int kP2Xbuf = 16 * kP2Stride;
// Per-wave transpose buffer: two 8x8-per-group images (fft_pair512.h layout).
constexpr int kP2Tbuf = 2 * kP512Buf;

__device__ __forceinline__ void pair2k_xchg_fwd(pc (&v)[16], pc* xb, int t) {
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1) xb[kP2Stride * k1 + t] = v[k1];
    __syncthreads();
    const pc* rb = xb + kP2Stride * (t >> 3) + (t & 7);
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = rb[8 * r];
    __syncthreads();
}
__device__ __forceinline__ void pair2k_xchg_inv(pc (&v)[16], pc* xb, int t) {
    pc* wb = xb + kP2Stride * (t >> 3) + (t & 7);
#pragma unroll
    for (int r = 0; r < 16; ++r) wb[8 * r] = v[r];
    __syncthreads();
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1) v[k1] = xb[kP2Stride * k1 + t];
    __syncthreads();
}
// 8x8 transpose inside each 8-lane group, registers 0-7 and 8-15 separately
// (its own inverse): (lane 8 g + x, reg 8 h + k) <-> (lane 8 g + k, reg 8 h + x).
__device__ __forceinline__ void pair2k_t8(pc (&v)[16], pc* tb, int l) {
    pc* wb = tb + 72 * (l >> 3) + (l & 7);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int k = 0; k < 8; ++k) wb[kP512Buf * h + 9 * k] = v[8 * h + k];
    wave_lds_fence();
    const pc* rb = tb + 72 * (l >> 3) + 9 * (l & 7);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int x = 0; x < 8; ++x) v[8 * h + x] = rb[kP512Buf * h + x];
    wave_lds_fence();
}

// w1[k1 - 1] = W2048^{t k1}, w2[k2 - 1] = W128^{(t & 7) k2}
struct Pair2kTw {
    pc w1[15];
    pc w2[15];
};
// Device table (float pairs): [15][128] of W2048^{t k1}, then [15][8] of W128^{x k2}.
constexpr int kP2Tw = 15 * 128 + 15 * 8;
__device__ __forceinline__ void pair2k_tw_load(Pair2kTw& tw, const pc* g, int t) {
#pragma unroll
    for (int k = 1; k < 16; ++k) {
        tw.w1[k - 1] = g[(k - 1) * 128 + t];
        tw.w2[k - 1] = g[15 * 128 + (k - 1) * 8 + (t & 7)];
    }
}

template <bool INV>
__device__ __forceinline__ void pdft8_halves(pc (&v)[16]) {
    pc lo[8], hi[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        lo[i] = v[i];
        hi[i] = v[8 + i];
    }
    pdft8<INV>(lo);
    pdft8<INV>(hi);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        v[i] = lo[i];
        v[8 + i] = hi[i];
    }
}

// FMA form (fft_pair.h Tw15F) for the first-stage twiddles W2048^{t k1} only:
// the inverse's last twiddle stage fuses into its last radix-16 (-8 packed
// operations per inverse, +4 VGPRs; both stages would spill the hot walker).
struct Pair2kTwF {
    Tw15F w1;
    pc w2[15];
};
__device__ __forceinline__ void pair2k_tw_load(Pair2kTwF& tw, const pc* g, int t) {
    tw15_load(tw.w1, [&](int k) { return g[(k - 1) * 128 + t]; });
#pragma unroll
    for (int k = 1; k < 16; ++k) tw.w2[k - 1] = g[15 * 128 + (k - 1) * 8 + (t & 7)];
}
// The walkers' choice (SH = H / 128), as Pair4kTwFor: the FMA form at H = 512
// without a gain only.
#ifdef CRLOT_PAIR_TW_CLASSIC
template <int SH, bool GAIN>
using Pair2kTwFor = Pair2kTw;
#else
template <int SH, bool GAIN>
using Pair2kTwFor = std::conditional_t<SH == 4, Pair2kTwF, Pair2kTw>;
#endif
__device__ __forceinline__ void pair2k_tw1_fwd(pc (&v)[16], const Pair2kTw& tw) {
#pragma unroll
    for (int k1 = 1; k1 < 16; ++k1) v[k1] = pc_mul(v[k1], tw.w1[k1 - 1]);
}
__device__ __forceinline__ void pair2k_tw1_fwd(pc (&v)[16], const Pair2kTwF& tw) { tw15_apply_fwd(v, tw.w1); }
// conj first-stage twiddles, then the inverse's last radix-16
__device__ __forceinline__ void pair2k_tw1_pdft16_inv(pc (&v)[16], const Pair2kTw& tw) {
#pragma unroll
    for (int k1 = 1; k1 < 16; ++k1) v[k1] = pc_mulc(v[k1], tw.w1[k1 - 1]);
    pdft16<true>(v);
}
__device__ __forceinline__ void pair2k_tw1_pdft16_inv(pc (&v)[16], const Pair2kTwF& tw) { tw15_pdft16_inv(v, tw.w1); }

template <typename TW>
__device__ __forceinline__ void pair2k_fwd(pc (&v)[16], pc* xb, pc* tb, const TW& tw, int t) {
    pdft16<false>(v);
    pair2k_tw1_fwd(v, tw);
    pair2k_xchg_fwd(v, xb, t);
    pdft16<false>(v);
#pragma unroll
    for (int k2 = 1; k2 < 16; ++k2) v[k2] = pc_mul(v[k2], tw.w2[k2 - 1]);
    pair2k_t8(v, tb, t & 63);
    pdft8_halves<false>(v);
}

template <typename TW>
__device__ __forceinline__ void pair2k_inv(pc (&v)[16], pc* xb, pc* tb, const TW& tw, int t) {
    pdft8_halves<true>(v);
    pair2k_t8(v, tb, t & 63);
#pragma unroll
    for (int k2 = 1; k2 < 16; ++k2) v[k2] = pc_mulc(v[k2], tw.w2[k2 - 1]);
    pdft16<true>(v);
    pair2k_xchg_inv(v, xb, t);
    pair2k_tw1_pdft16_inv(v, tw);
}

}  // namespace dev
}  // namespace crlot
