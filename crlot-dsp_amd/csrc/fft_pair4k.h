// fft_pair4k.h -- 4096-point complex FFT of one 256-lane workgroup, built for
// the two-frames-per-transform round trip at N = 4096 (K_pair4k, kernels.hip).
//
// Two real frames a, b of N = 4096 samples travel as one complex sequence
// z = a + i b (see fft_pair.h for why the round trip's real and imaginary parts
// are the two frames' round trips).  Lane t (0..255, four waves) holds
// z[t + 256 m], m = 0..15 in registers.  With n = t + 256 m, t = x + 16 r and
// k = k1 + 16 k2 + 256 k3:
//   X[k] = sum_x W16^{x k3} W256^{x k2} sum_r W16^{r k2} [W4096^{t k1} sum_m W16^{m k1} z[t + 256 m]]
// Forward: radix-16 over the registers (m), twiddle W4096^{t k1}, one
// workgroup-wide LDS exchange (lane t, reg k1) -> (lane 16 k1 + x, reg r),
// radix-16 over r, twiddle W256^{x k2}, the quarter-wave 16x16 transpose of
// fft_pair.h, radix-16 over x.  The spectrum stays bin-scrambled (lane
// 16 k1 + k2, register k3: pair4k_bin()); the inverse runs the same steps
// backwards with conjugate twiddles and ends lane-major in natural order.
// Three radix-16 passes and no lane/register swaps (v_permlane): one
// barrier-bracketed exchange and one wave-local transpose per transform.
#pragma once

#include "fft_pair.h"

namespace crlot {
namespace dev {

// Bin of register d in workgroup lane t after pair4k_fwd.
__host__ __device__ constexpr int pair4k_bin(int t, int d) { return (t >> 4) + 16 * (t & 15) + 256 * d; }

// Exchange buffer: sequence k1 at k1 * 272 + t (complex units).  Writes: 64
// consecutive elements per wave-instruction.  Reads: 16-lane groups of 16
// consecutive elements, the two groups of a 32-lane b64 read 272 elements
// (2176 B = 128 B mod 256 B) apart -- distinct banks.
constexpr int kP4Stride = 272;
constexpr int kP4Xbuf = 16 * kP4Stride;  // complex elements per workgroup

// (lane t, reg k1) -> (lane 16 k1 + x, reg r), t = x + 16 r.  Both barriers are
// needed: the first publishes the writes, the second keeps the next exchange's
// writes (after at least one other barrier-free stretch) from racing these reads.
__device__ __forceinline__ void pair4k_xchg_fwd(pc (&v)[16], pc* xb, int t) {
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1) xb[kP4Stride * k1 + t] = v[k1];
    __syncthreads();
    const pc* rb = xb + kP4Stride * (t >> 4) + (t & 15);
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = rb[16 * r];
    __syncthreads();
}
// The inverse mapping: (lane 16 k1 + x, reg r) -> (lane t = x + 16 r, reg k1).
__device__ __forceinline__ void pair4k_xchg_inv(pc (&v)[16], pc* xb, int t) {
    pc* wb = xb + kP4Stride * (t >> 4) + (t & 15);
#pragma unroll
    for (int r = 0; r < 16; ++r) wb[16 * r] = v[r];
    __syncthreads();
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1) v[k1] = xb[kP4Stride * k1 + t];
    __syncthreads();
}

// Per-lane twiddles, held in registers for the whole walk:
//   w1[k1 - 1] = W4096^{t k1}, w2[k2 - 1] = W256^{(t & 15) k2}.
struct Pair4kTw {
    pc w1[15];
    pc w2[15];
};
// Device table (float pairs): [15][256] of W4096^{t k1}, then [15][16] of W256^{x k2}.
constexpr int kP4Tw = 15 * 256 + 15 * 16;
__device__ __forceinline__ void pair4k_tw_load(Pair4kTw& tw, const pc* g, int t) {
#pragma unroll
    for (int k = 1; k < 16; ++k) {
        tw.w1[k - 1] = g[(k - 1) * 256 + t];
        tw.w2[k - 1] = g[15 * 256 + (k - 1) * 16 + (t & 15)];
    }
}

// The same twiddles in the FMA form (fft_pair.h Tw15F): the inverse's two
// twiddle stages fuse into the first layer of the radix-16 that follows them
// (-16 packed operations per inverse, +8 VGPRs).
struct Pair4kTwF {
    Tw15F w1, w2;
};
__device__ __forceinline__ void pair4k_tw_load(Pair4kTwF& tw, const pc* g, int t) {
    tw15_load(tw.w1, [&](int k) { return g[(k - 1) * 256 + t]; });
    tw15_load(tw.w2, [&](int k) { return g[15 * 256 + (k - 1) * 16 + (t & 15)]; });
}
// The walkers' choice, by hop (SH = H / 256) and gain, the same in the hot and
// the two-regime walker so their paired bits agree: the FMA form at H = 1024
// without a gain (config 3).  Elsewhere its registers spill the hot walk -- the
// gain-carrying one by 54 VGPRs even with only the first stage fused (-7.6 % at
// 4096/1024 with a gain, profiles/r05c_ab.log) -- so a plan with a gain rounds
// its transforms the classic way: equal to the no-gain plan within the FFT
// tolerance, not bit for bit, at N = 4096.
#ifdef CRLOT_PAIR_TW_CLASSIC
template <int SH, bool GAIN>
using Pair4kTwFor = Pair4kTw;
#else
template <int SH, bool GAIN>
using Pair4kTwFor = std::conditional_t<SH == 4 && !GAIN, Pair4kTwF, Pair4kTw>;
#endif

// Forward: natural z[t + 256 m] -> bin-scrambled X (pair4k_bin).
__device__ __forceinline__ void pair4k_fwd(pc (&v)[16], pc* xb, pc* qb, const Pair4kTw& tw, int t) {
    pdft16<false>(v);
#pragma unroll
    for (int k1 = 1; k1 < 16; ++k1) v[k1] = pc_mul(v[k1], tw.w1[k1 - 1]);
    pair4k_xchg_fwd(v, xb, t);
    pdft16<false>(v);
#pragma unroll
    for (int k2 = 1; k2 < 16; ++k2) v[k2] = pc_mul(v[k2], tw.w2[k2 - 1]);
    transpose16(v, qb, t & 63);
    pdft16<false>(v);
}
__device__ __forceinline__ void pair4k_fwd(pc (&v)[16], pc* xb, pc* qb, const Pair4kTwF& tw, int t) {
    pdft16<false>(v);
    tw15_apply_fwd(v, tw.w1);
    pair4k_xchg_fwd(v, xb, t);
    pdft16<false>(v);
    tw15_apply_fwd(v, tw.w2);
    transpose16(v, qb, t & 63);
    pdft16<false>(v);
}

// Inverse (unnormalised): bin-scrambled Y -> natural y[t + 256 m].
__device__ __forceinline__ void pair4k_inv(pc (&v)[16], pc* xb, pc* qb, const Pair4kTw& tw, int t) {
    pdft16<true>(v);
    transpose16(v, qb, t & 63);
#pragma unroll
    for (int k2 = 1; k2 < 16; ++k2) v[k2] = pc_mulc(v[k2], tw.w2[k2 - 1]);
    pdft16<true>(v);
    pair4k_xchg_inv(v, xb, t);
#pragma unroll
    for (int k1 = 1; k1 < 16; ++k1) v[k1] = pc_mulc(v[k1], tw.w1[k1 - 1]);
    pdft16<true>(v);
}
__device__ __forceinline__ void pair4k_inv(pc (&v)[16], pc* xb, pc* qb, const Pair4kTwF& tw, int t) {
    pdft16<true>(v);
    transpose16(v, qb, t & 63);
    tw15_pdft16_inv(v, tw.w2);
    pair4k_xchg_inv(v, xb, t);
    tw15_pdft16_inv(v, tw.w1);
}

}  // namespace dev
}  // namespace crlot
