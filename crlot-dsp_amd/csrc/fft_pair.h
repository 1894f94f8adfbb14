// fft_pair.h -- 1024-point complex FFT of one 64-lane wave, built for the
// two-frames-per-transform round trip (K_pair, kernels.hip).
//
// Two real frames a, b of N = 1024 samples travel as ONE complex sequence
// z[n] = a[n] + i b[n].  For a real, bin-symmetric spectral gain g (the
// reference's hook is the identity, e2e_benchmark.cc:161-162):
//     IFFT(g * FFT(z)) = IFFT(g * FFT(a)) + i IFFT(g * FFT(b)),
// so the real and imaginary parts of the round trip are the two frames'
// round trips (the textbook two-real-FFTs-for-one-complex identity), with no
// real split/merge stage between the transforms.
//
// Index bits (n = 10 bits): lane l holds z[l + 64 m], m = 0..15 in registers.
// The forward transform processes its four register bits, swaps two of them
// with lane bits 4 and 5 in registers (v_permlane16_swap / v_permlane32_swap,
// gfx950), processes those, then transposes 16x16 blocks through LDS once
// (padded layout, bank-conflict free, immediate offsets) and processes the
// remaining four bits:
//   n = L + 64 m, L = b + 16 a;  k = k1 + 16 (c + 4 d)
//   X[k] = sum_b W16^{b d} W64^{b c} sum_a W4^{a c} [W1024^{L k1} sum_m W16^{m k1} z[L + 64 m]]
// The spectrum is left in a bin-scrambled layout (lane = r + 16 q, register d,
// k1 = (r & 3) + 4 q, c = r >> 2; pair_bin()) that the inverse consumes
// directly, running the same steps backwards with conjugate twiddles and
// leaving y[L + 64 m] lane-major in natural order.  One LDS exchange per
// transform instead of two, and no exchange for the real split.
#pragma once

#include "fft_wave.h"

namespace crlot {
namespace dev {

// Bin index of register d in lane `lane` after pair_fft_fwd.
__host__ __device__ constexpr int pair_bin_lane(int lane) {
    return (lane & 3) + 4 * (lane >> 4) + 16 * ((lane >> 2) & 3);
}
__host__ __device__ constexpr int pair_bin(int lane, int d) { return pair_bin_lane(lane) + 64 * d; }

// a * W for the fixed rotations of a 16-point DFT; INV conjugates W.
// W16^j = (cos(pi j / 8), -sin(pi j / 8)) forward.
template <bool INV>
__device__ __forceinline__ cf crot(cf a, float c, float s) {  // a * (c - i s) [fwd] / (c + i s) [inv]
    return INV ? cf{__builtin_fmaf(a.r, c, -(a.i * s)), __builtin_fmaf(a.i, c, a.r * s)}
               : cf{__builtin_fmaf(a.r, c, a.i * s), __builtin_fmaf(a.i, c, -(a.r * s))};
}

// In-place 16-point DFT, natural order in and out: X[k] = sum_n x[n] W16^{+-nk}.
// n = 4 n1 + n2, k = k1 + 4 k2: four DFT4 over n1, twiddles W16^{n2 k1}, four
// DFT4 over n2 (outputs renamed in registers, no data movement).
template <bool INV>
__device__ __forceinline__ void dft16(cf (&x)[16]) {
    constexpr float c1 = 0.92387953251128675613f;  // cos(pi/8)
    constexpr float s1 = 0.38268343236508977173f;  // sin(pi/8)
    constexpr float h = 0.70710678118654752440f;   // sqrt(1/2)
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) dft4<INV>(x[n2], x[n2 + 4], x[n2 + 8], x[n2 + 12]);
    // a[n2][k1] now at x[n2 + 4 k1]; multiply by W16^{n2 k1}
    x[1 + 4 * 1] = crot<INV>(x[1 + 4 * 1], c1, s1);   // W^1
    x[1 + 4 * 2] = crot<INV>(x[1 + 4 * 2], h, h);     // W^2
    x[1 + 4 * 3] = crot<INV>(x[1 + 4 * 3], s1, c1);   // W^3
    x[2 + 4 * 1] = crot<INV>(x[2 + 4 * 1], h, h);     // W^2
    x[2 + 4 * 2] = mul_mi<INV>(x[2 + 4 * 2]);         // W^4 = -i
    x[2 + 4 * 3] = crot<INV>(x[2 + 4 * 3], -h, h);    // W^6
    x[3 + 4 * 1] = crot<INV>(x[3 + 4 * 1], s1, c1);   // W^3
    x[3 + 4 * 2] = crot<INV>(x[3 + 4 * 2], -h, h);    // W^6
    x[3 + 4 * 3] = crot<INV>(x[3 + 4 * 3], -c1, -s1); // W^9
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) dft4<INV>(x[4 * k1], x[4 * k1 + 1], x[4 * k1 + 2], x[4 * k1 + 3]);
    // X[k1 + 4 k2] sits at x[4 k1 + k2]: transpose the 4x4 register grid
    cf y[16];
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1)
#pragma unroll
        for (int k2 = 0; k2 < 4; ++k2) y[k1 + 4 * k2] = x[4 * k1 + k2];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = y[i];
}

// Swap lane bit 4 with register bit 2 and lane bit 5 with register bit 3
// (an involution).  v_permlane16_swap exchanges odd 16-lane rows of its first
// operand with even rows of its second; v_permlane32_swap the upper half of
// the first with the lower half of the second.
__device__ __forceinline__ void swap_f(float& a, float& b, bool b32) {
    const unsigned ua = __builtin_bit_cast(unsigned, a), ub = __builtin_bit_cast(unsigned, b);
    const auto r = b32 ? __builtin_amdgcn_permlane32_swap(ua, ub, false, false)
                       : __builtin_amdgcn_permlane16_swap(ua, ub, false, false);
    const unsigned r0 = r[0], r1 = r[1];
    a = __builtin_bit_cast(float, r0);
    b = __builtin_bit_cast(float, r1);
}
__device__ __forceinline__ void lane_reg_swap(cf (&v)[16]) {
#ifdef CRLOT_ABL_NOPERM  // timing-only ablation: wrong results
    return;
#endif
#pragma unroll
    for (int r = 0; r < 16; ++r)
        if (!(r & 4)) {
            swap_f(v[r].r, v[r | 4].r, false);
            swap_f(v[r].i, v[r | 4].i, false);
        }
#pragma unroll
    for (int r = 0; r < 16; ++r)
        if (!(r & 8)) {
            swap_f(v[r].r, v[r | 8].r, true);
            swap_f(v[r].i, v[r | 8].i, true);
        }
}

// 16x16 transpose inside each quarter wave through LDS: lane (x + 16 q),
// register y  ->  lane (y + 16 q), register x.  Layout: q * 288 + 18 * row + col
// (cf units): ds_write_b64 groups of 16 lanes hit 16 consecutive elements, and
// each lane reads its 16 elements as 8 ds_read_b128 of 16-byte aligned pairs
// whose starting banks 4 (9 x mod 16) are distinct in every b128 lane group --
// conflict free; every address is one per-lane base plus an immediate.
constexpr int kPairXbuf = 4 * 288;  // cf per wave
__device__ __forceinline__ void transpose16(cf (&v)[16], cf* buf, int lane) {
#ifdef CRLOT_ABL_NOXPOSE  // timing-only ablation: wrong results
    return;
#endif
    const int q = lane >> 4, x = lane & 15;
    cf* wb = buf + q * 288 + x;
    const float4* rb = reinterpret_cast<const float4*>(buf + q * 288 + 18 * x);
#pragma unroll
    for (int y = 0; y < 16; ++y) wb[18 * y] = v[y];
    wave_lds_fence();
#pragma unroll
    for (int y = 0; y < 8; ++y) {
        const float4 t = rb[y];
        v[2 * y] = cf{t.x, t.y};
        v[2 * y + 1] = cf{t.z, t.w};
    }
    wave_lds_fence();
}

// Twiddle table of the first pass, laid out for ds_read_b128: W1024^{l k1} for
// k1 = 2j+1+e at t1[j * 128 + 2 l + e] (j < 7), k1 = 15 at t1[896 + l].
constexpr int kPairT1 = 15 * 64;  // cf
__host__ __device__ constexpr int pair_t1_index(int k1, int l) {
    return k1 == 15 ? 896 + l : ((k1 - 1) >> 1) * 128 + 2 * l + ((k1 - 1) & 1);
}
template <bool INV>
__device__ __forceinline__ void pair_t1_apply(cf (&v)[16], const cf* t1, int lane) {
    const float4* t4 = reinterpret_cast<const float4*>(t1 + 2 * lane);
#pragma unroll
    for (int j = 0; j < 7; ++j) {
        const float4 t = t4[j * 64];
        const cf w0{t.x, t.y}, w1{t.z, t.w};
        v[2 * j + 1] = INV ? cmulc(v[2 * j + 1], w0) : cmul(v[2 * j + 1], w0);
        v[2 * j + 2] = INV ? cmulc(v[2 * j + 2], w1) : cmul(v[2 * j + 2], w1);
    }
    const cf w = t1[896 + lane];
    v[15] = INV ? cmulc(v[15], w) : cmul(v[15], w);
}

// Forward: natural z[lane + 64 m] -> bin-scrambled X (pair_bin).
//   t1: W1024^{l k1} (pair_t1_index), t2[16 (c - 1)] = W64^{(lane & 15) c} (LDS).
__device__ __forceinline__ void pair_fft_fwd(cf (&v)[16], cf* buf, const cf* t1, const cf* t2, int lane) {
    dft16<false>(v);
    pair_t1_apply<false>(v, t1, lane);
    lane_reg_swap(v);
#pragma unroll
    for (int j = 0; j < 4; ++j) dft4<false>(v[j], v[j + 4], v[j + 8], v[j + 12]);
#pragma unroll
    for (int c = 1; c < 4; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j + 4 * c] = cmul(v[j + 4 * c], t2[16 * (c - 1)]);
    transpose16(v, buf, lane);
    dft16<false>(v);
}

// Inverse (unnormalised): bin-scrambled Y -> natural y[lane + 64 m].
__device__ __forceinline__ void pair_fft_inv(cf (&v)[16], cf* buf, const cf* t1, const cf* t2, int lane) {
    dft16<true>(v);
    transpose16(v, buf, lane);
#pragma unroll
    for (int c = 1; c < 4; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j + 4 * c] = cmulc(v[j + 4 * c], t2[16 * (c - 1)]);
#pragma unroll
    for (int j = 0; j < 4; ++j) dft4<true>(v[j], v[j + 4], v[j + 8], v[j + 12]);
    lane_reg_swap(v);
    pair_t1_apply<true>(v, t1, lane);
    dft16<true>(v);
}

}  // namespace dev
}  // namespace crlot
