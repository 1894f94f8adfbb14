// fft_pair15.h -- 960-point complex FFT of one 64-lane wave for the frame-pair
// round trip at N = 960 (20 ms at 48 kHz; K_pair960, pair_any.hip).
//
// Lane l holds z[l + 64 m], m = 0..14 in registers v[0..14] (v[15] is a zero
// row).  960 = 15 x 64, n = l + 64 m, k = k1 + 15 k':
//   X[k] = DFT64_l( W960^{l k1} DFT15_m(z[l + 64 m])[k1] )[k']
// The 15-point DFT over the registers is Good-Thomas 3 x 5 (no twiddles, index
// maps renamed at compile time); after the W960^{l k1} twiddles the 16 register
// rows -- the 15 sequences k1 plus the zero row -- go through exactly the lane
// stage of fft_pair.h's 1024-point transform (lane/register swap of bits 4-5,
// radix 4, W64^{b c}, quarter-wave transpose, radix 16), which is a batch of
// 64-point DFTs over the lanes, one per register row.  The zero row stays zero
// both ways.  Spectrum bin of (lane, register d): k1 = (lane & 3) + 4 (lane >> 4)
// (k1 = 15: the zero row), k' = ((lane >> 2) & 3) + 4 d.
#pragma once

#include "fft_pair.h"

namespace crlot {
namespace dev {

__host__ __device__ constexpr int pair15_bin(int lane, int d) {
    return ((lane & 3) + 4 * (lane >> 4)) + 15 * (((lane >> 2) & 3) + 4 * d);  // k1 = 15: no bin
}
// N = 480 (pair15h_fwd): half-lane h = lane & 31 holds k1 = (h & 7) + 8 (h >> 4),
// c = (h >> 3) & 1 and, in register e, bin k1 + 15 (c + 2 e) (k1 = 15: the zero row)
__host__ __device__ constexpr int pair15h_bin(int lane, int e) {
    const int h = lane & 31;
    return ((h & 7) + 8 * (h >> 4)) + 15 * (((h >> 3) & 1) + 2 * e);
}

__device__ __forceinline__ pc pc_fma(pc a, pc b, pc c) { return __builtin_elementwise_fma(a, b, c); }

// DFT3 (forward W3 = e^{-2 pi i / 3}; INV conjugate): 7 packed ops
template <bool INV>
__device__ __forceinline__ void pdft3(pc& x0, pc& x1, pc& x2) {
    constexpr float c3 = 0.86602540378443864676f;  // sqrt(3)/2
    const pc s = x1 + x2, d = x1 - x2;
    const pc m = pc_fma(s, (pc){-0.5f, -0.5f}, x0);
    const pc e = d * (pc){c3, c3};
    x0 = x0 + s;
    x1 = pc_add_mi<INV>(m, e);  // m -+ i e
    x2 = pc_sub_mi<INV>(m, e);
}

// DFT5 (forward W5 = e^{-2 pi i / 5}; INV conjugate): 18 packed ops
template <bool INV>
__device__ __forceinline__ void pdft5(pc& x0, pc& x1, pc& x2, pc& x3, pc& x4) {
    constexpr float c1 = 0.30901699437494742410f;   // cos(2 pi / 5)
    constexpr float c2 = -0.80901699437494742410f;  // cos(4 pi / 5)
    constexpr float s1 = 0.95105651629515357212f;   // sin(2 pi / 5)
    constexpr float s2 = 0.58778525229247312917f;   // sin(4 pi / 5)
    const pc t1 = x1 + x4, t2 = x2 + x3, t3 = x1 - x4, t4 = x2 - x3;
    const pc a1 = pc_fma(t2, (pc){c2, c2}, pc_fma(t1, (pc){c1, c1}, x0));
    const pc a2 = pc_fma(t2, (pc){c1, c1}, pc_fma(t1, (pc){c2, c2}, x0));
    const pc b1 = pc_fma(t4, (pc){s2, s2}, t3 * (pc){s1, s1});
    const pc b2 = pc_fma(t4, (pc){-s1, -s1}, t3 * (pc){s2, s2});
    x0 = x0 + t1 + t2;
    x1 = pc_add_mi<INV>(a1, b1);  // a1 -+ i b1
    x4 = pc_sub_mi<INV>(a1, b1);
    x2 = pc_add_mi<INV>(a2, b2);
    x3 = pc_sub_mi<INV>(a2, b2);
}

// In-place 15-point DFT of v[0..14], natural order in and out (Good-Thomas:
// n = (5 n1 + 3 n2) mod 15, k = (10 k1 + 6 k2) mod 15).
template <bool INV>
__device__ __forceinline__ void pdft15(pc (&v)[16]) {
    pc y[3][5];
#pragma unroll
    for (int n2 = 0; n2 < 5; ++n2) {
        pc a = v[(3 * n2) % 15], b = v[(5 + 3 * n2) % 15], c = v[(10 + 3 * n2) % 15];
        pdft3<INV>(a, b, c);
        y[0][n2] = a;
        y[1][n2] = b;
        y[2][n2] = c;
    }
#pragma unroll
    for (int k1 = 0; k1 < 3; ++k1) {
        pdft5<INV>(y[k1][0], y[k1][1], y[k1][2], y[k1][3], y[k1][4]);
#pragma unroll
        for (int k2 = 0; k2 < 5; ++k2) v[(10 * k1 + 6 * k2) % 15] = y[k1][k2];
    }
}

// w1[k1 - 1] = W960^{lane k1} (k1 = 1..14), w2[c - 1] = W64^{(lane & 15) c}
struct Pair15Tw {
    pc w1[14];
    pc w2[3];
};
// Device table (float pairs): [14][64] of W960^{l k1}, then [3][16] of W64^{b c}.
constexpr int kP15Tw = 14 * 64 + 3 * 16;
__device__ __forceinline__ void pair15_tw_load(Pair15Tw& tw, const pc* g, int lane) {
#pragma unroll
    for (int k = 1; k < 15; ++k) tw.w1[k - 1] = g[(k - 1) * 64 + lane];
#pragma unroll
    for (int c = 1; c < 4; ++c) tw.w2[c - 1] = g[14 * 64 + 16 * (c - 1) + (lane & 15)];
}

// Forward: natural z[lane + 64 m] (v[15] = 0) -> bin-scrambled X (pair15_bin).
__device__ __forceinline__ void pair15_fwd(pc (&v)[16], pc* buf, const Pair15Tw& tw, int lane) {
    pdft15<false>(v);
    {
        constexpr int idx[14] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14};
        pc_tw_run<false>(v, idx, [&](int i) { return tw.w1[i]; });
    }
    lane_reg_swap(v);
#pragma unroll
    for (int j = 0; j < 4; ++j) pdft4<false>(v[j], v[j + 4], v[j + 8], v[j + 12]);
    {
        constexpr int idx[12] = {4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
        pc_tw_run<false>(v, idx, [&](int i) { return tw.w2[i / 4]; });
    }
    transpose16(v, buf, lane);
    pdft16<false>(v);
}

// Inverse (unnormalised): bin-scrambled Y -> natural y[lane + 64 m] in v[0..14].
__device__ __forceinline__ void pair15_inv(pc (&v)[16], pc* buf, const Pair15Tw& tw, int lane) {
    pdft16<true>(v);
    transpose16(v, buf, lane);
    {
        constexpr int idx[12] = {4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
        pc_tw_run<true>(v, idx, [&](int i) { return tw.w2[i / 4]; });
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) pdft4<true>(v[j], v[j + 4], v[j + 8], v[j + 12]);
    lane_reg_swap(v);
    {
        constexpr int idx[14] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14};
        pc_tw_run<true>(v, idx, [&](int i) { return tw.w1[i]; });
    }
    pdft15<true>(v);
}

// ---- N = 480 = 15 x 32: one transform per 32-lane half (two walks per wave).
// Half-lane h (0..31) holds z[h + 32 m], m < 15.  After the 15-point DFT over
// the registers and W480^{h k1}, a batch of 32-point DFTs over the half's lanes,
// h = b + 16 a: lane bit 4 (a) swapped with register bit 3 (v_permlane16_swap
// stays inside each 32-lane half), DFT2, W32^{b c}, the quarter-wave 16 x 16
// transpose, DFT16.  k = k1 + 15 (c + 2 d).
__device__ __forceinline__ void lane_reg_swap_b4r3(pc (&v)[16]) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        float ar = v[r].x, ai = v[r].y, br = v[r + 8].x, bi = v[r + 8].y;
        swap_f(ar, br, false);
        swap_f(ai, bi, false);
        v[r] = pc_mk(ar, ai);
        v[r + 8] = pc_mk(br, bi);
    }
}

// w1[k1 - 1] = W480^{h k1} (k1 = 1..14), w32 = W32^{h & 15}
struct Pair15hTw {
    pc w1[14];
    pc w32;
};
// Device table (float pairs): [14][32] of W480^{h k1}, then [16] of W32^{b}.
constexpr int kP15hTw = 14 * 32 + 16;
__device__ __forceinline__ void pair15h_tw_load(Pair15hTw& tw, const pc* g, int hl) {
#pragma unroll
    for (int k = 1; k < 15; ++k) tw.w1[k - 1] = g[(k - 1) * 32 + hl];
    tw.w32 = g[14 * 32 + (hl & 15)];
}

__device__ __forceinline__ void pair15h_fwd(pc (&v)[16], pc* buf, const Pair15hTw& tw, int lane) {
    pdft15<false>(v);
    {
        constexpr int idx[14] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14};
        pc_tw_run<false>(v, idx, [&](int i) { return tw.w1[i]; });
    }
    lane_reg_swap_b4r3(v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const pc a = v[j], b = v[j + 8];
        v[j] = a + b;
        v[j + 8] = a - b;
    }
    {
        constexpr int idx[8] = {8, 9, 10, 11, 12, 13, 14, 15};
        pc_tw_run<false>(v, idx, [&](int) { return tw.w32; });
    }
    transpose16(v, buf, lane);
    pdft16<false>(v);
}

__device__ __forceinline__ void pair15h_inv(pc (&v)[16], pc* buf, const Pair15hTw& tw, int lane) {
    pdft16<true>(v);
    transpose16(v, buf, lane);
    {
        constexpr int idx[8] = {8, 9, 10, 11, 12, 13, 14, 15};
        pc_tw_run<true>(v, idx, [&](int) { return tw.w32; });
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const pc a = v[j], b = v[j + 8];
        v[j] = a + b;
        v[j + 8] = a - b;
    }
    lane_reg_swap_b4r3(v);
    {
        constexpr int idx[14] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14};
        pc_tw_run<true>(v, idx, [&](int i) { return tw.w1[i]; });
    }
    pdft15<true>(v);
}

}  // namespace dev
}  // namespace crlot
