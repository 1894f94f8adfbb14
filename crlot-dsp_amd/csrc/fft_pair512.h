// fft_pair512.h -- 512-point complex FFT of one 64-lane wave, built for the
// two-frames-per-transform round trip at N = 512 (K_pair512, kernels.hip).
//
// Two real frames of N = 512 samples travel as one complex sequence (see
// fft_pair.h).  Lane l holds z[l + 64 m], m = 0..7.  With l = x + 8 r and
// k = k1 + 8 k2 + 64 k3:
//   X[k] = sum_x W8^{x k3} W64^{x k2} sum_r W8^{r k2} [W512^{l k1} sum_m W8^{m k1} z[l + 64 m]]
// Three packed radix-8 passes with two wave-local LDS exchanges between them:
// (lane l, reg k1) -> (lane 8 k1 + x, reg r), then the 8x8 transpose inside
// each 8-lane group; the spectrum is left bin-scrambled (lane 8 k1 + k2,
// register k3: pair512_bin()) and the inverse runs the steps backwards.
#pragma once

#include "fft_pair.h"

namespace crlot {
namespace dev {

__host__ __device__ constexpr int pair512_bin(int lane, int d) { return (lane >> 3) + 8 * (lane & 7) + 64 * d; }

// In-place 8-point DFT, natural order in and out (n = 4 n1 + n2, k = k1 + 2 k2).
// The radix-4 over n2 for k1 = 1 takes W8 x5 + m x6 + W8^3 x7 in the FMA form of
// pdft16's k1 = 2 group (W8 = h (1 -+ i)): 34 packed operations instead of 36.
template <bool INV>
__device__ __forceinline__ void pdft8_l2(pc (&x)[8]) {
    const pc kh = k16_h();
    const pc c0 = pc_add_mi<INV>(x[4], x[6]), c1 = pc_sub_mi<INV>(x[4], x[6]);
    const pc p = pc_add_mi<INV>(x[5], x[7]), q = pc_sub_mi<INV>(x[5], x[7]);
    const pc yp = pk_yform1<INV>(p), yq = pk_yform1<INV>(q);
    pdft4<INV>(x[0], x[1], x[2], x[3]);
    x[4] = pk_fmak<0, false>(yp, kh, c0);
    x[6] = pk_fmak<0, true>(yp, kh, c0);
    x[5] = pk_fma_mi<INV, true, 0>(yq, kh, c1);
    x[7] = pk_fma_mi<INV, false, 0>(yq, kh, c1);
    // X[k1 + 2 k2] sits at x[4 k1 + k2]
    pc y[8];
#pragma unroll
    for (int k1 = 0; k1 < 2; ++k1)
#pragma unroll
        for (int k2 = 0; k2 < 4; ++k2) y[k1 + 2 * k2] = x[4 * k1 + k2];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = y[i];
}
template <bool INV>
__device__ __forceinline__ void pdft8_fma(pc (&x)[8]) {
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) {
        const pc a = x[n2], b = x[n2 + 4];
        x[n2] = a + b;
        x[n2 + 4] = a - b;
    }
    pdft8_l2<INV>(x);
}
template <bool INV>
__device__ __forceinline__ void pdft8_rot(pc (&x)[8]) {
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) {
        const pc a = x[n2], b = x[n2 + 4];
        x[n2] = a + b;
        x[n2 + 4] = a - b;
    }
    x[5] = rot16<INV, 2>(x[5]);  // W8^1
    x[7] = rot16<INV, 6>(x[7]);  // W8^3   (W8^2 = -i on x[6] is folded into the DFT4)
    pdft4<INV>(x[0], x[1], x[2], x[3]);
    pdft4<INV, true>(x[4], x[5], x[6], x[7]);
    // X[k1 + 2 k2] sits at x[4 k1 + k2]
    pc y[8];
#pragma unroll
    for (int k1 = 0; k1 < 2; ++k1)
#pragma unroll
        for (int k2 = 0; k2 < 4; ++k2) y[k1 + 2 * k2] = x[4 * k1 + k2];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = y[i];
}
template <bool INV>
__device__ __forceinline__ void pdft8(pc (&x)[8]) {
#ifdef CRLOT_PDFT16_CLASSIC
    pdft8_rot<INV>(x);
#else
    pdft8_fma<INV>(x);
#endif
}

// One 576-element buffer per wave serves both exchanges (complex units):
//   exchange 1: element (lane l, reg k1) at 72 k1 + l, read back by lane 8 k1 + x as reg r (l = x + 8 r);
//   exchange 2: element (lane 8 g + x, reg k2) at 72 g + 9 k2 + x, read back by lane 8 g + k2 as reg x.
// 16-lane write groups and 32-lane b64 read groups are bank-conflict free in both.
constexpr int kP512Buf = 576;
__device__ __forceinline__ void p512_xchg1_fwd(pc (&v)[8], pc* buf, int l) {
#pragma unroll
    for (int k1 = 0; k1 < 8; ++k1) buf[72 * k1 + l] = v[k1];
    wave_lds_fence();
    const pc* rb = buf + 72 * (l >> 3) + (l & 7);
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = rb[8 * r];
    wave_lds_fence();
}
__device__ __forceinline__ void p512_xchg1_inv(pc (&v)[8], pc* buf, int l) {
    pc* wb = buf + 72 * (l >> 3) + (l & 7);
#pragma unroll
    for (int r = 0; r < 8; ++r) wb[8 * r] = v[r];
    wave_lds_fence();
#pragma unroll
    for (int k1 = 0; k1 < 8; ++k1) v[k1] = buf[72 * k1 + l];
    wave_lds_fence();
}
// the 8x8 transpose is its own inverse
__device__ __forceinline__ void p512_xchg2(pc (&v)[8], pc* buf, int l) {
    pc* wb = buf + 72 * (l >> 3) + (l & 7);
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2) wb[9 * k2] = v[k2];
    wave_lds_fence();
    const pc* rb = buf + 72 * (l >> 3) + 9 * (l & 7);
#pragma unroll
    for (int x = 0; x < 8; ++x) v[x] = rb[x];
    wave_lds_fence();
}

// Per-lane twiddles in registers: w1[k1 - 1] = W512^{l k1}, w2[k2 - 1] = W64^{(l & 7) k2}.
struct Pair512Tw {
    pc w1[7];
    pc w2[7];
};
// Device table (float pairs): [7][64] of W512^{l k1}, then [7][8] of W64^{x k2}.
constexpr int kP512Tw = 7 * 64 + 7 * 8;
__device__ __forceinline__ void pair512_tw_load(Pair512Tw& tw, const pc* g, int l) {
#pragma unroll
    for (int k = 1; k < 8; ++k) {
        tw.w1[k - 1] = g[(k - 1) * 64 + l];
        tw.w2[k - 1] = g[7 * 64 + (k - 1) * 8 + (l & 7)];
    }
}

// FMA form of the same twiddles: k = 1, 2, 3 as (T, C), k = 4..7 as (cos, sin)
// (no extra VGPRs).  The inverse's twiddled radix-8 takes them on its first
// layer, radix-2 pairs (n, n + 4): C_n (x_n - T (i x_n)) +- x_{n+4} w_{n+4} as one
// fma each -- 19 packed operations for the stage instead of 22.  The pending
// factor sits on input n because cos(2 pi l k / 512) vanishes at l = 32, k = 4
// (a T of 1e16 would overflow the unpaired regime's huge frames), while cos(2 pi
// l k / 512) for l < 64, k = 1..3 and cos(2 pi x k / 64) for x < 8 never do.
struct Tw7F {
    pc y[3];
    pc e[4];
};
template <typename WF>
__device__ __forceinline__ void tw7_load(Tw7F& tw, WF w) {
#pragma unroll
    for (int k = 1; k < 4; ++k) tw.y[k - 1] = tw_tc(w(k));
#pragma unroll
    for (int k = 4; k < 8; ++k) tw.e[k - 4] = w(k);
}
__device__ __forceinline__ void tw7_apply_fwd(pc (&v)[8], const Tw7F& tw) {
#pragma unroll
    for (int k = 1; k < 8; ++k) v[k] = k < 4 ? pk_tw_tc<false>(v[k], tw.y[k - 1]) : pc_mul(v[k], tw.e[k - 4]);
}
// a * K.y - b
__device__ __forceinline__ pc pk_fma_hi_sub_v(pc a, pc k, pc b) {
    pc r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[1,1,1] neg_lo:[0,0,1] neg_hi:[0,0,1]"
        : "=v"(r) : "v"(a), "v"(k), "v"(b));
    return r;
}
__device__ __forceinline__ void tw7_pdft8_inv(pc (&v)[8], const Tw7F& tw) {
    {
        const pc u1 = pc_mulc(v[4], tw.e[0]);
        const pc u0 = v[0];
        v[0] = u0 + u1;
        v[4] = u0 - u1;
    }
#pragma unroll
    for (int n = 1; n < 4; ++n) {
        const pc u1 = pc_mulc(v[n + 4], tw.e[n]);
        const pc y = pk_yform_v<true>(v[n], tw.y[n - 1]);
        v[n] = pk_fmak_v<1, false>(y, tw.y[n - 1], u1);
        v[n + 4] = pk_fma_hi_sub_v(y, tw.y[n - 1], u1);
    }
    pdft8_l2<true>(v);
}
struct Pair512TwF {
    Tw7F w1, w2;
};
__device__ __forceinline__ void pair512_tw_load(Pair512TwF& tw, const pc* g, int l) {
    tw7_load(tw.w1, [&](int k) { return g[(k - 1) * 64 + l]; });
    tw7_load(tw.w2, [&](int k) { return g[7 * 64 + (k - 1) * 8 + (l & 7)]; });
}
#ifdef CRLOT_PAIR_TW_CLASSIC
using Pair512TwReg = Pair512Tw;
#else
using Pair512TwReg = Pair512TwF;
#endif
__device__ __forceinline__ void pair512_fwd(pc (&v)[8], pc* buf, const Pair512TwF& tw, int l) {
    pdft8<false>(v);
    tw7_apply_fwd(v, tw.w1);
    p512_xchg1_fwd(v, buf, l);
    pdft8<false>(v);
    tw7_apply_fwd(v, tw.w2);
    p512_xchg2(v, buf, l);
    pdft8<false>(v);
}
__device__ __forceinline__ void pair512_inv(pc (&v)[8], pc* buf, const Pair512TwF& tw, int l) {
    pdft8<true>(v);
    p512_xchg2(v, buf, l);
    tw7_pdft8_inv(v, tw.w2);
    p512_xchg1_inv(v, buf, l);
    tw7_pdft8_inv(v, tw.w1);
}

__device__ __forceinline__ void pair512_fwd(pc (&v)[8], pc* buf, const Pair512Tw& tw, int l) {
    pdft8<false>(v);
#pragma unroll
    for (int k1 = 1; k1 < 8; ++k1) v[k1] = pc_mul(v[k1], tw.w1[k1 - 1]);
    p512_xchg1_fwd(v, buf, l);
    pdft8<false>(v);
#pragma unroll
    for (int k2 = 1; k2 < 8; ++k2) v[k2] = pc_mul(v[k2], tw.w2[k2 - 1]);
    p512_xchg2(v, buf, l);
    pdft8<false>(v);
}

__device__ __forceinline__ void pair512_inv(pc (&v)[8], pc* buf, const Pair512Tw& tw, int l) {
    pdft8<true>(v);
    p512_xchg2(v, buf, l);
#pragma unroll
    for (int k2 = 1; k2 < 8; ++k2) v[k2] = pc_mulc(v[k2], tw.w2[k2 - 1]);
    pdft8<true>(v);
    p512_xchg1_inv(v, buf, l);
#pragma unroll
    for (int k1 = 1; k1 < 8; ++k1) v[k1] = pc_mulc(v[k1], tw.w1[k1 - 1]);
    pdft8<true>(v);
}

}  // namespace dev
}  // namespace crlot
