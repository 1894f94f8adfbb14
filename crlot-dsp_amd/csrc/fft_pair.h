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

#include <type_traits>

#include "fft_wave.h"

namespace crlot {
namespace dev {

// Bin index of register d in lane `lane` after pair_fft_fwd.
__host__ __device__ constexpr int pair_bin_lane(int lane) {
    return (lane & 3) + 4 * (lane >> 4) + 16 * ((lane >> 2) & 3);
}
__host__ __device__ constexpr int pair_bin(int lane, int d) { return pair_bin_lane(lane) + 64 * d; }

// Packed complex: (re, im) in one 64-bit register pair, so every complex add is
// ONE v_pk_add_f32 and every rotation two packed ops (v_pk_mul_f32 +
// v_pk_fma_f32; swaps and sign flips ride on op_sel / neg modifiers).  On
// gfx950 a packed op moves twice the data per issue of a scalar one at about
// 1.2x its issue cost (tools/ubench/valu_issue.hip), and at 4 waves per SIMD
// this kernel is issue-bound, not VALU-throughput-bound.
typedef float pc __attribute__((ext_vector_type(2)));

__device__ __forceinline__ pc pc_mk(float r, float i) { return (pc){r, i}; }

// Single packed instructions with the operand swaps / sign flips as VOP3P
// modifiers (op_sel: half for the low lane, op_sel_hi: half for the high lane,
// neg_lo / neg_hi: negate that lane's operand).  Written out because the
// compiler materialises some of these shuffles with v_xor / v_mov.
// (a.x + b.y, a.y - b.x)
__device__ __forceinline__ pc pk_add_sw_nh(pc a, pc b) {
    pc r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// (a.x - b.y, a.y + b.x)
__device__ __forceinline__ pc pk_add_sw_nl(pc a, pc b) {
    pc r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// (a.y - a.x, -a.x - a.y)
__device__ __forceinline__ pc pk_w6f(pc a) {
    pc r;
    asm("v_pk_add_f32 %0, %1, %1 op_sel:[1,0] op_sel_hi:[0,1] neg_lo:[0,1] neg_hi:[1,1]" : "=v"(r) : "v"(a));
    return r;
}
// (-a.y - a.x, a.x - a.y)
__device__ __forceinline__ pc pk_w6i(pc a) {
    pc r;
    asm("v_pk_add_f32 %0, %1, %1 op_sel:[1,0] op_sel_hi:[0,1] neg_lo:[1,1] neg_hi:[0,1]" : "=v"(r) : "v"(a));
    return r;
}
// a * w = (a.x w.x - a.y w.y, a.x w.y + a.y w.x): one rounded product, one fma
__device__ __forceinline__ pc pc_mul(pc a, pc w) {
    pc p, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(p) : "v"(a), "v"(w));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
        : "=v"(r) : "v"(a), "v"(w), "v"(p));
    return r;
}
// a * conj(w) = (a.x w.x + a.y w.y, a.y w.x - a.x w.y)
__device__ __forceinline__ pc pc_mulc(pc a, pc w) {
    pc p, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1] neg_hi:[0,1]" : "=v"(p) : "v"(a), "v"(w));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1]" : "=v"(r) : "v"(a), "v"(w), "v"(p));
    return r;
}
// min(|a|, |b|, c) in one instruction (finite operands)
__device__ __forceinline__ float min3_abs(float a, float b, float c) {
    float r;
    asm("v_min3_f32 %0, |%1|, |%2|, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// min(e, frexp exponents of the 14 values a[0..7) .x/.y), computed only when some
// lane has smin < thr: a wave-uniform skip written inside one asm block, so the
// register allocator sees straight-line code (a C++ branch here costs the walker
// VGPR spills).
__device__ __forceinline__ int frexp_min_if(const pc* a, float smin, int e, float thr = 0x1p-89f) {
    int t0, t1;
    asm volatile("v_cmp_gt_f32 vcc, %[th], %[sm]\n\t"
                 "s_cbranch_vccz .Lfx_skip%=\n\t"
                 "v_frexp_exp_i32_f32 %[t0], %[x0]\n\t"
                 "v_frexp_exp_i32_f32 %[t1], %[y0]\n\t"
                 "v_min3_i32 %[e], %[t0], %[t1], %[e]\n\t"
                 "v_frexp_exp_i32_f32 %[t0], %[x1]\n\t"
                 "v_frexp_exp_i32_f32 %[t1], %[y1]\n\t"
                 "v_min3_i32 %[e], %[t0], %[t1], %[e]\n\t"
                 "v_frexp_exp_i32_f32 %[t0], %[x2]\n\t"
                 "v_frexp_exp_i32_f32 %[t1], %[y2]\n\t"
                 "v_min3_i32 %[e], %[t0], %[t1], %[e]\n\t"
                 "v_frexp_exp_i32_f32 %[t0], %[x3]\n\t"
                 "v_frexp_exp_i32_f32 %[t1], %[y3]\n\t"
                 "v_min3_i32 %[e], %[t0], %[t1], %[e]\n\t"
                 "v_frexp_exp_i32_f32 %[t0], %[x4]\n\t"
                 "v_frexp_exp_i32_f32 %[t1], %[y4]\n\t"
                 "v_min3_i32 %[e], %[t0], %[t1], %[e]\n\t"
                 "v_frexp_exp_i32_f32 %[t0], %[x5]\n\t"
                 "v_frexp_exp_i32_f32 %[t1], %[y5]\n\t"
                 "v_min3_i32 %[e], %[t0], %[t1], %[e]\n\t"
                 "v_frexp_exp_i32_f32 %[t0], %[x6]\n\t"
                 "v_frexp_exp_i32_f32 %[t1], %[y6]\n\t"
                 "v_min3_i32 %[e], %[t0], %[t1], %[e]\n\t"
                 ".Lfx_skip%=:"
                 : [e] "+v"(e), [t0] "=&v"(t0), [t1] "=&v"(t1)
                 : [sm] "v"(smin), [th] "s"(thr), [x0] "v"(a[0].x), [y0] "v"(a[0].y), [x1] "v"(a[1].x), [y1] "v"(a[1].y), [x2] "v"(a[2].x), [y2] "v"(a[2].y), [x3] "v"(a[3].x), [y3] "v"(a[3].y), [x4] "v"(a[4].x), [y4] "v"(a[4].y), [x5] "v"(a[5].x), [y5] "v"(a[5].y), [x6] "v"(a[6].x), [y6] "v"(a[6].y)
                 : "vcc");
    return e;
}
// The output sanitize's threshold test of the hot walkers, screened: the
// smallest frexp exponent over the first E registers' 2E values (zero's being 0), as
// min over every value would give wherever it can reach 2^MIN_EXP.  The window-edge
// registers (0 and E-1: the taps a window zeroes, whose outputs are often exact
// zeros) take the exact test; elsewhere min |v| >= thr on every lane (half a
// v_min3 per value) proves the test passes, and only a wave where some lane fails
// the screen (exact zero outputs: silence, zero-padded stream ends; or a tiny
// one) runs the exact test on the interior registers as well.
template <int E, int NV>
__device__ __forceinline__ int out_min_exp_screened(const pc (&v)[NV], float thr) {
    static_assert((E == 8 || E == 15 || E == 16) && NV >= E, "registers");
    const int e0 = min(min(__builtin_amdgcn_frexp_expf(v[0].x), __builtin_amdgcn_frexp_expf(v[0].y)),
                       min(__builtin_amdgcn_frexp_expf(v[E - 1].x), __builtin_amdgcn_frexp_expf(v[E - 1].y)));
    float s2[2] = {0x1p100f, 0x1p100f};
#pragma unroll
    for (int m = 1; m < E - 1; ++m) s2[m & 1] = min3_abs(v[m].x, v[m].y, s2[m & 1]);
    const float sm = __builtin_fminf(s2[0], s2[1]);
    int e = frexp_min_if(v + 1, sm, e0, thr);
    if constexpr (E > 8) e = frexp_min_if(v + 8, sm, e, thr);  // (E = 15: v[8..14])
    return e;
}
template <bool INV>
__device__ __forceinline__ pc pc_tw(pc a, pc w) { return INV ? pc_mulc(a, w) : pc_mul(a, w); }

// The same two instructions issued apart: a VOP3P result read by the next VOP3P
// right away costs a wait state (s_nop 0) on gfx950, so a run of rotations is
// issued skewed -- product i+1 before the fma of i (pc_tw_run).
template <bool INV>
__device__ __forceinline__ pc pc_tw_p(pc a, pc w) {
    pc p;
    if constexpr (INV)
        asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1] neg_hi:[0,1]" : "=v"(p) : "v"(a), "v"(w));
    else
        asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(p) : "v"(a), "v"(w));
    return p;
}
template <bool INV>
__device__ __forceinline__ pc pc_tw_f(pc a, pc w, pc p) {
    pc r;
    if constexpr (INV)
        asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1]" : "=v"(r) : "v"(a), "v"(w), "v"(p));
    else
        asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
            : "=v"(r) : "v"(a), "v"(w), "v"(p));
    return r;
}
// v[idx[i]] *= w[i] (conj for INV), i < K, skewed by one.
template <bool INV, int K, typename WF>
__device__ __forceinline__ void pc_tw_run(pc* v, const int (&idx)[K], WF w) {
    pc pp = pc_tw_p<INV>(v[idx[0]], w(0));
#pragma unroll
    for (int i = 1; i < K; ++i) {
        const pc pn = pc_tw_p<INV>(v[idx[i]], w(i));
        v[idx[i - 1]] = pc_tw_f<INV>(v[idx[i - 1]], w(i - 1), pp);
        pp = pn;
    }
    v[idx[K - 1]] = pc_tw_f<INV>(v[idx[K - 1]], w(K - 1), pp);
}
// a + m(b) and a - m(b), m = multiply by -i (forward) / +i (inverse)
template <bool INV>
__device__ __forceinline__ pc pc_add_mi(pc a, pc b) { return INV ? pk_add_sw_nl(a, b) : pk_add_sw_nh(a, b); }
template <bool INV>
__device__ __forceinline__ pc pc_sub_mi(pc a, pc b) { return INV ? pk_add_sw_nh(a, b) : pk_add_sw_nl(a, b); }

// DFT4; with MI2 the third input arrives as m^-1(x2) and is rotated on the fly
template <bool INV, bool MI2 = false>
__device__ __forceinline__ void pdft4(pc& x0, pc& x1, pc& x2, pc& x3) {
    const pc s0 = MI2 ? pc_add_mi<INV>(x0, x2) : x0 + x2;
    const pc s1 = MI2 ? pc_sub_mi<INV>(x0, x2) : x0 - x2;
    const pc s2 = x1 + x3, d3 = x1 - x3;
    x0 = s0 + s2;
    x2 = s0 - s2;
    x1 = pc_add_mi<INV>(s1, d3);
    x3 = pc_sub_mi<INV>(s1, d3);
}

// a * W16^j (forward) / conj (inverse) for the fixed rotations of a 16-point DFT.
// W8-type rotations (j = 2, 6) as h * (a + ...) : one add + one multiply.
template <bool INV, int J>
__device__ __forceinline__ pc rot16(pc a) {
    constexpr float c1 = 0.92387953251128675613f;  // cos(pi/8)
    constexpr float s1 = 0.38268343236508977173f;  // sin(pi/8)
    constexpr float h = 0.70710678118654752440f;   // sqrt(1/2)
    if constexpr (J == 1) return pc_tw<INV>(a, (pc){c1, -s1});
    if constexpr (J == 3) return pc_tw<INV>(a, (pc){s1, -c1});
    if constexpr (J == 9) return pc_tw<INV>(a, (pc){-c1, s1});
    // W^2 = h (1 - i): fwd h (a.x + a.y, a.y - a.x), inv h (a.x - a.y, a.y + a.x)
    if constexpr (J == 2) return (pc){h, h} * (INV ? pk_add_sw_nl(a, a) : pk_add_sw_nh(a, a));
    // W^6 = h (-1 - i): fwd h (a.y - a.x, -a.x - a.y), inv h (-a.x - a.y, a.x - a.y)
    if constexpr (J == 6) return (pc){h, h} * (INV ? pk_w6i(a) : pk_w6f(a));
    static_assert(J == 1 || J == 2 || J == 3 || J == 6 || J == 9, "rotation");
    return a;
}

// rot16 in two halves: _a (the product, or the W8-type add) and _b (the fma, or
// the scale by sqrt(1/2)).
template <bool INV, int J>
__device__ __forceinline__ pc rot16_a(pc a) {
    constexpr float c1 = 0.92387953251128675613f, s1 = 0.38268343236508977173f;
    if constexpr (J == 1) return pc_tw_p<INV>(a, (pc){c1, -s1});
    if constexpr (J == 3) return pc_tw_p<INV>(a, (pc){s1, -c1});
    if constexpr (J == 9) return pc_tw_p<INV>(a, (pc){-c1, s1});
    if constexpr (J == 2) return INV ? pk_add_sw_nl(a, a) : pk_add_sw_nh(a, a);
    if constexpr (J == 6) return INV ? pk_w6i(a) : pk_w6f(a);
    return a;
}
template <bool INV, int J>
__device__ __forceinline__ pc rot16_b(pc a, pc m) {
    constexpr float c1 = 0.92387953251128675613f, s1 = 0.38268343236508977173f;
    constexpr float h = 0.70710678118654752440f;
    if constexpr (J == 1) return pc_tw_f<INV>(a, (pc){c1, -s1}, m);
    if constexpr (J == 3) return pc_tw_f<INV>(a, (pc){s1, -c1}, m);
    if constexpr (J == 9) return pc_tw_f<INV>(a, (pc){-c1, s1}, m);
    return (pc){h, h} * m;  // J = 2, 6
}

// ---- FMA-fused (Goedecker) butterflies.  A twiddle w = C (1 + i T) (C = Re w,
// T = Im w / Re w) is applied as y = x + T (i x): ONE v_pk_fma_f32 whose
// operand swap and signs are op_sel / neg modifiers; C is left pending and
// multiplies the next butterfly's add as an fma, so a twiddled radix-4
// butterfly costs 11 packed operations instead of 14 (3 rotations of 2 + 8
// adds).  The constants sit in SGPR pairs (K[SEL] picks a half).
// b + (NEG ? -K[SEL] : K[SEL]) * a
template <int SEL, bool NEG>
__device__ __forceinline__ pc pk_fmak(pc a, pc k, pc b) {
    pc r;
    if constexpr (SEL == 0 && !NEG)
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(a), "s"(k), "v"(b));
    else if constexpr (SEL == 0 && NEG)
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1] neg_lo:[0,1,0] neg_hi:[0,1,0]" : "=v"(r) : "v"(a), "s"(k), "v"(b));
    else if constexpr (SEL == 1 && !NEG)
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "=v"(r) : "v"(a), "s"(k), "v"(b));
    else
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[1,1,1] neg_lo:[0,1,0] neg_hi:[0,1,0]" : "=v"(r) : "v"(a), "s"(k), "v"(b));
    return r;
}
// (b.x + sl K[SEL] a.y, b.y + sh K[SEL] a.x), sl = NL ? -1 : 1, sh = NH ? -1 : 1
template <int SEL, bool NL, bool NH>
__device__ __forceinline__ pc pk_fmasw(pc a, pc k, pc b) {
    static_assert(NL != NH, "one half negated");
    pc r;
    if constexpr (SEL == 0 && NL)
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_lo:[0,1,0]" : "=v"(r) : "v"(a), "s"(k), "v"(b));
    else if constexpr (SEL == 0 && NH)
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_hi:[0,1,0]" : "=v"(r) : "v"(a), "s"(k), "v"(b));
    else if constexpr (SEL == 1 && NL)
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[0,1,0]" : "=v"(r) : "v"(a), "s"(k), "v"(b));
    else
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[0,1,0]" : "=v"(r) : "v"(a), "s"(k), "v"(b));
    return r;
}
// y = x + T (i x) with T = +K[SEL] (POS) or -K[SEL]
template <int SEL, bool POS>
__device__ __forceinline__ pc pk_yform(pc x, pc k) { return pk_fmasw<SEL, POS, !POS>(x, k, x); }
// b + K[SEL] m(a) (PLUS) or b - K[SEL] m(a); m = multiply by -i (forward) / +i (inverse)
template <bool INV, bool PLUS, int SEL>
__device__ __forceinline__ pc pk_fma_mi(pc a, pc k, pc b) { return pk_fmasw<SEL, PLUS == INV, PLUS != INV>(a, k, b); }
// y = x + T (i x) for T = +1 (POS) / -1: one v_pk_add_f32
template <bool POS>
__device__ __forceinline__ pc pk_yform1(pc x) { return POS ? pk_add_sw_nl(x, x) : pk_add_sw_nh(x, x); }

// The same two forms with a per-lane constant pair K in VGPRs.
template <int SEL, bool NEG>
__device__ __forceinline__ pc pk_fmak_v(pc a, pc k, pc b) {
    pc r;
    if constexpr (SEL == 0 && !NEG)
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(a), "v"(k), "v"(b));
    else if constexpr (SEL == 0 && NEG)
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1] neg_lo:[0,1,0] neg_hi:[0,1,0]" : "=v"(r) : "v"(a), "v"(k), "v"(b));
    else if constexpr (SEL == 1 && !NEG)
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "=v"(r) : "v"(a), "v"(k), "v"(b));
    else
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[1,1,1] neg_lo:[0,1,0] neg_hi:[0,1,0]" : "=v"(r) : "v"(a), "v"(k), "v"(b));
    return r;
}
template <int SEL, bool NL, bool NH>
__device__ __forceinline__ pc pk_fmasw_v(pc a, pc k, pc b) {
    static_assert(NL != NH, "one half negated");
    pc r;
    if constexpr (SEL == 0 && NL)
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_lo:[0,1,0]" : "=v"(r) : "v"(a), "v"(k), "v"(b));
    else if constexpr (SEL == 0 && NH)
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_hi:[0,1,0]" : "=v"(r) : "v"(a), "v"(k), "v"(b));
    else if constexpr (SEL == 1 && NL)
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[0,1,0]" : "=v"(r) : "v"(a), "v"(k), "v"(b));
    else
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[0,1,0]" : "=v"(r) : "v"(a), "v"(k), "v"(b));
    return r;
}
// a * K.y (both halves)
__device__ __forceinline__ pc pk_mul_hi_v(pc a, pc k) {
    pc r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]" : "=v"(r) : "v"(a), "v"(k));
    return r;
}
// twiddle w = C (1 + i T) held as K = (T, C): y = x + T (i x) (CONJ: x - T (i x))
template <bool CONJ>
__device__ __forceinline__ pc pk_yform_v(pc x, pc tc) { return pk_fmasw_v<0, !CONJ, CONJ>(x, tc, x); }
// x * w (CONJ: x * conj w) with w held as (T, C): two operations, as pc_mul
template <bool CONJ>
__device__ __forceinline__ pc pk_tw_tc(pc x, pc tc) { return pk_mul_hi_v(pk_yform_v<CONJ>(x, tc), tc); }
// (T, C) of a unit twiddle given as (cos, sin); C != 0 for every table entry it is used on
__device__ __forceinline__ pc tw_tc(pc w) { return (pc){w.y / w.x, w.x}; }

// 16-point DFT constants: cos(pi/8), sin(pi/8); tan(pi/8), tan(3 pi/8); sqrt(1/2)
__device__ __forceinline__ pc k16_cs() { return (pc){0.92387953251128675613f, 0.38268343236508977173f}; }
__device__ __forceinline__ pc k16_tt() { return (pc){0.41421356237309504880f, 2.41421356237309504880f}; }
__device__ __forceinline__ pc k16_h() { return (pc){0.70710678118654752440f, 0.70710678118654752440f}; }

// In-place 16-point DFT, natural order in and out: X[k] = sum_n x[n] W16^{+-nk}.
// n = 4 n1 + n2, k = k1 + 4 k2: four DFT4 over n1, then four DFT4 over n2 whose
// inputs carry W16^{n2 k1} -- in the Goedecker form above (72 packed operations,
// 80 with explicit rotations); outputs renamed in registers, no data movement.
//   k1 = 1: W^1 = C1 (1 -+ i t8), W^2 = h (1 -+ i), W^3 = S1 (1 -+ i t38)
//   k1 = 2: W^2 (x9 + m x11), W^4 = m (free), as h (1 -+ i)
//   k1 = 3: W^3, W^6 = -h (1 +- i), W^9 = -C1 (1 -+ i t8)
// (upper signs forward; C1 = cos pi/8, S1 = sin pi/8, t8 = tan pi/8, t38 = tan 3pi/8)
// the second layer of pdft16_fma (inputs a[n2][k1] at x[n2 + 4 k1]) and the
// output renaming
template <bool INV>
__device__ __forceinline__ void pdft16_fma_l2(pc (&x)[16]) {
    const pc kcs = k16_cs(), ktt = k16_tt(), kh = k16_h();
    // the twiddled inputs' forms: k1 = 1 (x5, x6, x7), k1 = 3 (x13, x14, x15), k1 = 2 (x9 +- m x11)
    const pc y5 = pk_yform<0, INV>(x[5], ktt);   // T = -+ t8
    const pc y13 = pk_yform<1, INV>(x[13], ktt);  // T = -+ t38
    const pc p = pc_add_mi<INV>(x[9], x[11]);
    const pc y6 = pk_yform1<INV>(x[6]);           // T = -+ 1
    const pc y14 = pk_yform1<!INV>(x[14]);        // T = +- 1
    const pc q = pc_sub_mi<INV>(x[9], x[11]);
    const pc y7 = pk_yform<1, INV>(x[7], ktt);   // T = -+ t38
    const pc y15 = pk_yform<0, INV>(x[15], ktt);  // T = -+ t8
    const pc yp = pk_yform1<INV>(p), yq = pk_yform1<INV>(q);
    // first adds: u0 +- u2 and (u1 +- u3) / C(u1)
    const pc a0 = pk_fmak<0, false>(y6, kh, x[4]), a1 = pk_fmak<0, true>(y6, kh, x[4]);
    const pc b0 = pk_fmak<0, true>(y14, kh, x[12]), b1 = pk_fmak<0, false>(y14, kh, x[12]);
    const pc c0 = pc_add_mi<INV>(x[8], x[10]), c1 = pc_sub_mi<INV>(x[8], x[10]);
    const pc a2 = pk_fmak<0, false>(y7, ktt, y5), a3 = pk_fmak<0, true>(y7, ktt, y5);      // R = S1 / C1 = t8
    const pc b2 = pk_fmak<1, true>(y15, ktt, y13), b3 = pk_fmak<1, false>(y15, ktt, y13);  // R = -C1 / S1 = -t38
    pdft4<INV>(x[0], x[1], x[2], x[3]);
    // outputs: X[k1 + 4 k2] at x[4 k1 + k2]
    x[4] = pk_fmak<0, false>(a2, kcs, a0);
    x[12] = pk_fmak<1, false>(b2, kcs, b0);
    x[8] = pk_fmak<0, false>(yp, kh, c0);
    x[6] = pk_fmak<0, true>(a2, kcs, a0);
    x[14] = pk_fmak<1, true>(b2, kcs, b0);
    x[10] = pk_fmak<0, true>(yp, kh, c0);
    x[5] = pk_fma_mi<INV, true, 0>(a3, kcs, a1);
    x[13] = pk_fma_mi<INV, true, 1>(b3, kcs, b1);
    x[9] = pk_fma_mi<INV, true, 0>(yq, kh, c1);
    x[7] = pk_fma_mi<INV, false, 0>(a3, kcs, a1);
    x[15] = pk_fma_mi<INV, false, 1>(b3, kcs, b1);
    x[11] = pk_fma_mi<INV, false, 0>(yq, kh, c1);
    pc y[16];
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1)
#pragma unroll
        for (int k2 = 0; k2 < 4; ++k2) y[k1 + 4 * k2] = x[4 * k1 + k2];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = y[i];
}
template <bool INV>
__device__ __forceinline__ void pdft16_fma(pc (&x)[16]) {
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) pdft4<INV>(x[n2], x[n2 + 4], x[n2 + 8], x[n2 + 12]);
    pdft16_fma_l2<INV>(x);
}

// The same DFT with explicit rotations (80 packed operations); kept for A/B
// builds (-DCRLOT_PDFT16_CLASSIC).
template <bool INV>
__device__ __forceinline__ void pdft16_rot(pc (&x)[16]) {
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) pdft4<INV>(x[n2], x[n2 + 4], x[n2 + 8], x[n2 + 12]);
    // a[n2][k1] now at x[n2 + 4 k1]; multiply by W16^{n2 k1} (first halves of the
    // two-instruction rotations issued one ahead of their second halves)
    // (W^4 = -i on x[2 + 4 * 2] is applied inside the k1 = 2 DFT4 below)
    {
        pc m5 = rot16_a<INV, 1>(x[5]);
        const pc m9 = rot16_a<INV, 2>(x[9]);
        x[5] = rot16_b<INV, 1>(x[5], m5);
        const pc m13 = rot16_a<INV, 3>(x[13]);
        x[9] = rot16_b<INV, 2>(x[9], m9);
        const pc m6 = rot16_a<INV, 2>(x[6]);
        x[13] = rot16_b<INV, 3>(x[13], m13);
        const pc m14 = rot16_a<INV, 6>(x[14]);
        x[6] = rot16_b<INV, 2>(x[6], m6);
        const pc m7 = rot16_a<INV, 3>(x[7]);
        x[14] = rot16_b<INV, 6>(x[14], m14);
        const pc m11 = rot16_a<INV, 6>(x[11]);
        x[7] = rot16_b<INV, 3>(x[7], m7);
        m5 = rot16_a<INV, 9>(x[15]);
        x[11] = rot16_b<INV, 6>(x[11], m11);
        x[15] = rot16_b<INV, 9>(x[15], m5);
    }
    pdft4<INV>(x[0], x[1], x[2], x[3]);
    pdft4<INV>(x[4], x[5], x[6], x[7]);
    pdft4<INV, true>(x[8], x[9], x[10], x[11]);
    pdft4<INV>(x[12], x[13], x[14], x[15]);
    // X[k1 + 4 k2] sits at x[4 k1 + k2]: transpose the 4x4 register grid
    pc y[16];
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1)
#pragma unroll
        for (int k2 = 0; k2 < 4; ++k2) y[k1 + 4 * k2] = x[4 * k1 + k2];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = y[i];
}

template <bool INV>
__device__ __forceinline__ void pdft16(pc (&x)[16]) {
#ifdef CRLOT_PDFT16_CLASSIC
    pdft16_rot<INV>(x);
#else
    pdft16_fma<INV>(x);
#endif
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
__device__ __forceinline__ void lane_reg_swap(pc (&v)[16]) {
#ifdef CRLOT_ABL_NOPERM  // timing-only ablation: wrong results
    return;
#endif
#pragma unroll
    for (int r = 0; r < 16; ++r)
        if (!(r & 4)) {
            float ar = v[r].x, ai = v[r].y, br = v[r | 4].x, bi = v[r | 4].y;
            swap_f(ar, br, false);
            swap_f(ai, bi, false);
            v[r] = pc_mk(ar, ai);
            v[r | 4] = pc_mk(br, bi);
        }
#pragma unroll
    for (int r = 0; r < 16; ++r)
        if (!(r & 8)) {
            float ar = v[r].x, ai = v[r].y, br = v[r | 8].x, bi = v[r | 8].y;
            swap_f(ar, br, true);
            swap_f(ai, bi, true);
            v[r] = pc_mk(ar, ai);
            v[r | 8] = pc_mk(br, bi);
        }
}

// The same swap through LDS (one write and one read of every register, 16-lane
// write groups and 32-lane read groups each on distinct banks):
//   old (lane x + 16 q, reg a + 4 b) at x + 16 q + 64 a + 272 b (complex units),
//   read back as (lane x + 16 b, reg a + 4 q).
__device__ __forceinline__ void lane_reg_swap_lds(pc (&v)[16], pc* buf, int lane) {
    const int x = lane & 15, q = lane >> 4;
    pc* wb = buf + x + 16 * q;
    const pc* rb = buf + x + 272 * q;
#pragma unroll
    for (int r = 0; r < 16; ++r) wb[64 * (r & 3) + 272 * (r >> 2)] = v[r];
    wave_lds_fence();
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = rb[16 * (r >> 2) + 64 * (r & 3)];
    wave_lds_fence();
}
template <int MODE>
__device__ __forceinline__ void lane_reg_swap_any(pc (&v)[16], pc* buf, int lane) {
    if constexpr (MODE == 1)
        lane_reg_swap_lds(v, buf, lane);
    else
        lane_reg_swap(v);
}
#ifndef CRLOT_PAIR_SWAP_LDS
#define CRLOT_PAIR_SWAP_LDS 0  // measured: the LDS swap costs as many cycles as the permlanes and more power
#endif

// 16x16 transpose inside each quarter wave through LDS: lane (x + 16 q),
// register y  ->  lane (y + 16 q), register x.  Layout: q * 288 + 18 * row + col
// (complex units): ds_write_b64 groups of 16 lanes hit 16 consecutive elements,
// and each lane reads its 16 elements as 8 ds_read_b128 of 16-byte aligned pairs
// whose starting banks 4 (9 x mod 16) are distinct in every b128 lane group --
// conflict free; every address is one per-lane base plus an immediate.
constexpr int kPairXbuf = 4 * 288;  // complex elements per wave
__device__ __forceinline__ void transpose16(pc (&v)[16], pc* buf, int lane) {
#ifdef CRLOT_ABL_NOXPOSE  // timing-only ablation: wrong results
    return;
#endif
    const int q = lane >> 4, x = lane & 15;
    pc* wb = buf + q * 288 + x;
    const float4* rb = reinterpret_cast<const float4*>(buf + q * 288 + 18 * x);
#pragma unroll
    for (int y = 0; y < 16; ++y) wb[18 * y] = v[y];
    wave_lds_fence();
#pragma unroll
    for (int y = 0; y < 8; ++y) {
        const float4 t = rb[y];
        v[2 * y] = pc_mk(t.x, t.y);
        v[2 * y + 1] = pc_mk(t.z, t.w);
    }
    wave_lds_fence();
}

// Twiddle table of the first pass, laid out for ds_read_b128: W1024^{l k1} for
// k1 = 2j+1+e at t1[j * 128 + 2 l + e] (j < 7), k1 = 15 at t1[896 + l].
constexpr int kPairT1 = 15 * 64;  // complex elements
__host__ __device__ constexpr int pair_t1_index(int k1, int l) {
    return k1 == 15 ? 896 + l : ((k1 - 1) >> 1) * 128 + 2 * l + ((k1 - 1) & 1);
}
template <bool INV>
__device__ __forceinline__ void pair_t1_apply(pc (&v)[16], const pc* const& t1, int lane) {
    const float4* t4 = reinterpret_cast<const float4*>(t1 + 2 * lane);
#pragma unroll
    for (int j = 0; j < 7; ++j) {
#ifdef CRLOT_ABL_NOT1  // timing-only ablation: twiddles from registers, wrong results
        const float4 t = make_float4(0.6f + j * 0.01f, 0.8f, 0.6f, -0.8f - j * 0.01f);
#else
        const float4 t = t4[j * 64];
#endif
        v[2 * j + 1] = pc_tw<INV>(v[2 * j + 1], pc_mk(t.x, t.y));
        v[2 * j + 2] = pc_tw<INV>(v[2 * j + 2], pc_mk(t.z, t.w));
    }
    v[15] = pc_tw<INV>(v[15], t1[896 + lane]);
}

// Register-resident twiddles (3 waves per SIMD builds): w1[k1 - 1] = W1024^{lane k1},
// w2[c - 1] = W64^{(lane & 15) c}.
struct PairTw {
    pc w1[15];
    pc w2[3];
};
__device__ __forceinline__ void pair_tw_load(PairTw& tw, const pc* t1, const pc* t2, int lane) {
#pragma unroll
    for (int k1 = 1; k1 < 16; ++k1) tw.w1[k1 - 1] = t1[pair_t1_index(k1, lane)];
#pragma unroll
    for (int c = 1; c < 4; ++c) tw.w2[c - 1] = t2[16 * (c - 1)];
}
template <bool INV>
__device__ __forceinline__ void pair_t1_apply(pc (&v)[16], const PairTw& tw, int) {
    constexpr int idx[15] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
    pc_tw_run<INV>(v, idx, [&](int i) { return tw.w1[i]; });
}
__device__ __forceinline__ pc pair_t2(const pc* t2, int c) { return t2[16 * (c - 1)]; }
__device__ __forceinline__ pc pair_t2(const PairTw& tw, int c) { return tw.w2[c - 1]; }

// The same twiddles in the FMA-fused form (the release layout at H = 256).  The
// inverse runs decimation in time, so its twiddles sit on the INPUTS of the next
// radix-4 butterflies and fuse into them (Goedecker): per butterfly the input of
// index 2 keeps an explicit rotation (its C can be 0: W64^16 = -i at lane 8),
// inputs 1 and 3 become y = x - T (i x) with C1 pending and the ratio C3 / C1
// folded into the add -- 12 packed operations per radix-4 instead of 14.  The
// forward (decimation in frequency) applies the same twiddles explicitly, two
// operations each, as before.
// 15 per-lane twiddles w_k = W^{k}, k = 1..15 (geometric in k), FMA form:
// k in {1, 2, 3, 8, 9, 10, 11} as (cos, sin) in e[], k in {4..7, 12..15} as
// (T, C) in y[], r = C_{n+12} / C_{n+4} (n = 0..3); 34 VGPRs instead of 30.
struct Tw15F {
    pc e[7];
    pc y[8];
    pc r[2];
};
__host__ __device__ constexpr int tw15_e_slot(int k) { return k < 8 ? k - 1 : k - 5; }   // k in {1,2,3,8..11}
__host__ __device__ constexpr int tw15_y_slot(int k) { return k < 8 ? k - 4 : k - 8; }   // k in {4..7, 12..15}
__host__ __device__ constexpr bool tw15_is_e(int k) { return (k & 4) == 0; }
// w(k): (cos, sin) of w_k
template <typename WF>
__device__ __forceinline__ void tw15_load(Tw15F& tw, WF w) {
#pragma unroll
    for (int k = 1; k < 16; ++k) {
        if (tw15_is_e(k))
            tw.e[tw15_e_slot(k)] = w(k);
        else
            tw.y[tw15_y_slot(k)] = tw_tc(w(k));
    }
#pragma unroll
    for (int n = 0; n < 4; ++n) tw.r[n >> 1][n & 1] = tw.y[tw15_y_slot(n + 12)].y / tw.y[tw15_y_slot(n + 4)].y;
}
// forward (explicit, two operations each): v[k] *= w_k
__device__ __forceinline__ void tw15_apply_fwd(pc (&v)[16], const Tw15F& tw) {
#pragma unroll
    for (int k = 1; k < 16; ++k)
        v[k] = tw15_is_e(k) ? pc_mul(v[k], tw.e[tw15_e_slot(k)]) : pk_tw_tc<false>(v[k], tw.y[tw15_y_slot(k)]);
}
// inverse: conj(w_k) on register k fused with pdft16<true>'s first layer (one
// radix-4 over registers n, n+4, n+8, n+12 per n: inputs n and n+8 rotated
// explicitly, n+4 and n+12 in the y = x - T (i x) form, C_{n+4} pending), then
// pdft16<true>'s second layer.  54 + 40 packed operations instead of 30 + 72.
__device__ __forceinline__ void tw15_pdft16_inv(pc (&v)[16], const Tw15F& tw) {
#pragma unroll
    for (int n = 0; n < 4; ++n) {
        const pc u0 = n ? pc_mulc(v[n], tw.e[tw15_e_slot(n)]) : v[0];
        const pc u2 = pc_mulc(v[n + 8], tw.e[tw15_e_slot(n + 8)]);
        const pc tc = tw.y[tw15_y_slot(n + 4)];
        const pc y1 = pk_yform_v<true>(v[n + 4], tc);
        const pc y3 = pk_yform_v<true>(v[n + 12], tw.y[tw15_y_slot(n + 12)]);
        const pc s0 = u0 + u2, s1 = u0 - u2;
        pc s2, d3;
        if (n & 1) {
            s2 = pk_fmak_v<1, false>(y3, tw.r[n >> 1], y1);
            d3 = pk_fmak_v<1, true>(y3, tw.r[n >> 1], y1);
        } else {
            s2 = pk_fmak_v<0, false>(y3, tw.r[n >> 1], y1);
            d3 = pk_fmak_v<0, true>(y3, tw.r[n >> 1], y1);
        }
        v[n] = pk_fmak_v<1, false>(s2, tc, s0);
        v[n + 8] = pk_fmak_v<1, true>(s2, tc, s0);
        v[n + 4] = pk_fmasw_v<1, true, false>(d3, tc, s1);   // s1 + C (i d3)
        v[n + 12] = pk_fmasw_v<1, false, true>(d3, tc, s1);  // s1 - C (i d3)
    }
    pdft16_fma_l2<true>(v);
}

// K_pair's register twiddles in the FMA form: t1 = W1024^{l k} as a Tw15F; t2 =
// W64^{x c} (x = lane & 15): c = 2 as (cos, sin), c = 1, 3 as (T, C), rb.x = C3 / C1.
// Every C used as a divisor or pending factor is nonzero: cos(2 pi l k / 1024)
// for l < 64 and k in {4..7, 12..15} never meets a quarter turn (nor do the
// W4096 / W2048 / W256 / W128 tables of K_pair4k / K_pair2k), nor does
// cos(2 pi x c / 64) for x < 16 and c in {1, 3}; |T| <= 163 here (<= 652 at 4096).
struct PairTwF {
    Tw15F t1;
    pc w2, tc1, tc3, rb;
};
__device__ __forceinline__ void pair_tw_load(PairTwF& tw, const pc* t1, const pc* t2, int lane) {
    tw15_load(tw.t1, [&](int k) { return t1[pair_t1_index(k, lane)]; });
    const pc w1 = t2[0], w3 = t2[32];
    tw.w2 = t2[16];
    tw.tc1 = tw_tc(w1);
    tw.tc3 = tw_tc(w3);
    tw.rb = (pc){w3.x / w1.x, 0.f};
}
template <bool INV>
__device__ __forceinline__ void pair_t1_apply(pc (&v)[16], const PairTwF& tw, int) {
    static_assert(!INV, "the inverse fuses its t1 twiddles (tw15_pdft16_inv)");
    tw15_apply_fwd(v, tw.t1);
}
// forward t2: v[j + 4 c] *= W64^{x c}
__device__ __forceinline__ void pair_t2_fwd(pc (&v)[16], const PairTwF& tw) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        v[4 + j] = pk_tw_tc<false>(v[4 + j], tw.tc1);
        v[8 + j] = pc_mul(v[8 + j], tw.w2);
        v[12 + j] = pk_tw_tc<false>(v[12 + j], tw.tc3);
    }
}
// inverse: conj W64^{x c} on v[j + 4 c] fused into the radix-4 over c
__device__ __forceinline__ void pair_t2_dft4_inv(pc (&v)[16], const PairTwF& tw) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const pc u2 = pc_mulc(v[j + 8], tw.w2);
        const pc y1 = pk_yform_v<true>(v[j + 4], tw.tc1);
        const pc y3 = pk_yform_v<true>(v[j + 12], tw.tc3);
        const pc s0 = v[j] + u2, s1 = v[j] - u2;
        const pc s2 = pk_fmak_v<0, false>(y3, tw.rb, y1), d3 = pk_fmak_v<0, true>(y3, tw.rb, y1);
        v[j] = pk_fmak_v<1, false>(s2, tw.tc1, s0);
        v[j + 8] = pk_fmak_v<1, true>(s2, tw.tc1, s0);
        v[j + 4] = pk_fmasw_v<1, true, false>(d3, tw.tc1, s1);
        v[j + 12] = pk_fmasw_v<1, false, true>(d3, tw.tc1, s1);
    }
}

#ifdef CRLOT_PAIR_TW_CLASSIC
using PairTwReg = PairTw;
#else
using PairTwReg = PairTwF;
#endif

// Forward: natural z[lane + 64 m] -> bin-scrambled X (pair_bin).
//   t1: W1024^{l k1} (pair_t1_index), t2[16 (c - 1)] = W64^{(lane & 15) c} (LDS),
//   or both from a PairTw / PairTwF (T1 = the struct, t2 unused).
template <typename T1, typename T2>
__device__ __forceinline__ void pair_fft_fwd(pc (&v)[16], pc* buf, const T1& t1, const T2& t2, int lane) {
    pdft16<false>(v);
    pair_t1_apply<false>(v, t1, lane);
    lane_reg_swap_any<CRLOT_PAIR_SWAP_LDS>(v, buf, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) pdft4<false>(v[j], v[j + 4], v[j + 8], v[j + 12]);
    if constexpr (std::is_same_v<T2, PairTwF>) {
        pair_t2_fwd(v, t2);
    } else {
        constexpr int idx[12] = {4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
        pc_tw_run<false>(v, idx, [&](int i) { return pair_t2(t2, 1 + i / 4); });
    }
    transpose16(v, buf, lane);
    pdft16<false>(v);
}

// Inverse (unnormalised): bin-scrambled Y -> natural y[lane + 64 m].
template <typename T1, typename T2>
__device__ __forceinline__ void pair_fft_inv(pc (&v)[16], pc* buf, const T1& t1, const T2& t2, int lane) {
    pdft16<true>(v);
    transpose16(v, buf, lane);
    if constexpr (std::is_same_v<T2, PairTwF>) {
        pair_t2_dft4_inv(v, t2);
    } else {
        {
            constexpr int idx[12] = {4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
            pc_tw_run<true>(v, idx, [&](int i) { return pair_t2(t2, 1 + i / 4); });
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) pdft4<true>(v[j], v[j + 4], v[j + 8], v[j + 12]);
    }
    lane_reg_swap_any<CRLOT_PAIR_SWAP_LDS>(v, buf, lane);
    if constexpr (std::is_same_v<T1, PairTwF>) {
        tw15_pdft16_inv(v, t1.t1);
    } else {
        pair_t1_apply<true>(v, t1, lane);
        pdft16<true>(v);
    }
}

}  // namespace dev
}  // namespace crlot
