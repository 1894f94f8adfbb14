// fft_pairn.h -- N-point complex FFT of one 64-lane wave for a compile-time N
// whose factors are 2, 3, 5 and 7, in ONE LDS buffer of N elements: the
// frame-pair transform of the sizes that neither the register-resident
// power-of-two kernels nor K_pair15 (N = 15 L) take -- 882 and 1764 (20 / 40 ms
// at 44.1 kHz), 1920 (40 ms at 48 kHz), 1000, 640, 400, 320.
//
// Stockham autosort over a short list of composite radices (882 = 9 x 7 x 14,
// 1764 = 9 x 14 x 14, 1000 = 10 x 10 x 10 ...): pass i with radix R and sub-length
// ns (the product of the earlier radices) runs butterflies j < M = N / R:
// x_q = buf[j + q M] W_{ns R}^{q (j mod ns)}, an R-point DFT in registers,
// buf[(j / ns) ns R + j mod ns + q ns] = y_q.  Each lane reads and computes its
// butterflies (ceil(M / 64) of them), the wave fences, and the outputs are
// written back in place -- one buffer per transform.  Three passes instead of
// one per prime factor: every pass moves the whole transform through LDS twice,
// and LDS bandwidth is what bounds these sizes.
//
// The R-point DFT is written out at compile time: 2, 4 and the odd primes 3, 5,
// 7 directly (odd primes as the symmetric DFT: (R-1)/2 sums and differences,
// then (R-1)^2 / 2 multiply-adds for each half), composite R = A B as a
// Cooley-Tukey step in registers (B-point DFTs, constant twiddles W_R^{n1 k2},
// A-point DFTs; the index maps are register renames).  Natural order in and
// out.  The walker (pair_n.hip) fuses the first forward pass with the frame
// loads and the last inverse pass with the overlap-add.
#pragma once

#include "fft_pair.h"

namespace crlot {
namespace dev {

// ------------------------------------------------------------------ compile-time trig
struct PnCS {
    double c, s;
};
// cos / sin (2 pi a / b) by quadrant reduction and Taylor series (constexpr)
__host__ __device__ constexpr PnCS pn_cossin(long a, long b) {
    a %= b;
    if (a < 0) a += b;
    const long q = (4 * a) / b;  // quadrant
    const double pi = 3.14159265358979323846264338327950288;
    double x = 2.0 * pi * (double(4 * a - q * b) / double(4 * b));  // [0, pi/2)
    const bool co = x > pi / 4;
    if (co) x = pi / 2 - x;
    double x2 = x * x, ts = x, ss = x, tc = 1.0, sc = 1.0;
    for (int i = 1; i < 14; ++i) {
        ts *= -x2 / double((2 * i) * (2 * i + 1));
        ss += ts;
        tc *= -x2 / double((2 * i - 1) * (2 * i));
        sc += tc;
    }
    const double c = co ? ss : sc, s = co ? sc : ss;  // of the reduced angle
    switch (q) {
        case 0: return {c, s};
        case 1: return {-s, c};
        case 2: return {-c, -s};
        default: return {s, -c};
    }
}
template <int R>
struct PnTrig {
    float c[R], s[R];  // cos / sin (2 pi r / R)
};
template <int R>
__host__ __device__ constexpr PnTrig<R> pn_trig() {
    PnTrig<R> t{};
    for (int r = 0; r < R; ++r) {
        const PnCS w = pn_cossin(r, R);
        t.c[r] = float(w.c);
        t.s[r] = float(w.s);
    }
    return t;
}

// ------------------------------------------------------------------ plans
struct PnFac {
    int size = 0;    // N
    int n = 0;       // passes
    int r[8] = {};   // radices
    int ns[8] = {};  // sub-length before the pass
    int off[8] = {}; // twiddle offset: W_{ns r}^{q jm} at off + (q - 1) ns + jm (ns > 1)
    int tw_len = 0;  // complex twiddles over all passes
    int rest = 1;    // N / product of the radices (1 for a supported N)
};
__host__ __device__ constexpr PnFac pn_plan_of(int N, const int* rs, int k) {
    PnFac f{};
    f.size = N;
    int m = N, ns = 1, off = 0;
    for (int i = 0; i < k; ++i) {
        f.r[i] = rs[i];
        f.ns[i] = ns;
        f.off[i] = off;
        if (ns > 1) off += (rs[i] - 1) * ns;
        ns *= rs[i];
        m /= rs[i];
    }
    f.n = k;
    f.tw_len = off;
    f.rest = m;
    return f;
}
// Plan key K = N + 100000 V + 1000000 (L / 64 - 1) + 10000000 lean: V selects an
// alternative radix list (A/B builds), L the lanes one transform spans (64: one
// wave, 128: two waves of a workgroup, fenced with workgroup barriers); lean
// (the walker's) keeps the windows in global memory and an exact-size ring.
__host__ __device__ constexpr int pn_lanes(int K) { return 64 * (1 + (K % 10000000) / 1000000); }
__host__ __device__ constexpr PnFac pn_factor(int K) {
    // three passes each: the first radix is the pass fused with the frame loads,
    // the last the one fused with the overlap-add
    const int N = K % 100000, V = (K % 1000000) / 100000;
    // (measured, 1024 x 480 000: 882/441 {9,7,14} 229k, {18,7,7} 225k, {7,7,18} 221k,
    // {14,7,9} 220k; 1764/441 {9,14,14} 87.5k, {14,14,9} 82.7k, {7,7,36} 76.2k,
    // {12,7,21} 69.6k Msamples/s; profiles/r03_pn_plans.jsonl)
    constexpr int p882[4][3] = {{9, 7, 14}, {7, 7, 18}, {14, 7, 9}, {18, 7, 7}};
    constexpr int p1764[4][3] = {{9, 14, 14}, {7, 7, 36}, {14, 14, 9}, {12, 7, 21}};
    // 960 / 480 run on K_pair15 (register-resident: 194-197k / 197-203k against
    // 139k / 120k for the best lists here, profiles/r03_pn15_ab.jsonl); these
    // lists serve the -DCRLOT_PN_15 A/B build.  1920/480 (two waves per
    // transform): {15,8,16} 83.6k, {8,15,16} 75.8k, {16,15,8} 66.2k Msamples/s.
    constexpr int p960[4][3] = {{15, 8, 8}, {8, 8, 15}, {10, 12, 8}, {12, 10, 8}};
    constexpr int p480[4][3] = {{8, 6, 10}, {10, 6, 8}, {6, 8, 10}, {15, 4, 8}};
    constexpr int p1920[4][3] = {{15, 8, 16}, {8, 15, 16}, {16, 15, 8}, {12, 10, 16}};
    constexpr int p1000[3] = {10, 10, 10};
    constexpr int p640[3] = {8, 8, 10}, p400[3] = {8, 5, 10}, p320[3] = {8, 8, 5};
    if (V > 3) {
        PnFac f{};
        f.rest = N;
        return f;
    }
    switch (N) {
        case 882: return pn_plan_of(N, p882[V], 3);
        case 1764: return pn_plan_of(N, p1764[V], 3);
        case 960: return pn_plan_of(N, p960[V], 3);
        case 480: return pn_plan_of(N, p480[V], 3);
        case 1920: return pn_plan_of(N, p1920[V], 3);
        case 1000: return pn_plan_of(N, p1000, 3);
        case 640: return pn_plan_of(N, p640, 3);
        case 400: return pn_plan_of(N, p400, 3);
        case 320: return pn_plan_of(N, p320, 3);
        default: {
            PnFac f{};
            f.rest = N;
            return f;
        }
    }
}

// a * w (conj(w) for INV) for a compile-time w held in an SGPR pair: pc_tw's
// instructions with a scalar operand, so the walker's many constant twiddles are
// rematerialised with s_mov instead of occupying (and spilling) VGPR pairs.
template <bool INV>
__device__ __forceinline__ pc pc_tw_k(pc a, pc w) {
    pc p, r;
    if constexpr (INV) {
        asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1] neg_hi:[0,1]" : "=v"(p) : "v"(a), "s"(w));
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1]" : "=v"(r) : "v"(a), "s"(w), "v"(p));
    } else {
        asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(p) : "v"(a), "s"(w));
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
            : "=v"(r) : "v"(a), "s"(w), "v"(p));
    }
    return r;
}
// c * a + b for a compile-time scalar c (an SGPR pair {c, c})
__device__ __forceinline__ pc pfma_k(float c, pc a, pc b) {
    pc r;
    const pc k = {c, c};
    asm("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(r) : "s"(k), "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ pc pmul_k(float c, pc a) {
    pc r;
    const pc k = {c, c};
    asm("v_pk_mul_f32 %0, %1, %2" : "=v"(r) : "s"(k), "v"(a));
    return r;
}

// ------------------------------------------------------------------ R-point DFTs in registers
// a * W_R^e (forward; conjugate for INV), exact for quarter turns; e is a
// constant once the caller's loops unroll
template <bool INV, int R>
__device__ __forceinline__ pc pn_rot(pc a, int e) {
    constexpr PnTrig<R> T = pn_trig<R>();
    e %= R;
    if (e == 0) return a;
    if ((4 * e) % R == 0) {
        const int qt = (4 * e) / R;  // W^e = (-i)^qt
        if (qt == 2) return -a;
        if ((qt == 1) != INV) return pc_mk(a.y, -a.x);  // -i a
        return pc_mk(-a.y, a.x);                        // +i a
    }
    return pc_tw_k<INV>(a, (pc){T.c[e], -T.s[e]});  // W = cos - i sin
}

__host__ __device__ constexpr int pn_split(int R) {
    // the first radix of a composite R: 4, 2, 3, 5, 7 (smaller than R)
    return (R % 4 == 0 && R > 4)   ? 4
           : (R % 2 == 0 && R > 2) ? 2
           : (R % 3 == 0 && R > 3) ? 3
           : (R % 5 == 0 && R > 5) ? 5
           : (R % 7 == 0 && R > 7) ? 7
                                   : 1;
}

template <bool INV, int R>
__device__ __forceinline__ void pn_dft(pc* x) {
    if constexpr (R == 1) {
        return;
    } else if constexpr (R == 2) {
        const pc a = x[0], b = x[1];
        x[0] = a + b;
        x[1] = a - b;
    } else if constexpr (R == 4) {
        pdft4<INV>(x[0], x[1], x[2], x[3]);
    } else if constexpr (R == 3 || R == 5 || R == 7) {
        // y_s = x0 + sum_q c_qs t_q  -/+ i sum_q s_qs u_q  (t/u: x_q +/- x_{R-q})
        constexpr PnTrig<R> T = pn_trig<R>();
        constexpr int K = (R - 1) / 2;
        pc t[K], u[K];
#pragma unroll
        for (int q = 1; q <= K; ++q) {
            t[q - 1] = x[q] + x[R - q];
            u[q - 1] = x[q] - x[R - q];
        }
        const pc x0 = x[0];
        pc y0 = x0 + t[0];
#pragma unroll
        for (int q = 1; q < K; ++q) y0 = y0 + t[q];
        pc a[K], b[K];
#pragma unroll
        for (int s = 1; s <= K; ++s) {
            pc av = x0, bv = {0.0f, 0.0f};
#pragma unroll
            for (int q = 1; q <= K; ++q) {
                const float c = T.c[(q * s) % R], sv = T.s[(q * s) % R];
                av = pfma_k(c, t[q - 1], av);
                bv = q == 1 ? pmul_k(sv, u[0]) : pfma_k(sv, u[q - 1], bv);
            }
            a[s - 1] = av;
            b[s - 1] = bv;
        }
        x[0] = y0;
#pragma unroll
        for (int s = 1; s <= K; ++s) {
            x[s] = pc_add_mi<INV>(a[s - 1], b[s - 1]);
            x[R - s] = pc_sub_mi<INV>(a[s - 1], b[s - 1]);
        }
    } else {
        // R = A B: n = n1 + A n2, k = B k1 + k2;
        // X[B k1 + k2] = sum_n1 W_A^{n1 k1} W_R^{n1 k2} sum_n2 W_B^{n2 k2} x[n1 + A n2]
        constexpr int A = pn_split(R), B = R / A;
        static_assert(A > 1, "radix");
        pc y[R];
#pragma unroll
        for (int n1 = 0; n1 < A; ++n1) {
            pc t[B];
#pragma unroll
            for (int n2 = 0; n2 < B; ++n2) t[n2] = x[n1 + A * n2];
            pn_dft<INV, B>(t);
#pragma unroll
            for (int k2 = 0; k2 < B; ++k2) y[n1 * B + k2] = pn_rot<INV, R>(t[k2], n1 * k2);
        }
#pragma unroll
        for (int k2 = 0; k2 < B; ++k2) {
            pc u[A];
#pragma unroll
            for (int n1 = 0; n1 < A; ++n1) u[n1] = y[n1 * B + k2];
            pn_dft<INV, A>(u);
#pragma unroll
            for (int k1 = 0; k1 < A; ++k1) x[B * k1 + k2] = u[k1];
        }
    }
}

// ------------------------------------------------------------------ passes
template <int N, int I>
struct PnPass {
    static constexpr PnFac F = pn_factor(N);
    static constexpr int R = F.r[I], NS = F.ns[I], OFF = F.off[I];
    static constexpr int L = pn_lanes(N);  // lanes per transform
    static constexpr int M = F.size / R, ITS = (M + L - 1) / L;
    static constexpr bool FULL = M % L == 0;
    static __device__ __forceinline__ bool live(int it, int j) { return FULL || it + 1 < ITS || j < M; }
    // butterfly of iteration it: past M (the last iteration's idle lanes) the
    // lane recomputes butterfly M - 1, so every register is defined on every
    // path (no divergent branches around the DFTs; only stores are guarded)
    static __device__ __forceinline__ int bf(int lane, int it) {
        const int j = lane + L * it;
        return (FULL || it + 1 < ITS) ? j : min(j, M - 1);
    }
    // output index of register q of butterfly j
    static __device__ __forceinline__ int out(int j, int q) {
        const int jb = j / NS, jm = j - jb * NS;
        return jb * NS * R + jm + q * NS;
    }
};

// Twiddles and the R-point DFT of butterfly j (inputs already in x).
template <bool INV, int N, int I>
__device__ __forceinline__ void pn_bfly(pc* x, const pc* tw, int j) {
    using P = PnPass<N, I>;
    if constexpr (P::NS > 1) {
        const pc* t = tw + P::OFF + j % P::NS;
#pragma unroll
        for (int q = 1; q < P::R; ++q) {
            x[q] = pc_tw<INV>(x[q], t[(q - 1) * P::NS]);
            // large radices: twiddles in groups of 8 (their loads would otherwise
            // all be hoisted together, 2 R VGPRs on top of the inputs)
            if constexpr (P::R > 12)
                if (q % 8 == 0) __builtin_amdgcn_sched_barrier(0);
        }
    }
    pn_dft<INV, P::R>(x);
}

// Pass I read from buf and computed into x (not written back).
template <bool INV, int N, int I>
__device__ __forceinline__ void pn_pass_compute(const pc* buf, const pc* tw, int lane,
                                                pc (&x)[PnPass<N, I>::ITS][PnPass<N, I>::R]) {
    using P = PnPass<N, I>;
#pragma unroll
    for (int it = 0; it < P::ITS; ++it) {
        const int j = P::bf(lane, it);
#pragma unroll
        for (int q = 0; q < P::R; ++q) x[it][q] = buf[j + q * P::M];
        pn_bfly<INV, N, I>(x[it], tw, j);
        if constexpr (P::ITS * P::R > 12) __builtin_amdgcn_sched_barrier(0);  // one butterfly's loads at a time
    }
}
template <int N, int I>
__device__ __forceinline__ void pn_pass_store(pc* buf, int lane, const pc (&x)[PnPass<N, I>::ITS][PnPass<N, I>::R]) {
    using P = PnPass<N, I>;
#pragma unroll
    for (int it = 0; it < P::ITS; ++it) {
        const int j = lane + P::L * it;
        if (P::live(it, j)) {
            pc* o = buf + P::out(j, 0);
#pragma unroll
            for (int q = 0; q < P::R; ++q) o[q * P::NS] = x[it][q];
        }
    }
}

// The transform's LDS fence: the wave's own (one wave per transform) or the
// workgroup barrier (two waves per transform; every transform of the workgroup
// passes it together)
template <int K>
__device__ __forceinline__ void pn_fence() {
    if constexpr (pn_lanes(K) == 64)
        wave_lds_fence();
    else
        __syncthreads();
}

// Passes I .. I1-1 in place, each fenced after its reads and after its writes.
template <bool INV, int N, int I, int I1>
__device__ __forceinline__ void pn_passes(pc* buf, const pc* tw, int lane) {
    if constexpr (I < I1) {
        pc x[PnPass<N, I>::ITS][PnPass<N, I>::R];
        pn_pass_compute<INV, N, I>(buf, tw, lane, x);
        pn_fence<N>();
        pn_pass_store<N, I>(buf, lane, x);
        pn_fence<N>();
        pn_passes<INV, N, I + 1, I1>(buf, tw, lane);
    }
}

// The lane index through an opaque move: every pass's addresses depend only on
// it, and hoisted out of the caller's frame loop they would hold ~100 VGPRs for
// the whole walk; recomputed per transform they cost a few VALU.
__device__ __forceinline__ int pn_opaque(int lane) {
    int ln;
    asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
    return ln;
}

}  // namespace dev
}  // namespace crlot
