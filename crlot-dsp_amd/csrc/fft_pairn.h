// fft_pairn.h -- N-point complex FFT of one 64-lane wave for a compile-time N
// with small prime factors (2, 3, 5, 7), in ONE LDS buffer of N elements: the
// frame-pair transform of the sizes that neither the register-resident
// power-of-two kernels nor K_pair15 (N = 15 L) take -- 882 and 1764 (20 / 40 ms
// at 44.1 kHz), 1000, 640, 400, 320 ...
//
// Stockham autosort, pass i with radix R and sub-length ns (the product of the
// earlier radices), butterflies j < M = N / R: x_q = buf[j + q M] W_{ns R}^{q (j
// mod ns)}, a length-R DFT, buf[(j / ns) ns R + j mod ns + q ns] = y_q.  Every
// lane first reads all of its butterflies' inputs (ceil(M / 64) x R values into
// registers), the wave fences, then writes every output: in place, so one
// buffer per transform.  N, R, ns and the twiddle offsets are compile-time, so
// the butterfly loops unroll with constant strides and divisions.  Radix 7 (and
// 3, 5) is the symmetric odd-prime DFT: (R-1)/2 sums and differences, then
// (R-1)^2 / 2 packed multiply-adds for each half.  Natural order in and out.
#pragma once

#include "fft_pair.h"

namespace crlot {
namespace dev {

struct PnFac {
    int n = 0;          // passes
    int r[24] = {};     // radices
    int ns[24] = {};    // sub-length before the pass
    int off[24] = {};   // twiddle offset: W_{ns r}^{q jm} at off + (q - 1) ns + jm
    int tw_len = 0;     // complex twiddles over all passes
    int rest = 1;       // factor left over (1 when N is 2^a 3^b 5^c 7^d)
};
// radix order: 7s, 5s, 3s, then 4s and a last 2
__host__ __device__ constexpr PnFac pn_factor(int N) {
    PnFac f{};
    int m = N, ns = 1, off = 0;
    const int order[5] = {7, 5, 3, 4, 2};
    for (int oi = 0; oi < 5; ++oi) {
        const int d = order[oi];
        while (m % d == 0 && f.n < 24) {
            f.r[f.n] = d;
            f.ns[f.n] = ns;
            f.off[f.n] = off;
            off += (d - 1) * ns;
            ns *= d;
            m /= d;
            ++f.n;
        }
    }
    f.tw_len = off;
    f.rest = m;
    return f;
}

__device__ __forceinline__ pc pfma(pc a, pc b, pc c) { return __builtin_elementwise_fma(a, b, c); }

// Length-R DFT of x[0..R) in place (forward W_R = e^{-2 pi i / R}; INV conjugate).
template <bool INV, int R>
__device__ __forceinline__ void pn_bfly(pc* x) {
    if constexpr (R == 2) {
        const pc a = x[0], b = x[1];
        x[0] = a + b;
        x[1] = a - b;
    } else if constexpr (R == 4) {
        pdft4<INV>(x[0], x[1], x[2], x[3]);
    } else {
        // odd prime: y_s = x0 + sum_q c_qs t_q  -/+ i sum_q s_qs u_q  (t/u: x_q +/- x_{R-q})
        static_assert(R == 3 || R == 5 || R == 7, "radix");
        constexpr int K = (R - 1) / 2;
        // cos / sin (2 pi r / R), r = 0..R-1
        constexpr float C3[3] = {1.0f, -0.5f, -0.5f};
        constexpr float S3[3] = {0.0f, 0.86602540378443864676f, -0.86602540378443864676f};
        constexpr float C5[5] = {1.0f, 0.30901699437494742410f, -0.80901699437494742410f, -0.80901699437494742410f,
                                 0.30901699437494742410f};
        constexpr float S5[5] = {0.0f, 0.95105651629515357212f, 0.58778525229247312917f, -0.58778525229247312917f,
                                 -0.95105651629515357212f};
        constexpr float C7[7] = {1.0f,
                                 0.62348980185873353053f,
                                 -0.22252093395631440429f,
                                 -0.90096886790241912624f,
                                 -0.90096886790241912624f,
                                 -0.22252093395631440429f,
                                 0.62348980185873353053f};
        constexpr float S7[7] = {0.0f,
                                 0.78183148246802980871f,
                                 0.97492791218182360702f,
                                 0.43388373911755812048f,
                                 -0.43388373911755812048f,
                                 -0.97492791218182360702f,
                                 -0.78183148246802980871f};
        auto cs = [](int r) { return R == 3 ? C3[r] : R == 5 ? C5[r] : C7[r]; };
        auto sn = [](int r) { return R == 3 ? S3[r] : R == 5 ? S5[r] : S7[r]; };
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
            pc av = x0, bv;
#pragma unroll
            for (int q = 1; q <= K; ++q) {
                const float c = cs((q * s) % R), sv = sn((q * s) % R);
                av = pfma((pc){c, c}, t[q - 1], av);
                bv = q == 1 ? (pc){sv, sv} * u[0] : pfma((pc){sv, sv}, u[q - 1], bv);
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
    }
}

// Pass I of the N-point transform, in place in buf (one wave; fenced on both sides
// by the caller's previous pass / this one).
template <bool INV, int N, int I>
__device__ __forceinline__ void pn_pass(pc* buf, const pc* tw, int lane) {
    constexpr PnFac F = pn_factor(N);
    constexpr int R = F.r[I], NS = F.ns[I], OFF = F.off[I];
    constexpr int M = N / R, ITS = (M + 63) / 64;
    constexpr bool FULL = M % 64 == 0;
    // every butterfly computed before the fence (only the writes must wait for
    // every lane's reads): just the outputs stay live across it
    pc x[ITS][R];
#pragma unroll
    for (int it = 0; it < ITS; ++it) {
        const int j = lane + 64 * it;
        if (FULL || it + 1 < ITS || j < M) {
#pragma unroll
            for (int q = 0; q < R; ++q) x[it][q] = buf[j + q * M];
            if constexpr (NS > 1) {
                const int jm = j % NS;
                const pc* t = tw + OFF + jm;
#pragma unroll
                for (int q = 1; q < R; ++q) x[it][q] = pc_tw<INV>(x[it][q], t[(q - 1) * NS]);
            }
            pn_bfly<INV, R>(x[it]);
        }
        if constexpr (ITS * R > 12) __builtin_amdgcn_sched_barrier(0);  // one butterfly's loads live at a time
    }
    wave_lds_fence();
#pragma unroll
    for (int it = 0; it < ITS; ++it) {
        const int j = lane + 64 * it;
        if (FULL || it + 1 < ITS || j < M) {
            const int jb = j / NS, jm = j - jb * NS;
            pc* o = buf + jb * NS * R + jm;
#pragma unroll
            for (int q = 0; q < R; ++q) o[q * NS] = x[it][q];
        }
    }
    wave_lds_fence();
}

template <bool INV, int N, int I = 0>
__device__ __forceinline__ void pn_fft_passes(pc* buf, const pc* tw, int lane) {
    constexpr PnFac F = pn_factor(N);
    if constexpr (I < F.n) {
        pn_pass<INV, N, I>(buf, tw, lane);
        pn_fft_passes<INV, N, I + 1>(buf, tw, lane);
    }
}
// The lane index passes through an opaque move first: every pass's addresses
// depend only on it, and hoisted out of the caller's frame loop they would hold
// ~100 VGPRs for the whole walk; recomputed per transform they cost a few VALU.
template <bool INV, int N>
__device__ __forceinline__ void pn_fft(pc* buf, const pc* tw, int lane) {
    int ln;
    asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
    pn_fft_passes<INV, N>(buf, tw, ln);
}

}  // namespace dev
}  // namespace crlot
