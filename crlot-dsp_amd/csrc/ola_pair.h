// ola_pair.h -- the OLA stage of the frame-pair hot walkers with the blocks of a
// frame pair held as register pairs (K_pair pair1k.hip, K_pair4k / K_pair2k /
// K_pair512 pair_hot.hip).
//
// A pair transform leaves frame k's push_frame_AoS input in v[m].x and frame
// k+1's in v[m].y (m = register, sample lane + L m).  Frame k adds v[m].x to OLA
// block k + m/SH, frame k+1 adds v[m].y to block k + 1 + m/SH; every block's
// adds must run in ascending frame order (fma(fma(o, w, 0), g, acc) per frame,
// OLAAccumulator.cc:124-160 via kernels.cc:24-28).  With blocks 2i and 2i+1 in one
// register pair, acc2[i][q] = (block 2i, block 2i+1) (ring indices modulo NB;
// k is even), the adds of register m with m/SH even are ONE packed fma for both
// frames -- frame k into the even block, frame k+1 into the odd one -- and the
// rest stay scalar, ordered so each block still sees frame k before frame k+1:
//   1. frame k into the odd blocks k+1, k+3, .. (block k+NB-1 opens from zero);
//   2. the packed adds into the block pairs (k+2i, k+2i+1), after 1;
//   3. frame k+1 into the even blocks k+2, k+4, .., after 2;
//   4. produce blocks k and k+1 (both complete after 2): packed divisions;
//   5. frame k+1 opens block k+NB in block k's register (ola_pair_open).
// Lane for lane these are the scalar walk's IEEE operations, so the bits equal
// the two-regime walkers' (tests/test_gpu_parity.py).
#pragma once

#include "fft_pair.h"
#include "fused_common.h"

namespace crlot {
namespace fk {

// steps 1-3 for the pair whose frame k has ring index B0 (even)
template <int E, int SH, int NB, int B0>
__device__ __forceinline__ void ola_pair_push(dev::pc (&acc2)[NB / 2][SH], const dev::pc (&v)[E], float g) {
    static_assert(NB % 2 == 0 && B0 % 2 == 0 && NB * SH == E, "block pairs");
    const dev::pc gg = {g, g};
#pragma unroll
    for (int m = 0; m < E; ++m)
        if ((m / SH) % 2 == 1) {
            const int b = (B0 + m / SH) % NB;
            acc2[b / 2][m % SH][b % 2] = __builtin_fmaf(v[m].x, g, m / SH == NB - 1 ? 0.0f : acc2[b / 2][m % SH][b % 2]);
        }
#pragma unroll
    for (int m = 0; m < E; ++m)
        if ((m / SH) % 2 == 0) {
            dev::pc& r = acc2[((B0 + m / SH) % NB) / 2][m % SH];
            r = __builtin_elementwise_fma(v[m], gg, r);
        }
#pragma unroll
    for (int m = 0; m < E; ++m)
        if ((m / SH) % 2 == 1 && m / SH != NB - 1) {
            const int b = (B0 + 1 + m / SH) % NB;
            acc2[b / 2][m % SH][b % 2] = __builtin_fmaf(v[m].y, g, acc2[b / 2][m % SH][b % 2]);
        }
}

// step 5: frame k+1 opens block k+NB (ring index B0)
template <int E, int SH, int NB, int B0>
__device__ __forceinline__ void ola_pair_open(dev::pc (&acc2)[NB / 2][SH], const dev::pc (&v)[E], float g) {
#pragma unroll
    for (int m = (NB - 1) * SH; m < E; ++m) acc2[B0 / 2][m % SH][0] = __builtin_fmaf(v[m].y, g, 0.0f);
}

// steps 1-3 and 5 with the synthesis window and the OLA gain folded into the
// adds: acc = fma(v, ws[m] g, acc), one rounding where push_frame_AoS has two
// (fma(fma(o, w, 0), g, acc)); the walkers stage ws * g (exactly ws when g = 1)
// and every walker of the kernel uses this form, so their bits still agree
template <int E, int SH, int NB, int B0>
__device__ __forceinline__ void ola_pair_push_w(dev::pc (&acc2)[NB / 2][SH], const dev::pc (&v)[E],
                                                const float (&wg)[E]) {
    static_assert(NB % 2 == 0 && B0 % 2 == 0 && NB * SH == E, "block pairs");
#pragma unroll
    for (int m = 0; m < E; ++m)
        if ((m / SH) % 2 == 1) {
            const int b = (B0 + m / SH) % NB;
            acc2[b / 2][m % SH][b % 2] =
                __builtin_fmaf(v[m].x, wg[m], m / SH == NB - 1 ? 0.0f : acc2[b / 2][m % SH][b % 2]);
        }
#pragma unroll
    for (int m = 0; m < E; ++m)
        if ((m / SH) % 2 == 0) {
            dev::pc& r = acc2[((B0 + m / SH) % NB) / 2][m % SH];
            r = __builtin_elementwise_fma(v[m], dev::pc{wg[m], wg[m]}, r);
        }
#pragma unroll
    for (int m = 0; m < E; ++m)
        if ((m / SH) % 2 == 1 && m / SH != NB - 1) {
            const int b = (B0 + 1 + m / SH) % NB;
            acc2[b / 2][m % SH][b % 2] = __builtin_fmaf(v[m].y, wg[m], acc2[b / 2][m % SH][b % 2]);
        }
}
template <int E, int SH, int NB, int B0>
__device__ __forceinline__ void ola_pair_open_w(dev::pc (&acc2)[NB / 2][SH], const dev::pc (&v)[E],
                                                const float (&wg)[E]) {
#pragma unroll
    for (int m = (NB - 1) * SH; m < E; ++m) acc2[B0 / 2][m % SH][0] = __builtin_fmaf(v[m].y, wg[m], 0.0f);
}

// {den, rden} of blocks k and k+1 as register pairs (DevTables::pden2 rows of L lanes)
template <int L, int SH>
__device__ __forceinline__ void load_den_pair(dev::pc (&d2)[SH], dev::pc (&r2)[SH], __amdgpu_buffer_rsrc_t rp2,
                                              int t, int kb) {
#pragma unroll
    for (int j = 0; j < SH; ++j) {
        const auto w = __builtin_amdgcn_raw_buffer_load_b128(rp2, t * (16 * SH), kb * (16 * L * SH) + 16 * j, 0);
        const unsigned u0 = w[0], u1 = w[1], u2 = w[2], u3 = w[3];  // (see bload2)
        dev::pc& lo = j < SH / 2 ? d2[2 * j] : r2[2 * j - SH];
        dev::pc& hi = j < SH / 2 ? d2[2 * j + 1] : r2[2 * j + 1 - SH];
        lo = dev::pc{__builtin_bit_cast(float, u0), __builtin_bit_cast(float, u1)};
        hi = dev::pc{__builtin_bit_cast(float, u2), __builtin_bit_cast(float, u3)};
    }
}

// step 4: produce(H) of blocks k and k+1 -- Markstein's division (mk_div) on both
// at once -- into o0 / o1; false when a sum lies outside Markstein's exact range
// (0 or |acc| in [2^-64, 2^64]: frexp exponents in [-63, 65], zero's being 0)
template <int SH>
__device__ __forceinline__ bool mk_div_pair(const dev::pc (&a)[SH], const dev::pc (&d2)[SH], const dev::pc (&r2)[SH],
                                            float (&o0)[SH], float (&o1)[SH]) {
    int ex_lo = 0, ex_hi = 0;
#pragma unroll
    for (int i = 0; i < 2 * SH; ++i) {
        const int e = __builtin_amdgcn_frexp_expf(a[i >> 1][i & 1]);
        ex_lo = min(ex_lo, e);
        ex_hi = max(ex_hi, e);
    }
#pragma unroll
    for (int q = 0; q < SH; ++q) {
        const dev::pc qv = a[q] * r2[q];
        const dev::pc y = __builtin_elementwise_fma(__builtin_elementwise_fma(-qv, d2[q], a[q]), r2[q], qv);
        o0[q] = y.x;
        o1[q] = y.y;
    }
    return (ex_lo >= -63) & (ex_hi <= 65);
}

}  // namespace fk
}  // namespace crlot
