// fft_pair32.h -- 1024-point complex FFT of one HALF wave (32 lanes x 32
// registers), for the frame-pair round trip (fft_pair.h explains the pairing).
//
// Index bits (n = 10 bits): lane l = lane & 31 of half h = lane >> 5 holds
// z[l + 32 m], m = 0..31 in registers.  n = l + 32 m, k = k1 + 32 k2:
//   X[k1 + 32 k2] = sum_l W32^{l k2} W1024^{l k1} sum_m W32^{m k1} z[l + 32 m]
// A 32-point DFT over the registers, the twiddle W1024^{l k1}, ONE 32 x 32
// transpose through LDS inside each half, a 32-point DFT over the registers:
// five index bits move per exchange, so there is no lane-bit swap (fft_pair.h
// moves four bits through LDS and two through v_permlane16/32_swap).  The
// spectrum stays at lane k1, register k2 (pair32_bin); the inverse runs the
// steps backwards with conjugate twiddles and leaves y[l + 32 m] natural.
#pragma once

#include "fft_pair.h"

namespace crlot {
namespace dev {

__host__ __device__ constexpr int pair32_bin(int lane, int r) { return (lane & 31) + 32 * r; }

// In-place 32-point DFT, natural order in and out: two 16-point DFTs over the
// even and odd inputs, W32^k on the odd outputs, a radix-2 step.
template <bool INV>
__device__ __forceinline__ void pdft32(pc (&x)[32]) {
    pc e[16], o[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        e[i] = x[2 * i];
        o[i] = x[2 * i + 1];
    }
    pdft16<INV>(e);
    pdft16<INV>(o);
    // W32^k = (cos 2pi k/32, -sin 2pi k/32); k = 4, 12 are W8-type (rot16 J = 2, 6),
    // k = 8 is -i (folded into the butterfly)
    constexpr float C[8] = {1.0f, 0.98078528040323044913f, 0.92387953251128675613f, 0.83146961230254523708f,
                            0.70710678118654752440f, 0.55557023301960222474f, 0.38268343236508977173f,
                            0.19509032201612826785f};
    auto w32 = [&](int k) -> pc {  // k in 1..15, k != 4, 8, 12
        const float c = k < 8 ? C[k] : -C[16 - k];
        const float s = k < 8 ? C[8 - k] : C[k - 8];
        return (pc){c, -s};
    };
    {
        constexpr int idx[12] = {1, 2, 3, 5, 6, 7, 9, 10, 11, 13, 14, 15};
        pc_tw_run<INV>(o, idx, [&](int i) { return w32(idx[i]); });
    }
    o[4] = rot16<INV, 2>(o[4]);
    o[12] = rot16<INV, 6>(o[12]);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        if (k == 8) {
            x[8] = pc_add_mi<INV>(e[8], o[8]);
            x[24] = pc_sub_mi<INV>(e[8], o[8]);
        } else {
            x[k] = e[k] + o[k];
            x[k + 16] = e[k] - o[k];
        }
    }
}

// 32 x 32 transpose inside each half wave through LDS: lane (l + 32 h), register
// r  ->  lane (r + 32 h), register l.  Row stride 34 complex: ds_write_b64 rows
// are 32 consecutive elements, and the ds_read_b128 of 16 consecutive lanes
// start on dword banks 4 x (mod 64) -- conflict free.
constexpr int kP32Row = 34;
constexpr int kP32Half = 32 * kP32Row;
constexpr int kP32Xbuf = 2 * kP32Half;  // complex elements per wave
__device__ __forceinline__ void transpose32(pc (&v)[32], pc* buf, int lane) {
    const int h = lane >> 5, l = lane & 31;
    pc* wb = buf + h * kP32Half + l;
    const float4* rb = reinterpret_cast<const float4*>(buf + h * kP32Half + kP32Row * l);
#pragma unroll
    for (int r = 0; r < 32; ++r) wb[kP32Row * r] = v[r];
    wave_lds_fence();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const float4 t = rb[r];
        v[2 * r] = pc_mk(t.x, t.y);
        v[2 * r + 1] = pc_mk(t.z, t.w);
    }
    wave_lds_fence();
}

// Twiddles W1024^{l k1}, k1 = 1..31, laid out for ds_read_b128: k1 = 2j+1+e at
// t[j * 64 + 2 l + e] (j < 15), k1 = 31 at t[960 + l].
constexpr int kP32T = 31 * 32;
__host__ __device__ constexpr int pair32_t_index(int k1, int l) {
    return k1 == 31 ? 960 + l : ((k1 - 1) >> 1) * 64 + 2 * l + ((k1 - 1) & 1);
}
// (in groups of 8 twiddles: all 31 loaded at once would hold 62 VGPRs beside
// the walk's 160 of data, hops and OLA blocks)
template <bool INV>
__device__ __forceinline__ void pair32_tw_apply(pc (&v)[32], const pc* t, int lane) {
    const float4* t4 = reinterpret_cast<const float4*>(t + 2 * (lane & 31));
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        pc w[8];
        const int jn = g < 3 ? 4 : 3;  // b128 pairs in this group (15 in all)
#pragma unroll
        for (int j = 0; j < jn; ++j) {
            const float4 q = t4[(4 * g + j) * 32];
            w[2 * j] = pc_mk(q.x, q.y);
            w[2 * j + 1] = pc_mk(q.z, q.w);
        }
        if (g == 3) w[6] = t[960 + (lane & 31)];
        const int cnt = g < 3 ? 8 : 7;
#pragma unroll
        for (int i = 0; i < cnt; ++i) v[1 + 8 * g + i] = pc_tw<INV>(v[1 + 8 * g + i], w[i]);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Forward: natural z[l + 32 m] -> X at (lane k1, register k2) = bin k1 + 32 k2.
__device__ __forceinline__ void pair32_fft_fwd(pc (&v)[32], pc* buf, const pc* t, int lane) {
    pdft32<false>(v);
    pair32_tw_apply<false>(v, t, lane);
    transpose32(v, buf, lane);
    pdft32<false>(v);
}

// Inverse (unnormalised): X at (lane k1, register k2) -> natural y[l + 32 m].
__device__ __forceinline__ void pair32_fft_inv(pc (&v)[32], pc* buf, const pc* t, int lane) {
    pdft32<true>(v);
    transpose32(v, buf, lane);
    pair32_tw_apply<true>(v, t, lane);
    pdft32<true>(v);
}

}  // namespace dev
}  // namespace crlot
