// pair32.hip -- K_pair's paired-only walk (pair1k.hip) on HALF waves: the
// 1024-point pair transform of fft_pair32.h (32 lanes x 32 registers, one LDS
// transpose, no lane-bit swap), two walks per wave (the two halves walk the
// same chunk of streams 2u and 2u+1, so every branch is uniform).
//
// A timing experiment for VERDICT r02 item 3 (in -DCRLOT_PAIR32_EXPERIMENT builds
// CRLOT_PAIR32=1 selects it at N = 1024, H = 256): its FFT rounds differently from the fix-up walker's, so a
// chunk the fix-up walker redoes would not match its neighbours bit for bit --
// the release path keeps K_pair.  Lane hl of half h holds sample hl + 32 q of
// each hop (q < 8), frame sample hl + 32 m (m < 32); everything else is K_pair's
// walk: hops rotating through register slots, OLA blocks in registers, frames
// k, k+1 as one transform, Markstein division with {den, 1/den} pairs, flags for
// the fix-up walker.
#include <cmath>
#include <cstdlib>

#include "fft_pair32.h"
#include "fused_common.h"

namespace crlot {
namespace fk {

namespace {
constexpr int kP32Waves = 8;  // one workgroup per CU, two waves per SIMD
struct P32Lds {
    static constexpr size_t tw = 0;
    static constexpr size_t wa = tw + sizeof(dev::pc) * dev::kP32T;
    static constexpr size_t ws = wa + sizeof(float) * 1024;
    static constexpr size_t bufs = ws + sizeof(float) * 1024;
    static constexpr size_t bytes = bufs + sizeof(dev::pc) * dev::kP32Xbuf * kP32Waves;
};
}  // namespace

__global__ __launch_bounds__(64 * kP32Waves) __attribute__((amdgpu_waves_per_eu(2, 2)))
void k_stft_ola_pair32(const FusedArgs a) {
    constexpr int SH = 8, NB = 4, E = 32, H = 256, R = 8, U = 4;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    dev::pc* tw = reinterpret_cast<dev::pc*>(smem + P32Lds::tw);
    float* wa4 = reinterpret_cast<float*>(smem + P32Lds::wa);  // tap hl + 32 m at (m/4) 128 + 4 hl + m%4
    float* ws4 = reinterpret_cast<float*>(smem + P32Lds::ws);
    for (int i = threadIdx.x; i < dev::kP32T; i += blockDim.x) {
        const int k1 = i < 960 ? ((i >> 6) << 1) + 1 + (i & 1) : 31;
        const int l = i < 960 ? (i & 63) >> 1 : i - 960;
        double s, c;
        sincospi(-2.0 * double(l * k1) / 1024.0, &s, &c);
        tw[i] = dev::pc_mk(float(c), float(s));
    }
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) {
        const int l = i & 31, m = i >> 5;
        const int d = (m >> 2) * 128 + l * 4 + (m & 3);
        wa4[d] = a.t.wa[i];
        ws4[d] = a.t.wsn[i];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, hl = lane & 31, half = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    dev::pc* buf = reinterpret_cast<dev::pc*>(smem + P32Lds::bufs) + wave * dev::kP32Xbuf;
    const int units = (a.n_streams + 1) / 2;
    const int gw = blockIdx.x * kP32Waves + wave;
    if (gw >= units * a.n_chunks) return;
    const int u = gw / a.n_chunks, c = gw - u * a.n_chunks;
    const int s0 = 2 * u;
    const bool both = s0 + 1 < a.n_streams;
    const int f0 = c * a.M;
    const int f1 = min(a.F, f0 + a.M);
    const int fs = max(0, f0 - (NB - 1)) & ~1;
    const __amdgpu_buffer_rsrc_t rx =
        dev::make_rsrc(a.x + int64_t(s0) * a.ld_x, uint32_t((both ? a.ld_x + a.T : a.T) * 4));
    const __amdgpu_buffer_rsrc_t ry =
        dev::make_rsrc(a.y + int64_t(s0) * a.ld_y, uint32_t((both ? a.ld_y + a.out_len : a.out_len) * 4));
    const __amdgpu_buffer_rsrc_t ry_null = dev::make_rsrc(a.y, 0u);
    const float2* const dr2 = reinterpret_cast<const float2*>(a.t.den_rden);
    const __amdgpu_buffer_rsrc_t rden = dev::make_rsrc(dr2, uint32_t(a.ring_blocks * H) * 8u);
    const int xo = half * int(a.ld_x), yo = half * int(a.ld_y);
    const float g = a.gain;
    const uint32_t xlo_b = __builtin_bit_cast(uint32_t, a.t.px_lo), xhi_b = __builtin_bit_cast(uint32_t, a.t.px_hi);

    // hop at `origin`: samples origin + hl + 32 q of the half's stream (0 outside [0, T))
    auto load_hop = [&](float (&d)[SH], int origin) {
        if (origin >= 0 && origin + H <= a.T) {
            const int v = (xo + origin + hl) * 4;
#pragma unroll
            for (int q = 0; q < SH; ++q) d[q] = dev::bload1(rx, v + q * 128, 0);
        } else {
#pragma unroll
            for (int q = 0; q < SH; ++q) {
                const int t = origin + hl + 32 * q;
                d[q] = dev::bload1(rx, (t >= 0 && t < a.T) ? (xo + t) * 4 : 0x7ffffff0, 0);
            }
        }
    };
    bool bad = false;
    auto hop_check = [&](const float (&h)[SH]) {
        uint32_t mx = 0u, mn = ~0u;
#pragma unroll
        for (int q = 0; q < SH; ++q) {
            const uint32_t w = __builtin_bit_cast(uint32_t, h[q]) & 0x7fffffffu;
            mx = max(mx, w);
            mn = min(mn, w - 1u);
        }
        bad |= (mx > xhi_b) | (mn < xlo_b - 1u);
    };
    float xr[R][SH];
#pragma unroll
    for (int h = 0; h <= NB; ++h) {
        load_hop(xr[h], (fs + h) * H - a.pad);
        hop_check(xr[h]);
    }
    float acc[NB][SH];
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int q = 0; q < SH; ++q) acc[j][q] = 0.f;

    auto load_dens = [&](float2 (&d)[SH], int b) {
#pragma unroll
        for (int q = 0; q < SH; ++q) d[q] = dev::bload2(rden, (hl + 32 * q) * 8, b * H * 8);
    };
    auto emit = [&](const float (&av)[SH], int k, const float2 (&d)[SH]) {
        int ex_lo = 0, ex_hi = 0;
#pragma unroll
        for (int q = 0; q < SH; ++q) {
            const int e = __builtin_amdgcn_frexp_expf(av[q]);
            ex_lo = min(ex_lo, e);
            ex_hi = max(ex_hi, e);
        }
        bad |= !((ex_lo >= -63) & (ex_hi <= 65));
        const __amdgpu_buffer_rsrc_t rk = k >= f0 ? ry : ry_null;
#pragma unroll
        for (int q = 0; q < SH; ++q) {
            const float o = mk_div(av[q], d[q].x, d[q].y);
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o), rk, (yo + k * H + hl) * 4,
                                                  q * 128, 0);
        }
    };

    auto step = [&](auto phc, int k) {
        constexpr int PH = decltype(phc)::value;
        constexpr int S0 = (2 * PH) % R, B0 = (2 * PH) % NB;
        load_hop(xr[(S0 + NB + 1) % R], (k + NB + 1) * H - a.pad);
        load_hop(xr[(S0 + NB + 2) % R], (k + NB + 2) * H - a.pad);
        dev::pc v[E];
#pragma unroll
        for (int m4 = 0; m4 < E / 4; ++m4) {
            const float4 w = *reinterpret_cast<const float4*>(wa4 + m4 * 128 + hl * 4);
            const float wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
                const int m = 4 * m4 + q4;
                v[m] = dev::pc_mk(xr[(S0 + m / SH) % R][m % SH] * wv[q4], xr[(S0 + 1 + m / SH) % R][m % SH] * wv[q4]);
            }
        }
        dev::pair32_fft_fwd(v, buf, tw, lane);
        float2 d0[SH], d1[SH];
        load_dens(d0, k % a.ring_blocks);
        load_dens(d1, (k + 1) % a.ring_blocks);
        dev::pair32_fft_inv(v, buf, tw, lane);
        {
            int e[4] = {0, 0, 0, 0};
#pragma unroll
            for (int m = 0; m < E; ++m)
                e[m & 3] = min(e[m & 3], min(__builtin_amdgcn_frexp_expf(v[m].x), __builtin_amdgcn_frexp_expf(v[m].y)));
            bad |= min(min(e[0], e[1]), min(e[2], e[3])) <= -89;
        }
#pragma unroll
        for (int m4 = 0; m4 < E / 4; ++m4) {
            const dev::pc* w2 = reinterpret_cast<const dev::pc*>(ws4 + m4 * 128 + hl * 4);
            const dev::pc wl = w2[0], wh = w2[1];
            v[4 * m4 + 0] = v[4 * m4 + 0] * dev::pc{wl.x, wl.x};
            v[4 * m4 + 1] = v[4 * m4 + 1] * dev::pc{wl.y, wl.y};
            v[4 * m4 + 2] = v[4 * m4 + 2] * dev::pc{wh.x, wh.x};
            v[4 * m4 + 3] = v[4 * m4 + 3] * dev::pc{wh.y, wh.y};
        }
#pragma unroll
        for (int m = 0; m < E; ++m) {
            float& r = acc[(B0 + m / SH) % NB][m % SH];
            r = __builtin_fmaf(v[m].x, g, m / SH == NB - 1 ? 0.0f : r);
        }
        emit(acc[B0], k, d0);
#pragma unroll
        for (int m = 0; m < E; ++m) {
            float& r = acc[(B0 + 1 + m / SH) % NB][m % SH];
            r = __builtin_fmaf(v[m].y, g, m / SH == NB - 1 ? 0.0f : r);
        }
        emit(acc[(B0 + 1) % NB], k + 1 < f1 ? k + 1 : -1, d1);
        hop_check(xr[(S0 + NB + 1) % R]);
        hop_check(xr[(S0 + NB + 2) % R]);
    };
    for (int k = fs; k < f1; k += 2 * U) {
        step(std::integral_constant<int, 0>(), k);
        if (k + 2 >= f1) break;
        step(std::integral_constant<int, 1>(), k + 2);
        if (k + 4 >= f1) break;
        step(std::integral_constant<int, 2>(), k + 4);
        if (k + 6 >= f1) break;
        step(std::integral_constant<int, 3>(), k + 6);
    }
    const uint64_t bal = __builtin_amdgcn_ballot_w64(bad);
    if (hl == 0 && (half == 0 || both)) {
        const uint64_t mine = half ? (bal >> 32) : (bal & 0xffffffffull);
        a.t.pflags[(s0 + half) * a.n_chunks + c] = mine != 0 ? 1u : 0u;
    }
}

// Experiment builds only (-DCRLOT_PAIR32_EXPERIMENT, e.g. `make variant`): then
// CRLOT_PAIR32=1 selects this walker.  The release library always runs K_pair.
bool pair32_enabled() {
#ifdef CRLOT_PAIR32_EXPERIMENT
    static const bool v = [] {
        const char* e = ab_env("CRLOT_PAIR32");
        return e && e[0] == '1';
    }();
    return v;
#else
    return false;
#endif
}

hipError_t launch_pair32(const FusedArgs& a, hipStream_t stream) {
    if (!a.t.den_rden || !a.t.wsn || a.cs != 1 || a.pad_mode != 0 || a.t.gain) return hipErrorInvalidValue;
    const int64_t units = (a.n_streams + 1) / 2;
    const int64_t waves = units * a.n_chunks;
    const size_t lds = P32Lds::bytes;
    hipError_t e = set_lds(k_stft_ola_pair32, lds);
    if (e != hipSuccess) return e;
    note_launch(CRLOT_K_EXPERIMENT, (waves + kP32Waves - 1) / kP32Waves);
    hipLaunchKernelGGL(k_stft_ola_pair32, dim3(unsigned((waves + kP32Waves - 1) / kP32Waves)), dim3(64 * kP32Waves),
                       lds, stream, a);
    return hipGetLastError();
}

}  // namespace fk
}  // namespace crlot
