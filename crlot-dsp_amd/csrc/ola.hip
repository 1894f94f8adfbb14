// ola.hip -- device arithmetic of the OLAAccumulator object (crlot_ola_*, objects.cpp).
//
// The object keeps the reference's ring per channel in HBM, [C][R] floats
// (R = ring_len), plus den[R] = (norm > eps ? norm : eps).  The host side runs
// the reference's state machine (read_pos_, produced_, flush, reset:
// OLAAccumulator.cc:54-247); these kernels do the per-sample work of one call:
//
//   k_ola_add      add_frame_SoA / push_frame_AoS after clamping
//                  (OLAAccumulator.cc:54-160): ring[c][(start + j) mod R] =
//                  fma(fma(src, w, 0), g, ring) with a window, fma(src, g, ring)
//                  without (kernels.cc:18-28, the scalar forms Highway matches);
//                  source element (c, j) at src[c*cs + j*js], so the same
//                  kernel reads SoA frames (cs = ld, js = 1) and interleaved
//                  AoS frames (cs = 1, js = C: aos_to_soa.cc:7-18 fused away).
//   k_ola_produce  produce (OLAAccumulator.cc:162-221) -> normalize_and_clear
//                  (kernels.cc:30-36): out = ring / den (IEEE division), ring = 0,
//                  and the channel-0 peak meter (:289-295) as a running maximum
//                  of |out| kept in device memory (NaN never raises it, as with
//                  std::max(peak, NaN)).
//
// A call touches each ring position at most once (len <= R), so threads never
// race; calls are ordered by the stream.  One thread per (sample, channel):
// these are tiny HBM/L2-resident launches whose cost is the launch itself.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"

namespace crlot {
namespace {

__global__ void __launch_bounds__(256) k_ola_add(float* __restrict__ ring, int64_t R,
                                                 const float* __restrict__ src, int64_t cs,
                                                 int64_t js, const float* __restrict__ win,
                                                 int64_t start, int64_t len, float gain) {
    const int64_t j = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const int64_t c = blockIdx.y;
    if (j >= len) return;
    int64_t p = start + j;
    if (p >= R) p -= R;  // second span of RingBuffer::split (ring_buffer.cc:44-85)
    float* r = ring + c * R + p;
    const float s = src[c * cs + j * js];
    if (win)
        *r = __builtin_fmaf(__builtin_fmaf(s, win[j], 0.0f), gain, *r);
    else
        *r = __builtin_fmaf(s, gain, *r);
}

__device__ inline float wave_max(float v) {
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

__global__ void __launch_bounds__(256) k_ola_produce(float* __restrict__ ring, int64_t R,
                                                     const float* __restrict__ den,
                                                     float* __restrict__ out, int64_t ldo,
                                                     int64_t rp, int64_t len, int64_t n_total,
                                                     unsigned* __restrict__ peak) {
    const int64_t j = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const int64_t c = blockIdx.y;
    float v = 0.0f;
    bool have = false;
    if (j < len) {
        int64_t p = rp + j;
        if (p >= R) p -= R;
        float* r = ring + c * R + p;
        v = *r / den[p];
        out[c * ldo + j] = v;
        *r = 0.0f;
        have = true;
    } else if (c == 0 && peak && j < n_total) {
        // produce(n) with n > R: split() clamps the work to R samples but the
        // meter still reads n (OLAAccumulator.cc:217 over the caller's buffer)
        v = out[j];
        have = true;
    }
    if (c != 0 || !peak) return;
    float a = (have && !(v != v)) ? fabsf(v) : 0.0f;
    a = wave_max(a);
    if ((threadIdx.x & 63) == 0 && a > 0.0f) atomicMax(peak, __float_as_uint(a));
}

// Interleaved PCM <-> channel planes (crlot_roundtrip_interleaved for plans
// off the direct K_pair path; Framer(N, H, C) frames N*C interleaved samples,
// framer.cc:15-35).  A workgroup moves a tile of TR rows x C channels: the
// tile's TR*C interleaved floats are one contiguous run (coalesced loads or
// stores), each plane's TR floats another; the transpose runs through LDS with
// rows padded to C+1 words, so the column walks are bank-conflict-free.
constexpr int kIlvTileFloats = 8192;  // 32 KB of LDS (+ padding) per workgroup
__host__ __device__ constexpr int ilv_rows(int C) {
    const int r = kIlvTileFloats / C;
    return r >= 1024 ? 1024 : r < 64 ? 64 : r & ~63;
}
__global__ void __launch_bounds__(256) k_deinterleave(const float* __restrict__ x, int64_t ld_x,
                                                      float* __restrict__ planes, int64_t T, int C) {
    extern __shared__ float tile[];
    const int TR = ilv_rows(C);
    const int64_t g = blockIdx.y, r0 = int64_t(blockIdx.x) * TR;
    const int rows = int(T - r0 < TR ? T - r0 : TR);
    const float* src = x + g * ld_x + r0 * C;
    for (int e = threadIdx.x; e < rows * C; e += 256) {
        const int r = e / C;
        tile[e + r] = src[e];  // [r][c] at r * (C + 1) + c
    }
    __syncthreads();
    float* dst = planes + g * C * T + r0;
    for (int c = 0; c < C; ++c)
        for (int r = threadIdx.x; r < rows; r += 256) dst[int64_t(c) * T + r] = tile[r * (C + 1) + c];
}

__global__ void __launch_bounds__(256) k_interleave(const float* __restrict__ planes, int64_t L,
                                                    float* __restrict__ y, int64_t ld_y, int C) {
    extern __shared__ float tile[];
    const int TR = ilv_rows(C);
    const int64_t g = blockIdx.y, r0 = int64_t(blockIdx.x) * TR;
    const int rows = int(L - r0 < TR ? L - r0 : TR);
    const float* src = planes + g * C * L + r0;
    for (int c = 0; c < C; ++c)
        for (int r = threadIdx.x; r < rows; r += 256) tile[r * (C + 1) + c] = src[int64_t(c) * L + r];
    __syncthreads();
    float* dst = y + g * ld_y + r0 * C;
    for (int e = threadIdx.x; e < rows * C; e += 256) {
        const int r = e / C;
        dst[e] = tile[e + r];
    }
}

}  // namespace

hipError_t launch_deinterleave(const float* x, int64_t ld_x, float* planes, int groups, int64_t T, int C,
                               hipStream_t s) {
    if (groups <= 0 || T <= 0) return hipSuccess;
    const int tr = ilv_rows(C);
    const size_t lds = sizeof(float) * size_t(tr) * (C + 1);
    hipLaunchKernelGGL(k_deinterleave, dim3(unsigned((T + tr - 1) / tr), unsigned(groups)), dim3(256), lds, s,
                       x, ld_x, planes, T, C);
    return hipGetLastError();
}

hipError_t launch_interleave(const float* planes, int64_t L, float* y, int64_t ld_y, int groups, int C,
                             hipStream_t s) {
    if (groups <= 0 || L <= 0) return hipSuccess;
    const int tr = ilv_rows(C);
    const size_t lds = sizeof(float) * size_t(tr) * (C + 1);
    hipLaunchKernelGGL(k_interleave, dim3(unsigned((L + tr - 1) / tr), unsigned(groups)), dim3(256), lds, s,
                       planes, L, y, ld_y, C);
    return hipGetLastError();
}

hipError_t launch_ola_add(float* ring, int channels, int64_t R, const float* src, int64_t cs,
                          int64_t js, const float* win, int64_t start, int64_t len, float gain,
                          hipStream_t s) {
    if (len <= 0 || channels <= 0) return hipSuccess;
    const dim3 grid(unsigned((len + 255) / 256), unsigned(channels));
    hipLaunchKernelGGL(k_ola_add, grid, dim3(256), 0, s, ring, R, src, cs, js, win, start, len, gain);
    return hipGetLastError();
}

hipError_t launch_ola_produce(float* ring, int channels, int64_t R, const float* den, float* out,
                              int64_t ldo, int64_t rp, int64_t len, int64_t n_total, unsigned* peak,
                              hipStream_t s) {
    const int64_t span = peak && n_total > len ? n_total : len;
    if (span <= 0 || channels <= 0) return hipSuccess;
    const dim3 grid(unsigned((span + 255) / 256), unsigned(channels));
    hipLaunchKernelGGL(k_ola_produce, grid, dim3(256), 0, s, ring, R, den, out, ldo, rp, len, n_total,
                       peak);
    return hipGetLastError();
}

}  // namespace crlot
