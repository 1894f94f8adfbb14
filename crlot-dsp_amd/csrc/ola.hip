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

// dsp::axpy / axpy_windowed / normalize_and_clear (kernels.h:28-53) over a batch
// of rows: row b of dst at dst + b*ld_dst, of src at src + b*ld_src; the window
// and the norm row are shared by every row (the OLA's use).  Per element the
// reference's scalar forms (kernels.cc:18-36), which its Highway versions match:
//   axpy           dst = fma(src, g, dst)
//   axpy_windowed  dst = fma(fma(src, win, 0), g, dst)
//   normalize      out = acc / (norm > eps ? norm : eps)   (IEEE division), acc = 0
// HBM-bound elementwise work (12 B per element, the shared row cache-resident):
// VEC moves 4 elements per thread with 16-byte accesses when every row is
// 16-byte aligned; otherwise one element per thread.
template <bool VEC, bool WIN>
__global__ void __launch_bounds__(256) k_axpy(float* __restrict__ dst, int64_t ld_dst,
                                              const float* __restrict__ src, int64_t ld_src,
                                              const float* __restrict__ win, float g, int64_t n) {
    const int64_t b = blockIdx.y;
    const int64_t i = (int64_t(blockIdx.x) * 256 + threadIdx.x) * (VEC ? 4 : 1);
    if (i >= n) return;
    float* d = dst + b * ld_dst + i;
    const float* s = src + b * ld_src + i;
    if constexpr (VEC) {
        const float4 sv = *reinterpret_cast<const float4*>(s);
        float4 dv = *reinterpret_cast<const float4*>(d);
        float4 wv = make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (WIN) wv = *reinterpret_cast<const float4*>(win + i);
        dv.x = __builtin_fmaf(WIN ? __builtin_fmaf(sv.x, wv.x, 0.0f) : sv.x, g, dv.x);
        dv.y = __builtin_fmaf(WIN ? __builtin_fmaf(sv.y, wv.y, 0.0f) : sv.y, g, dv.y);
        dv.z = __builtin_fmaf(WIN ? __builtin_fmaf(sv.z, wv.z, 0.0f) : sv.z, g, dv.z);
        dv.w = __builtin_fmaf(WIN ? __builtin_fmaf(sv.w, wv.w, 0.0f) : sv.w, g, dv.w);
        *reinterpret_cast<float4*>(d) = dv;
    } else {
        const float x = WIN ? __builtin_fmaf(*s, win[i], 0.0f) : *s;
        *d = __builtin_fmaf(x, g, *d);
    }
}

template <bool VEC>
__global__ void __launch_bounds__(256) k_normalize_and_clear(float* __restrict__ out, int64_t ld_out,
                                                             float* __restrict__ acc, int64_t ld_acc,
                                                             const float* __restrict__ norm, float eps,
                                                             int64_t n) {
    const int64_t b = blockIdx.y;
    const int64_t i = (int64_t(blockIdx.x) * 256 + threadIdx.x) * (VEC ? 4 : 1);
    if (i >= n) return;
    float* o = out + b * ld_out + i;
    float* a = acc + b * ld_acc + i;
    if constexpr (VEC) {
        const float4 av = *reinterpret_cast<const float4*>(a);
        const float4 nv = *reinterpret_cast<const float4*>(norm + i);
        float4 r;
        r.x = av.x / ((nv.x > eps) ? nv.x : eps);
        r.y = av.y / ((nv.y > eps) ? nv.y : eps);
        r.z = av.z / ((nv.z > eps) ? nv.z : eps);
        r.w = av.w / ((nv.w > eps) ? nv.w : eps);
        *reinterpret_cast<float4*>(o) = r;
        *reinterpret_cast<float4*>(a) = make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
        const float nv = norm[i];
        *o = *a / ((nv > eps) ? nv : eps);
        *a = 0.0f;
    }
}

// dsp::FrameQueue (FrameQueue.cc:9-115, Indexing.h:18-70) materialised on the
// device: frame k of stream s is padded positions [k*H, k*H + N) of the stream
// padded by `pad` (N/2 with center, else 0) on both sides; original index
// idx = k*H + j - pad, taken from x where 0 <= idx < T, else from the pad rule
// (CONSTANT 0, REFLECT reflect-101 about the ends, EDGE the end sample; any
// rule gives 0 for an empty stream).  One thread per frame sample.
__device__ __forceinline__ int64_t fq_reflect101(int64_t i, int64_t n) {
    if (n <= 1) return 0;
    while (i < 0 || i >= n) i = i < 0 ? -i - 1 : 2 * n - 2 - i;  // Indexing.h:18-33
    return i;
}
__global__ void __launch_bounds__(256) k_fq_frames(const float* __restrict__ x, int64_t T, int64_t ld_x,
                                                   float* __restrict__ frames, int64_t F, int64_t N, int64_t H,
                                                   int64_t pad, int pad_mode) {
    const int64_t s = blockIdx.y;
    const int64_t e = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (e >= F * N) return;
    const int64_t k = e / N, j = e - k * N;
    const int64_t idx = k * H + j - pad;
    const float* xs = x + s * ld_x;
    float v = 0.0f;
    if (idx >= 0 && idx < T)
        v = xs[idx];
    else if (T > 0 && pad_mode == 1)
        v = xs[fq_reflect101(idx, T)];
    else if (T > 0 && pad_mode == 2)
        v = xs[idx < 0 ? 0 : T - 1];
    frames[s * F * N + e] = v;
}

// Batched drop-in speculation (batch.cpp): the analysis products the e2e loop
// forms on the host, p[k][j] = frame_k[j] * w[j] with frame_k[j] = x[k H + j]
// (zero past T), one plain multiply each -- the same product, so the same bits.
__global__ void __launch_bounds__(256) k_windowed_frames(const float* __restrict__ x, int64_t T,
                                                         const float* __restrict__ w, float* __restrict__ p,
                                                         int64_t F, int64_t N, int64_t H) {
    const int64_t e = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (e >= F * N) return;
    const int64_t k = e / N, j = e - k * N;
    const int64_t idx = k * H + j;
    p[e] = (idx < T ? x[idx] : 0.0f) * w[j];
}

// ... and the spectral step a caller applies between forward and inverse when
// it is a fixed real gain per bin (batch.cpp learns it): out[k][2b + c] =
// spec[k][2b + c] * g[b], one plain multiply (std::complex<float> *= float).
__global__ void __launch_bounds__(256) k_bin_gain(const float* __restrict__ spec, float* __restrict__ out,
                                                  const float* __restrict__ g, int64_t rows, int64_t ld,
                                                  int64_t bins) {
    const int64_t e = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (e >= rows * bins) return;
    const int64_t k = e / bins, b = e - k * bins;
    const float gb = g[b];
    const float2 v = *reinterpret_cast<const float2*>(spec + k * ld + 2 * b);
    float2 o;
    o.x = v.x * gb;
    o.y = v.y * gb;
    *reinterpret_cast<float2*>(out + k * ld + 2 * b) = o;
}

}  // namespace

hipError_t launch_bin_gain(const float* spec, float* out, const float* g, int64_t rows, int64_t ld, int64_t bins,
                           hipStream_t s) {
    if (rows <= 0 || bins <= 0) return hipSuccess;
    if (rows * bins > (int64_t(1) << 40) || (ld & 1)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_bin_gain, dim3(unsigned((rows * bins + 255) / 256)), dim3(256), 0, s, spec, out, g, rows, ld,
                       bins);
    return hipGetLastError();
}

hipError_t launch_windowed_frames(const float* x, int64_t T, const float* w, float* p, int64_t F, int64_t N,
                                  int64_t H, hipStream_t s) {
    if (F <= 0 || N <= 0) return hipSuccess;
    if (F * N > (int64_t(1) << 40)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_windowed_frames, dim3(unsigned((F * N + 255) / 256)), dim3(256), 0, s, x, T, w, p, F, N, H);
    return hipGetLastError();
}

hipError_t launch_axpy(float* dst, int64_t ld_dst, const float* src, int64_t ld_src, const float* win, float g,
                       int64_t n, int64_t batch, hipStream_t s) {
    if (n <= 0 || batch <= 0) return hipSuccess;
    if (batch > 65535) return hipErrorInvalidValue;
    auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; };
    const bool vec = n % 4 == 0 && al16(dst) && al16(src) && (!win || al16(win)) &&
                     (batch == 1 || (ld_dst % 4 == 0 && ld_src % 4 == 0));
    const int64_t per = vec ? 1024 : 256;
    const dim3 grid(unsigned((n + per - 1) / per), unsigned(batch));
    auto k = vec ? (win ? k_axpy<true, true> : k_axpy<true, false>)
                 : (win ? k_axpy<false, true> : k_axpy<false, false>);
    hipLaunchKernelGGL(k, grid, dim3(256), 0, s, dst, ld_dst, src, ld_src, win, g, n);
    return hipGetLastError();
}

hipError_t launch_normalize_and_clear(float* out, int64_t ld_out, float* acc, int64_t ld_acc, const float* norm,
                                      float eps, int64_t n, int64_t batch, hipStream_t s) {
    if (n <= 0 || batch <= 0) return hipSuccess;
    if (batch > 65535) return hipErrorInvalidValue;
    auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; };
    const bool vec = n % 4 == 0 && al16(out) && al16(acc) && al16(norm) &&
                     (batch == 1 || (ld_out % 4 == 0 && ld_acc % 4 == 0));
    const int64_t per = vec ? 1024 : 256;
    const dim3 grid(unsigned((n + per - 1) / per), unsigned(batch));
    auto k = vec ? k_normalize_and_clear<true> : k_normalize_and_clear<false>;
    hipLaunchKernelGGL(k, grid, dim3(256), 0, s, out, ld_out, acc, ld_acc, norm, eps, n);
    return hipGetLastError();
}

hipError_t launch_fq_frames(const float* x, int64_t T, int64_t ld_x, int n_streams, float* frames, int64_t F,
                            int64_t N, int64_t H, int64_t pad, int pad_mode, hipStream_t s) {
    if (F <= 0 || n_streams <= 0) return hipSuccess;
    if (n_streams > 65535 || F * N > (int64_t(1) << 40)) return hipErrorInvalidValue;
    const dim3 grid(unsigned((F * N + 255) / 256), unsigned(n_streams));
    hipLaunchKernelGGL(k_fq_frames, grid, dim3(256), 0, s, x, T, ld_x, frames, F, N, H, pad, pad_mode);
    return hipGetLastError();
}

hipError_t launch_deinterleave(const float* x, int64_t ld_x, float* planes, int groups, int64_t T, int C,
                               hipStream_t s) {
    if (groups <= 0 || T <= 0) return hipSuccess;
    const int tr = ilv_rows(C);
    const size_t lds = sizeof(float) * size_t(tr) * (C + 1);
    note_launch(CRLOT_K_DEINTERLEAVE, (T + tr - 1) / tr * groups);
    hipLaunchKernelGGL(k_deinterleave, dim3(unsigned((T + tr - 1) / tr), unsigned(groups)), dim3(256), lds, s,
                       x, ld_x, planes, T, C);
    return hipGetLastError();
}

hipError_t launch_interleave(const float* planes, int64_t L, float* y, int64_t ld_y, int groups, int C,
                             hipStream_t s) {
    if (groups <= 0 || L <= 0) return hipSuccess;
    const int tr = ilv_rows(C);
    const size_t lds = sizeof(float) * size_t(tr) * (C + 1);
    note_launch(CRLOT_K_INTERLEAVE, (L + tr - 1) / tr * groups);
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
