// Drop-in for the reference's dsp/ola/kernels.h (kernels.h:5-97) on MI355X.
//
//   axpy / axpy_windowed / normalize_and_clear (kernels.h:28-53)
//       the reference's noexcept host-pointer calls, computed on the device by the
//       resident call kernel (crlot::dsp::axpy & co, include/crlot_dsp.hpp)
//   *_hwy (kernels.h:59-61)
//       the reference's "optimised implementation" slot: the same device kernels
//       (what the reference's Highway dispatch is to its CPU, the device path is here)
//   *_scalar (kernels.h:67-69)
//       the reference's scalar reference kernels, kept host-side as the baseline
//       they are in kernels_test.cc / kernels_benchmark.cc: fma(src, g, dst),
//       fma(fma(src, win, 0), g, dst), acc / max(norm, eps) -- the operations of
//       kernels.cc:18-36; the device kernels equal them bit for bit
//   get_supported_targets / get_current_target / print_kernel_dispatch_info /
//   get_simd_lanes (kernels.h:79-97)
//       report the device: its ISA ("gfx950") and its wavefront width (64 lanes)
#pragma once

#include <cmath>
#include <cstddef>
#include <cstdio>

#include "../../../crlot_dsp.hpp"

namespace dsp {

constexpr size_t kMaxFrameSize = 16384;  // kernels.h:11

using crlot::dsp::axpy;                 // kernels.h:28
using crlot::dsp::axpy_windowed;        // kernels.h:40
using crlot::dsp::normalize_and_clear;  // kernels.h:53

inline void axpy_hwy(float* dst, const float* src, float g, size_t n) noexcept { crlot::dsp::axpy(dst, src, g, n); }
inline void axpy_windowed_hwy(float* dst, const float* src, const float* win, float g, size_t n) noexcept {
    crlot::dsp::axpy_windowed(dst, src, win, g, n);
}
inline void normalize_and_clear_hwy(float* out, float* acc, const float* norm, float eps, size_t n) noexcept {
    crlot::dsp::normalize_and_clear(out, acc, norm, eps, n);
}

inline void axpy_scalar(float* dst, const float* src, float g, size_t n) noexcept {
    for (size_t i = 0; i < n; ++i) dst[i] = std::fma(src[i], g, dst[i]);
}
inline void axpy_windowed_scalar(float* dst, const float* src, const float* win, float g, size_t n) noexcept {
    for (size_t i = 0; i < n; ++i) dst[i] = std::fma(std::fma(src[i], win[i], 0.0f), g, dst[i]);
}
inline void normalize_and_clear_scalar(float* out, float* acc, const float* norm, float eps, size_t n) noexcept {
    for (size_t i = 0; i < n; ++i) {
        const float d = norm[i] > eps ? norm[i] : eps;
        out[i] = acc[i] / d;
        acc[i] = 0.0f;
    }
}

inline const char* get_supported_targets() noexcept { return crlot_device_target(); }
inline const char* get_current_target() noexcept { return crlot_device_target(); }
inline size_t get_simd_lanes() noexcept { return 64; }  // one wavefront
inline void print_kernel_dispatch_info() noexcept {
    std::printf("dsp kernels: device %s, wave64 (%zu lanes), resident call kernel for host pointers, "
                "batched device forms crlot_axpy / crlot_axpy_windowed / crlot_normalize_and_clear\n",
                get_current_target(), get_simd_lanes());
}

}  // namespace dsp
