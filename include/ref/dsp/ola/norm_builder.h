// Drop-in for the reference's dsp/ola/norm_builder.h (norm_builder.h:5-31):
// build_norm_linear, host code, bit-exact with norm_builder.cc
// (crlot_build_norm_linear; pinned against the compiled reference in
// tests/test_host_abi.py).
#pragma once

#include <cstddef>
#include <cstdint>

#include "../../../crlot_dsp.h"

namespace dsp {
namespace ola {
inline void build_norm_linear(float* norm, const float* window, size_t ring_len, size_t frame_size, size_t hop) {
    crlot_build_norm_linear(norm, window, int64_t(ring_len), int64_t(frame_size), int64_t(hop));
}
}  // namespace ola
}  // namespace dsp
