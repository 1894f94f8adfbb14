// host_tables.cpp -- the reference's table builders, restated in the product's
// host code (plan creation time only; never on the per-sample path).
//
//   window:  WindowLUT::createWindow / generate*Window / applyNormalization
//            (dsp/window/WindowLUT.cc:215-388), computed in double, cast to float
//   ring:    OLAAccumulator::calculate_ring_size (OLAAccumulator.cc:249-258)
//   norm:    OLAAccumulator::initialize_normalization (OLAAccumulator.cc:260-288)
//            + dsp::ola::build_norm_linear (norm_builder.cc:8-52)
//
// Bit-exactness against the reference's compiled sources is checked by
// tests/test_host_abi.py (test_window_tables_bit_exact_vs_reference,
// test_norm_tables_bit_exact_vs_reference) on tests/golden/ref_tables.npz.  This file is built
// with -ffp-contract=off: the reference builds these translation units as ISO
// C++17 where GCC 11 keeps each double operation separately rounded.
#include <cmath>
#include <cstdint>
#include <vector>

#include "batch.h"
#include "crlot_dsp.h"

namespace {

void normalize(float* w, int64_t n, int32_t norm) {
    switch (norm) {
        case CRLOT_NORM_SUM_TO_ONE: {
            double s = 0.0;
            for (int64_t i = 0; i < n; ++i) s += static_cast<double>(w[i]);
            if (s > 0.0) {
                const float sc = static_cast<float>(1.0 / s);
                for (int64_t i = 0; i < n; ++i) w[i] *= sc;
            }
            break;
        }
        case CRLOT_NORM_L2:
        case CRLOT_NORM_OLA_UNITY_GAIN:
        case CRLOT_NORM_OLA_SUM_WSQ: {  // hop_size = 0 in createWindow -> L2 branch
            double s = 0.0;
            for (int64_t i = 0; i < n; ++i) {
                const double v = static_cast<double>(w[i]);
                s += v * v;
            }
            if (s > 0.0) {
                const float sc = static_cast<float>(1.0 / std::sqrt(s));
                for (int64_t i = 0; i < n; ++i) w[i] *= sc;
            }
            break;
        }
        default:
            break;
    }
}

}  // namespace

extern "C" int crlot_window_table(int32_t type, int64_t n, int32_t periodic, int32_t norm,
                                  float* out) {
    if (n <= 0 || out == nullptr) return CRLOT_EINVAL;
    if (type < CRLOT_WIN_HANN || type > CRLOT_WIN_RECT) return CRLOT_EINVAL;
    if (norm < CRLOT_NORM_NONE || norm > CRLOT_NORM_OLA_SUM_WSQ) return CRLOT_EINVAL;
    if (type == CRLOT_WIN_RECT) {
        for (int64_t i = 0; i < n; ++i) out[i] = 1.0f;
    } else if (n == 1) {
        out[0] = 1.0f;
    } else {
        const double pi = M_PI;
        const double den = periodic ? static_cast<double>(n) : static_cast<double>(n - 1);
        const double factor = 2.0 * pi / den;
        for (int64_t i = 0; i < n; ++i) {
            const double angle = factor * static_cast<double>(i);
            if (type == CRLOT_WIN_HANN) {
                out[i] = static_cast<float>(0.5 * (1.0 - std::cos(angle)));
            } else if (type == CRLOT_WIN_HAMMING) {
                out[i] = static_cast<float>(0.54 - 0.46 * std::cos(angle));
            } else {
                const double c1 = std::cos(angle), c2 = std::cos(2.0 * angle);
                out[i] = static_cast<float>(0.42 - 0.5 * c1 + 0.08 * c2);
            }
        }
    }
    if (norm != CRLOT_NORM_NONE) normalize(out, n, norm);
    crlot::note_window(out, n);  // a table the batched speculation may meet (batch.h)
    return CRLOT_OK;
}

extern "C" int64_t crlot_ring_len(int64_t frame_size, int64_t hop) {
    if (frame_size <= 0 || hop <= 0) return CRLOT_EINVAL;
    const int64_t min_overlaps = (frame_size + hop - 1) / hop;
    return (min_overlaps + 20) * hop;
}

// norm_builder.cc:8-52 build_norm_linear: frame starts k*H, k in
// [floor(-N/H), ceil((R+N-1)/H)], accumulated in ascending k, each start split
// into <= 2 ring spans.
extern "C" int crlot_build_norm_linear(float* out, const float* window, int64_t ring_len, int64_t n, int64_t h) {
    if (n <= 0 || h <= 0 || ring_len <= 0 || out == nullptr || window == nullptr) return CRLOT_EINVAL;
    for (int64_t i = 0; i < ring_len; ++i) out[i] = 0.0f;
    const int64_t R = ring_len;
    const int64_t a = -n;
    const int64_t k_start = (a - h + 1) / h;
    const int64_t k_end = (R + n - 1 + h - 1) / h;
    for (int64_t k = k_start; k <= k_end; ++k) {
        int64_t s = k * h;
        if (s < 0) {
            s = R + (s % R);
            if (s < 0) s += R;
        }
        const int64_t st = s % R;
        const int64_t first = n < R - st ? n : R - st;
        const int64_t second = n - first;
        for (int64_t i = 0; i < first; ++i) out[st + i] += window[i];
        for (int64_t i = 0; i < second; ++i) out[i] += window[first + i];
    }
    return CRLOT_OK;
}

extern "C" int crlot_norm_table(const float* window, int64_t n, int64_t h, int64_t ring_len,
                                int32_t apply_window_inside, float eps, float* out) {
    if (n <= 0 || h <= 0 || ring_len <= 0 || out == nullptr) return CRLOT_EINVAL;
    if (window == nullptr || !apply_window_inside) {
        for (int64_t i = 0; i < ring_len; ++i) out[i] = 1.0f;
        return CRLOT_OK;
    }
    if (h == n) {
        for (int64_t i = 0; i < ring_len; ++i) {
            const float w = window[i % n];
            out[i] = w > eps ? w : eps;  // std::max(window_[i % N], eps)
        }
        return CRLOT_OK;
    }
    return crlot_build_norm_linear(out, window, ring_len, n, h);
}
