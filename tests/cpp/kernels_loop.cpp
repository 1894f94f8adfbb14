// kernels_loop: bench/kernels_benchmark.cc's scalar-vs-"Highway"-vs-default
// pattern (:83-225) and kernels_test.cc's 1-ULP comparison (:214-429), written
// against the reference's own header: #include "dsp/ola/kernels.h" resolves to
// include/ref/dsp/ola/kernels.h (-I include/ref), where *_hwy and the default
// entry points run on the device and *_scalar stay the host baseline.
// Prints one line per (kernel, size) with the ULP distance of the device result
// from the scalar result and the per-call times; exits 1 on any distance > 1 ULP.
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "dsp/ola/kernels.h"

using namespace dsp;

static uint32_t ulp(float a, float b) {
    int32_t ia, ib;
    std::memcpy(&ia, &a, 4);
    std::memcpy(&ib, &b, 4);
    if (ia < 0) ia = int32_t(0x80000000u - uint32_t(ia));
    if (ib < 0) ib = int32_t(0x80000000u - uint32_t(ib));
    const int64_t d = int64_t(ia) - int64_t(ib);
    return uint32_t(d < 0 ? -d : d);
}

template <typename F>
static double us_per_call(F&& f, int reps) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; ++r) f();
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / reps;
}

int main() {
    std::printf("target %s, %zu lanes, kMaxFrameSize %zu\n", get_current_target(), get_simd_lanes(), kMaxFrameSize);
    print_kernel_dispatch_info();
    std::mt19937 rng(42);  // kernels_test.cc:219
    std::uniform_real_distribution<float> u(-10.0f, 10.0f);
    int bad = 0;
    for (size_t n : {size_t(1), size_t(7), size_t(64), size_t(1000), size_t(4096), size_t(32768)}) {
        std::vector<float> src(n), win(n), dst0(n), norm(n);
        for (size_t i = 0; i < n; ++i) {
            src[i] = u(rng), win[i] = std::fabs(u(rng)) * 0.1f, dst0[i] = u(rng);
            norm[i] = i % 5 ? std::fabs(u(rng)) : 1e-12f;
        }
        const float g = 0.75f, eps = 1e-8f;
        std::vector<float> a = dst0, b = dst0, c = dst0;
        axpy_scalar(a.data(), src.data(), g, n);
        axpy_hwy(b.data(), src.data(), g, n);
        axpy(c.data(), src.data(), g, n);
        uint32_t m = 0;
        for (size_t i = 0; i < n; ++i) m = std::max(m, std::max(ulp(a[i], b[i]), ulp(a[i], c[i])));
        bad += m > 1;
        std::vector<float> w1 = dst0, w2 = dst0;
        axpy_windowed_scalar(w1.data(), src.data(), win.data(), g, n);
        axpy_windowed_hwy(w2.data(), src.data(), win.data(), g, n);
        uint32_t mw = 0;
        for (size_t i = 0; i < n; ++i) mw = std::max(mw, ulp(w1[i], w2[i]));
        bad += mw > 1;
        std::vector<float> acc1 = dst0, acc2 = dst0, o1(n), o2(n);
        normalize_and_clear_scalar(o1.data(), acc1.data(), norm.data(), eps, n);
        normalize_and_clear_hwy(o2.data(), acc2.data(), norm.data(), eps, n);
        uint32_t mn = 0;
        for (size_t i = 0; i < n; ++i) mn = std::max(mn, std::max(ulp(o1[i], o2[i]), ulp(acc1[i], acc2[i])));
        bad += mn > 1;
        std::vector<float> d = dst0;
        const double ts = us_per_call([&] { axpy_scalar(d.data(), src.data(), g, n); }, 200);
        const double th = us_per_call([&] { axpy_hwy(d.data(), src.data(), g, n); }, 200);
        std::printf("n %6zu  ulp axpy %u windowed %u normalize %u  axpy scalar %.2f us, device %.2f us\n", n, m, mw,
                    mn, ts, th);
    }
    std::printf("%s\n", bad ? "FAIL" : "OK");
    return bad ? 1 : 0;
}
