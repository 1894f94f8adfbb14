// kernels_bench: counterparts of the reference's bench/micro_kernels_benchmark.cc
// (AxpyKernel / AxpyWindowedKernel / NormalizeAndClearKernel at 1024 elements,
// OLAAccumulatePush / OLAAccumulatePull on the OLA object, :80-175) and
// bench/kernels_benchmark.cc (axpy / axpy_windowed / normalize_and_clear at
// 16..32768 elements, :13-281), against the drop-in API of include/crlot_dsp.hpp:
//   per_call   the reference's host-pointer signatures (crlot::dsp::axpy & co:
//              the resident call kernel), p50 us per call, per size
//   ola        OLAAccumulator::add_frame_SoA alone and produce(H) + refill add
//              (the fixture's pull loop), p50 us per call
//   batched    the GPU-native forms (crlot_axpy / _windowed / normalize_and_clear
//              over `rows` rows of n), HIP-event time, GB/s of algorithmic traffic
//              (axpy: 12 B per element, normalize_and_clear: 12 B, the shared
//              window / norm row cache-resident) against the 8 TB/s HBM peak
// Usage: kernels_bench [calls=2000]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "../include/crlot_dsp.hpp"

using clk = std::chrono::steady_clock;

static double p50(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[v.size() / 2];
}

template <typename F>
static double per_call_us(F f, int calls) {
    for (int i = 0; i < 20; ++i) f();
    std::vector<double> t;
    t.reserve(size_t(calls));
    for (int i = 0; i < calls; ++i) {
        const auto t0 = clk::now();
        f();
        t.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
    }
    return p50(t);
}

template <typename F>
static double event_ms(F f, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    f();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a, nullptr);
    for (int i = 0; i < reps; ++i) f();
    (void)hipEventRecord(b, nullptr);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return double(ms) / reps;
}

int main(int argc, char** argv) {
    const int calls = argc > 1 ? std::atoi(argv[1]) : 2000;
    namespace D = crlot::dsp;
    std::mt19937 gen(12345);  // kernels_benchmark.cc:57
    std::uniform_real_distribution<float> U(-1.0f, 1.0f);
    std::string js = "{\"harness\": \"kernels_bench\", \"reference\": [\"bench/micro_kernels_benchmark.cc\", "
                     "\"bench/kernels_benchmark.cc\"], \"per_call_us_p50\": [";
    try {
        const int sizes[] = {16, 32, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768};
        bool first = true;
        for (int n : sizes) {
            const size_t un = size_t(n);
            std::vector<float> dst(un), src(un), win(un), norm(un), out(un);
            for (int i = 0; i < n; ++i) {
                dst[size_t(i)] = U(gen);
                src[size_t(i)] = U(gen);
                win[size_t(i)] = 0.5f + 0.5f * U(gen);
                norm[size_t(i)] = 1.0f + U(gen);
            }
            const double a = per_call_us([&] { D::axpy(dst.data(), src.data(), 0.5f, size_t(n)); }, calls);
            const double w =
                per_call_us([&] { D::axpy_windowed(dst.data(), src.data(), win.data(), 0.5f, size_t(n)); }, calls);
            const double z =
                per_call_us([&] { D::normalize_and_clear(out.data(), dst.data(), norm.data(), 1e-8f, size_t(n)); },
                            calls);
            char buf[256];
            std::snprintf(buf, sizeof buf, "%s{\"n\": %d, \"axpy\": %.3f, \"axpy_windowed\": %.3f, "
                          "\"normalize_and_clear\": %.3f}", first ? "" : ", ", n, a, w, z);
            js += buf;
            first = false;
        }
        js += "], ";

        // the OLA object as micro_kernels_benchmark.cc:80-120 drives it (N 1024, H 256, window inside)
        const size_t N = 1024, H = 256;
        auto wl = D::WindowLUT::getInstance().GetWindowSafe(D::WindowType::HANN, N);
        D::OLAConfig c;
        c.sample_rate = 48000;
        c.frame_size = N;
        c.hop_size = H;
        c.channels = 1;
        c.eps = 1e-8f;
        c.apply_window_inside = true;
        D::OLAAccumulator ola(c);
        ola.set_window(wl.get(), int(N));
        std::vector<float> fr(N);
        for (auto& v : fr) v = U(gen);
        const float* ch[1] = {fr.data()};
        size_t k = 0;
        const double push = per_call_us([&] { ola.add_frame_SoA(ch, wl.get(), (k++ % 10) * H, 0, N, 1.0f); },
                                        calls);
        D::OLAAccumulator ola2(c);
        ola2.set_window(wl.get(), int(N));
        for (size_t i = 0; i < 10; ++i) ola2.add_frame_SoA(ch, wl.get(), i * H, 0, N, 1.0f);
        std::vector<float> hop(H);
        float* out[1] = {hop.data()};
        size_t fc = 10;
        const double pull = per_call_us(
            [&] {
                ola2.produce(out, H);
                ola2.add_frame_SoA(ch, wl.get(), fc++ * H, 0, N, 1.0f);
            },
            calls);
        char buf[256];
        std::snprintf(buf, sizeof buf, "\"ola_us_p50\": {\"OLAAccumulatePush\": %.3f, \"OLAAccumulatePull\": %.3f}, ",
                      push, pull);
        js += buf;

        // batched device forms: 65535 rows of 1024 (and 4096 rows of 16384)
        js += "\"batched\": [";
        first = true;
        for (auto shape : {std::pair<size_t, size_t>{65535, 1024}, std::pair<size_t, size_t>{4096, 16384}}) {
            const size_t rows = shape.first, n = shape.second, el = rows * n;
            float *dd, *ds, *dw;
            if (hipMalloc(&dd, el * 4) || hipMalloc(&ds, el * 4) || hipMalloc(&dw, n * 4)) return 5;
            (void)hipMemset(dd, 0, el * 4);
            (void)hipMemset(ds, 0, el * 4);
            (void)hipMemset(dw, 0, n * 4);
            const double ma = event_ms([&] { D::axpy_device(dd, ds, 0.5f, n, rows); }, 20);
            const double mw = event_ms([&] { D::axpy_windowed_device(dd, ds, dw, 0.5f, n, rows); }, 20);
            const double mz = event_ms([&] { D::normalize_and_clear_device(dd, ds, dw, 1e-8f, n, rows); }, 20);
            const double gb = double(el) * 12.0 / 1e9;
            std::snprintf(buf, sizeof buf,
                          "%s{\"rows\": %zu, \"n\": %zu, \"axpy_ms\": %.4f, \"axpy_gbs\": %.1f, \"axpy_windowed_ms\": "
                          "%.4f, \"axpy_windowed_gbs\": %.1f, \"normalize_ms\": %.4f, \"normalize_gbs\": %.1f}",
                          first ? "" : ", ", rows, n, ma, gb / (ma * 1e-3), mw, gb / (mw * 1e-3), mz,
                          gb / (mz * 1e-3));
            js += buf;
            first = false;
            (void)hipFree(dd);
            (void)hipFree(ds);
            (void)hipFree(dw);
        }
        js += "], \"bytes_per_element\": 12, \"hbm_peak_gbs\": 8000}";
    } catch (const std::exception& e) {
        std::fprintf(stderr, "exception: %s\n", e.what());
        return 4;
    }
    std::printf("%s\n", js.c_str());
    return 0;
}
