// C++ drop-in surface test (runs on the GPU box): the reference's own
// known-answer checks from tests/fft_test.cc and the e2e round trip, written
// against crlot::dsp::* exactly as the reference tests use dsp::*.
// Links the product (libcrlot_dsp.so) and, as the checker only, the oracle.
#include <cmath>
#include <complex>
#include <cstdio>
#include <vector>

#include "../../include/crlot_dsp.hpp"
#include "../../oracle/crlot_oracle.h"

using namespace crlot::dsp;
using namespace crlot::dsp::fft;

#ifndef CRLOT_GOLDEN_DIR
#define CRLOT_GOLDEN_DIR "tests/golden"  // run from the repository root
#endif

static int failures = 0;
#define EXPECT(cond, ...)                                             \
    do {                                                              \
        if (!(cond)) {                                                \
            ++failures;                                               \
            std::printf("FAIL %s:%d: %s ", __FILE__, __LINE__, #cond); \
            std::printf(__VA_ARGS__);                                 \
            std::printf("\n");                                        \
        }                                                             \
    } while (0)

static FftPlanDesc real_desc(int n, int batch = 1, int si = 1, int so = 1) {
    return FftPlanDesc{FftDomain::Real, n, false, batch, si, so};
}

int main() {
    // fft_test.cc:131-155 DC
    {
        auto plan = MakeFftPlan(real_desc(512));
        std::vector<float> x(512, 1.0f);
        std::vector<std::complex<float>> X(257);
        plan->forward(x.data(), X.data());
        EXPECT(std::fabs(std::abs(X[0]) - 512.0f) < 1e-3f, "DC %g", std::abs(X[0]));
        for (int i = 1; i < 257; ++i) EXPECT(std::abs(X[i]) < 1e-3f, "bin %d %g", i, std::abs(X[i]));
    }
    // fft_test.cc:157-197 cos at bin 10, round trip
    for (int n : {512, 1024, 2048}) {
        auto plan = MakeFftPlan(real_desc(n));
        std::vector<float> x(n), y(n);
        for (int i = 0; i < n; ++i) x[i] = 2.0f * std::cos(2.0f * float(M_PI) * 10.0f * (float(i) / n));
        std::vector<std::complex<float>> X(n / 2 + 1);
        plan->forward(x.data(), X.data());
        EXPECT(std::fabs(std::abs(X[10]) - float(n)) < 1e-3f * n / 512, "n=%d |X10|=%g", n, std::abs(X[10]));
        EXPECT(std::fabs(std::arg(X[10])) < 1e-3f, "phase");
        plan->inverse(X.data(), y.data());
        double e = 0;
        for (int i = 0; i < n; ++i) e += double(x[i] - y[i]) * (x[i] - y[i]);
        EXPECT(std::sqrt(e / n) < 1e-5, "n=%d rms %g", n, std::sqrt(e / n));
    }
    // fft_test.cc:199-221 NaN / denormal / Inf
    {
        auto plan = MakeFftPlan(real_desc(512));
        std::vector<float> x(512, 0.0f), y(512);
        x[0] = NAN;
        x[1] = 1e-40f;
        x[2] = INFINITY;
        std::vector<std::complex<float>> X(257);
        plan->forward(x.data(), X.data());
        plan->inverse(X.data(), y.data());
        for (float v : y) EXPECT(std::isfinite(v), "non-finite");
    }
    // fft_test.cc:223-248 invalid configuration
    {
        bool threw = false;
        try {
            MakeFftPlan(real_desc(513));
        } catch (const std::runtime_error&) {
            threw = true;
        }
        EXPECT(threw, "odd N must throw");
    }
    // fft_test.cc:450-495 stride layout
    {
        const int n = 256, B = 3, st = 2;  // reference uses 128; device path starts at 256
        auto plan = MakeFftPlan(real_desc(n, B, st, st));
        std::vector<float> in(B * n * st, 0.0f), rec(B * n * st, 0.0f);
        for (int b = 0; b < B; ++b)
            for (int i = 0; i < n; ++i) in[b * n * st + i * st] = std::sin(2.0f * float(M_PI) * (b + 1) * i / n);
        std::vector<std::complex<float>> out(B * (n / 2 + 1) * st);
        plan->forward(in.data(), out.data(), B);
        plan->inverse(out.data(), rec.data(), B);
        for (int b = 0; b < B; ++b)
            for (int i = 0; i < n; ++i)
                EXPECT(std::fabs(in[b * n * st + i * st] - rec[b * n * st + i * st]) < 1e-4f, "stride b=%d i=%d", b, i);
    }
    // fft_test.cc:227-247 batch ceiling: 2 is fine, 17 throws
    {
        bool ok2 = true, threw17 = false;
        try {
            MakeFftPlan(real_desc(512, 2));
        } catch (...) {
            ok2 = false;
        }
        try {
            MakeFftPlan(real_desc(512, 17));
        } catch (const std::runtime_error&) {
            threw17 = true;
        }
        EXPECT(ok2 && threw17, "batch 2 ok, 17 throws");
    }
    // fft_test.cc:251-288 complex tone round trip, and the complex DFT vs the oracle's kiss_fft
    for (int n : {256, 128, 2048}) {
        auto plan = MakeFftPlan(FftPlanDesc{FftDomain::Complex, n, false, 1, 1, 1});
        EXPECT(plan->domain() == FftDomain::Complex && plan->size() == n, "complex plan info");
        std::vector<std::complex<float>> in(n), X(n), back(n);
        for (int i = 0; i < n; ++i) {
            const float t = float(i) / float(n);
            in[i] = {std::cos(2.0f * float(M_PI) * 10.0f * t), std::sin(2.0f * float(M_PI) * 10.0f * t)};
        }
        plan->forward_complex(in.data(), X.data());
        plan->inverse_complex(X.data(), back.data());
        float max_error = 0.0f;
        for (int i = 0; i < n; ++i)
            max_error = std::fmax(max_error, std::fmax(std::fabs(back[i].real() - in[i].real()),
                                                       std::fabs(back[i].imag() - in[i].imag())));
        EXPECT(max_error < 1e-5f, "complex n=%d round trip %g", n, max_error);
        EXPECT(std::fabs(std::abs(X[10]) - float(n)) < 1e-3f * n, "complex n=%d |X10|=%g", n, std::abs(X[10]));
        or_kfft_cfg* cfg = or_kfft_alloc(n, 0);
        std::vector<std::complex<float>> ref(in);
        or_kfft(cfg, reinterpret_cast<float*>(ref.data()), reinterpret_cast<float*>(ref.data()));
        or_kfft_free(cfg);
        double num = 0, den = 0;
        for (int i = 0; i < n; ++i) {
            num += std::norm(std::complex<double>(X[i]) - std::complex<double>(ref[i]));
            den += std::norm(std::complex<double>(ref[i]));
        }
        EXPECT(std::sqrt(num / den) < 1e-6, "complex n=%d vs kiss rel %g", n, std::sqrt(num / den));
    }
    // domain mismatch: the reference's runtime_error both ways
    {
        auto rp = MakeFftPlan(real_desc(512));
        auto cp = MakeFftPlan(FftPlanDesc{FftDomain::Complex, 256, false, 1, 1, 1});
        std::vector<std::complex<float>> z(512);
        std::vector<float> r(512);
        int threw = 0;
        try {
            rp->forward_complex(z.data(), z.data());
        } catch (const std::runtime_error&) {
            ++threw;
        }
        try {
            cp->forward(r.data(), z.data());
        } catch (const std::runtime_error&) {
            ++threw;
        }
        EXPECT(threw == 2, "domain mismatch must throw runtime_error");
    }
    // WindowLUT: the reference default (symmetric Hann) equals the oracle bit for bit
    {
        WindowLUT lut(1024, WindowType::HANN);
        std::vector<float> ref(1024);
        or_window(OR_HANN, 1024, 0, OR_NORM_NONE, ref.data());
        for (int i = 0; i < 1024; ++i) EXPECT(lut.data()[i] == ref[i], "window %d", i);
    }
    // WindowLUT cache (window_lut_test.cc): GetWindowSafe hits within a generation,
    // handles outlive clearCache(), the deprecated GetWindow stays bit-identical
    {
        WindowLUT& lut = WindowLUT::getInstance();
        EXPECT(&lut == &WindowLUT::getInstance(), "singleton");
        lut.clearCache(true);
        auto a = lut.GetWindowSafe(WindowType::HANN, 1024);
        auto b = lut.GetWindowSafe(WindowType::HANN, 1024);
        EXPECT(a.get() == b.get() && lut.getCacheSize() == 1, "cache hit");
        auto p = lut.GetWindowSafe(WindowType::HANN, 1024, true);
        EXPECT(p.get() != a.get() && lut.getCacheSize() == 2, "periodic is its own key");
        const uint64_t g0 = lut.getCurrentGeneration();
        lut.clearCache();
        EXPECT(lut.getCurrentGeneration() == g0 + 1, "generation");
        auto c = lut.GetWindowSafe(WindowType::HANN, 1024);
        EXPECT(c.get() != a.get() && a.get()[512] == c.get()[512], "old handle survives, new table equal");
        std::vector<float> ref(1024);
        or_window(OR_HANN, 1024, 0, OR_NORM_NONE, ref.data());
        for (int i = 0; i < 1024; ++i) EXPECT(c.get()[i] == ref[i], "cached window %d", i);
#pragma GCC diagnostic push
#pragma GCC diagnostic ignored "-Wdeprecated-declarations"
        const float* raw = lut.GetWindow(WindowType::HAMMING, 512);
        EXPECT(raw == lut.GetWindow(WindowType::HAMMING, 512), "legacy cache hit");
#pragma GCC diagnostic pop
        WindowLUT inst(512, WindowType::HAMMING);
        for (int i = 0; i < 512; ++i) EXPECT(raw[i] == inst.data()[i], "legacy %d", i);
        EXPECT(inst.size() == 512 && inst.type() == WindowType::HAMMING && !inst.periodic(), "getters");
        int threw = 0;
        try { lut.GetWindowSafe(WindowType::HANN, 0); } catch (const std::invalid_argument&) { ++threw; }
        try { WindowLUT bad(0, WindowType::HANN); } catch (const std::invalid_argument&) { ++threw; }
        try { WindowLUT bh(64, WindowType::BLACKMAN_HARRIS); } catch (const std::invalid_argument&) { ++threw; }
        try { WindowLUT empty; (void)empty.data(); } catch (const std::runtime_error&) { ++threw; }
        EXPECT(threw == 4, "WindowLUT exceptions %d", threw);
        EXPECT(std::fabs(WindowLUT::calculateSum(inst.data(), 512) - 0.54 * 511 - 0.54) < 1.0, "sum");
    }
    // Framer / OLAAccumulator exception types (framer.cc:15-35, OLAAccumulator.cc:17-19, 38-45)
    {
        int threw = 0;
        Framer f;
        try { f.set_params(0, 1); } catch (const std::invalid_argument&) { ++threw; }
        EXPECT(!f.pop(nullptr) && !f.push(nullptr, 4), "framer guards");
        OLAConfig bad;
        bad.sample_rate = 48000;
        bad.frame_size = 256;
        bad.hop_size = 64;
        bad.channels = 0;
        try { OLAAccumulator o(bad); } catch (const std::invalid_argument&) { ++threw; }
        OLAConfig ok = bad;
        ok.channels = 2;
        ok.apply_window_inside = true;
        OLAAccumulator o(ok);
        try { o.set_window(nullptr, 256); } catch (const std::invalid_argument&) { ++threw; }
        std::vector<float> w(256, 1.0f);
        try { o.set_window(w.data(), 255); } catch (const std::invalid_argument&) { ++threw; }
        try { o.push_frame_AoS(nullptr, nullptr, 0, 0, 256, 1.0f); } catch (const std::invalid_argument&) { ++threw; }
        float* outs[2] = {nullptr, nullptr};
        try { o.produce(outs, 1); } catch (const std::invalid_argument&) { ++threw; }
        EXPECT(threw == 6, "exceptions %d", threw);
        o.set_window(w.data(), 256);
        std::vector<float> aos(512);
        for (int i = 0; i < 512; ++i) aos[i] = (i % 2) ? -0.25f : 0.5f;
        o.push_frame_AoS(aos.data(), nullptr, 0, 0, 256, 1.0f);
        std::vector<float> c0(64), c1(64);
        float* co[2] = {c0.data(), c1.data()};
        EXPECT(o.produce(co, 64) == 64 && o.read_pos() == 64 && o.produced_samples() == 256, "counters");
        EXPECT(o.meter_peak() > 0.0f && o.has_window() && o.ring_size() == 24 * 64, "state");
        o.reset();
        EXPECT(!o.has_window() && o.produced_samples() == 0 && o.meter_peak() == 0.0f, "reset");
    }
    // e2e round trip: StftEngine vs the oracle restatement of e2e_benchmark.cc
    {
        crlot::StftEngine::Config c;
        crlot::StftEngine eng(c);
        const int S = 3;
        const int64_t T = 48000;
        std::vector<float> x(S * T);
        for (int s = 0; s < S; ++s) or_synth_fill(x.data() + s * T, T, 1000 + s);
        auto y = eng.roundtrip(x, S, T);
        const int64_t L = eng.output_length(T);
        std::vector<float> ref(L);
        for (int s = 0; s < S; ++s) {
            or_roundtrip(x.data() + s * T, T, 1024, 256, OR_HANN, 0, OR_ZERO_PAD, ref.data(), L, nullptr, nullptr);
            double num = 0, den = 0, mx = 0;
            for (int64_t i = 0; i < L; ++i) {
                double d = double(y[s * L + i]) - ref[i];
                num += d * d;
                den += double(ref[i]) * ref[i];
                mx = std::fmax(mx, std::fabs(d));
            }
            EXPECT(std::sqrt(num / den) < 1e-6 && mx < 2e-6, "stream %d rel %g max %g", s, std::sqrt(num / den), mx);
        }
        // the split round trip (stft_device -> istft_ola_device) and a per-frame mask
        // through the same engine: within the FFT tolerance of the round trip, and
        // the masked round trip of the oracle's masked loop
        const int64_t F = eng.frame_count(T), B = eng.bins(), R = 1024 + 2;
        crlot::DeviceBuffer<float> dx(S * T), dy(S * L), dspec(S * F * R), dmask(F * B);
        crlot::hip_check(hipMemcpy(dx.get(), x.data(), sizeof(float) * S * T, hipMemcpyHostToDevice), "up");
        eng.stft_device(dx.get(), dspec.get(), S, T, T, F * R, R);
        eng.istft_ola_device(dspec.get(), dy.get(), S, F, F * R, R, L);
        std::vector<float> y2(S * L), mask(F * B), ym(L);
        crlot::hip_check(hipMemcpy(y2.data(), dy.get(), sizeof(float) * S * L, hipMemcpyDeviceToHost), "down");
        double mx2 = 0;
        for (int64_t i = 0; i < S * L; ++i) mx2 = std::fmax(mx2, std::fabs(double(y2[i]) - y[i]));
        EXPECT(mx2 < 2e-6, "istft_ola(stft) vs roundtrip max %g", mx2);
        for (int64_t k = 0; k < F; ++k)
            for (int64_t b = 0; b < B; ++b) mask[k * B + b] = float(0.5 + 0.5 * std::cos(0.01 * double(b) + 0.3 * double(k)));
        crlot::hip_check(hipMemcpy(dmask.get(), mask.data(), sizeof(float) * F * B, hipMemcpyHostToDevice), "up");
        eng.set_spectral_mask(dmask.get());
        eng.roundtrip_device(dx.get(), dy.get(), S, T, T, L);
        eng.set_spectral_mask(nullptr);
        crlot::hip_check(hipMemcpy(y2.data(), dy.get(), sizeof(float) * S * L, hipMemcpyDeviceToHost), "down");
        for (int s = 0; s < S; ++s) {
            or_roundtrip_mask(x.data() + s * T, T, 1024, 256, OR_HANN, 0, OR_ZERO_PAD, 1, 0, 1, nullptr, mask.data(),
                              size_t(B), ym.data(), L, nullptr);
            double mxm = 0;
            for (int64_t i = 0; i < L; ++i) mxm = std::fmax(mxm, std::fabs(double(y2[s * L + i]) - ym[i]));
            EXPECT(mxm < 2e-6, "masked stream %d max %g", s, mxm);
        }
    }
    // io::WavReader / WavWriter (wav_io_test.cc WriteAndRead) + the oboe fixture
    {
        crlot::io::WavReader r;
        EXPECT(!r.open("nonexistent.wav") && !r.is_open(), "nonexistent");
        if (r.open(CRLOT_GOLDEN_DIR "/oboe.wav")) {
            EXPECT(r.get_channels() == 2 && r.get_sample_rate() == 44100 && r.get_bits_per_sample() == 16 &&
                       r.get_total_frames() == 285315,
                   "oboe info");
            EXPECT(r.read_all().size() == 285315u * 2, "oboe read_all");
        } else {
            EXPECT(false, "oboe.wav fixture missing");
        }
        const char* path = "/tmp/crlot_cpp_wav_test.wav";
        std::vector<float> d(2 * 1000);
        for (size_t i = 0; i < d.size(); ++i) d[i] = 0.4f * std::sin(0.01f * float(i));
        crlot::io::WavWriter w;
        size_t put = 0;
        EXPECT(w.open(path, 2, 48000, 24) && w.write(d.data(), 1000, &put) && put == 1000, "wav write");
        w.close();
        crlot::io::WavReader r2;
        EXPECT(r2.open(path) && r2.get_total_frames() == 1000 && r2.get_bits_per_sample() == 24, "wav reopen");
        auto back = r2.read_all();
        float mx = 0;
        for (size_t i = 0; i < d.size(); ++i) mx = std::fmax(mx, std::fabs(back[i] - d[i]));
        EXPECT(back.size() == d.size() && mx < 1e-4f, "24-bit round trip %g", mx);
        std::remove(path);
    }
    std::printf("%s (%d failures)\n", failures ? "FAILED" : "OK", failures);
    return failures ? 1 : 0;
}
