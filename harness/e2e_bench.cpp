// e2e_bench: counterpart of the reference's bench/e2e_benchmark.cc, written
// against the drop-in classes of include/crlot_dsp.hpp exactly as the reference
// writes it against dsp::* -- Framer, WindowLUT::GetWindowSafe, MakeFftPlan
// (one plan for forward and inverse), OLAAccumulator(apply_window_inside) --
// on its input (1 s of 48 kHz mono, 0.5 sin 440 + 0.3 sin 880 + 0.2 sin 1320,
// :26-40).  One JSON line:
//   full_pipeline   the :138-186 loop per iteration (push 48000 samples, pop /
//                   window / forward / inverse / push_frame_AoS per frame), in
//                   the streaming-interleaved order (produce(H) after each push:
//                   SURVEY Q3) -- ms per iteration, x real-time (48000 samples /
//                   time, :311-317), us per frame
//   harness_order   the same loop in the harness's literal order (every push,
//                   then the produce loop; its ring aliases, Q3), timed alike
//   per_call        p50 us of each call of the loop, in the loop
//   spectral_gain   the streaming-interleaved loop with a spectral step where
//                   :161-162 marks one ("filtering or other processing could go
//                   here"): every bin k of each spectrum scaled by the real gain
//                   0.5 + 0.5 cos(pi k / (N/2)) on the host, between forward
//                   and inverse -- ms per iteration, us per frame, per-call p50
//   spectral_mask   the same with a time-varying mask: frame k scaled by mask
//                   k mod 8, 0.5 + 0.5 cos(pi k / (N/2) + 0.7 j) (no fixed gain)
//   fft1024         IFftPlan::forward alone, p50 us (:187-205, 10000 calls)
//   quality         SNR and cross-correlation delay exactly as :77-128 compute
//                   them, on the streaming-interleaved output
//   (fft_forward_us_p50: the same at the frame size given, 1024 by default)
// Usage: e2e_bench [hop=256] [iterations=200] [frame=1024]
#include <algorithm>
#include <chrono>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <vector>

#include "../include/crlot_dsp.hpp"

using namespace crlot::dsp;
using namespace crlot::dsp::fft;
using clk = std::chrono::steady_clock;

static double us_since(clk::time_point t0) {
    return std::chrono::duration<double, std::micro>(clk::now() - t0).count();
}

static double pct(std::vector<double> v, double q) {
    if (v.empty()) return 0.0;
    std::sort(v.begin(), v.end());
    return v[size_t(q * double(v.size() - 1))];
}
static double p50(const std::vector<double>& v) { return pct(v, 0.5); }

// e2e_benchmark.cc:77-100
static double calculate_snr(const std::vector<float>& original, const std::vector<float>& processed) {
    if (original.size() != processed.size()) return -std::numeric_limits<double>::infinity();
    double signal_power = 0.0, noise_power = 0.0;
    for (size_t i = 0; i < original.size(); ++i) {
        const double diff = original[i] - processed[i];
        signal_power += original[i] * original[i];
        noise_power += diff * diff;
    }
    if (noise_power < 1e-12) return std::numeric_limits<double>::infinity();
    return 10.0 * std::log10(signal_power / noise_power);
}

// e2e_benchmark.cc:103-122 (ms)
static double calculate_delay(const std::vector<float>& original, const std::vector<float>& processed, double sr) {
    const size_t max_delay = 1024;
    double max_corr = -1.0;
    size_t best_delay = 0;
    for (size_t delay = 0; delay < max_delay; ++delay) {
        double corr = 0.0;
        const size_t overlap = std::min(original.size() - delay, processed.size());
        for (size_t i = 0; i < overlap; ++i) corr += original[i] * processed[i + delay];
        if (corr > max_corr) {
            max_corr = corr;
            best_delay = delay;
        }
    }
    return double(best_delay) / sr * 1000.0;
}

struct Pipeline {
    size_t N, H;
    Framer framer;
    std::shared_ptr<const float> win_holder;
    const float* window = nullptr;
    std::unique_ptr<OLAAccumulator> ola;
    std::unique_ptr<IFftPlan> plan;

    Pipeline(size_t n, size_t h) : N(n), H(h) {
        framer.set_params(N, H, 1, BoundaryMode::ZERO_PAD);
        win_holder = WindowLUT::getInstance().GetWindowSafe(WindowType::HANN, N);
        window = win_holder.get();
        OLAConfig c;
        c.sample_rate = 48000;
        c.frame_size = N;
        c.hop_size = H;
        c.channels = 1;
        c.apply_window_inside = true;
        ola = std::make_unique<OLAAccumulator>(c);
        ola->set_window(window, int(N));
        FftPlanDesc d;
        d.domain = FftDomain::Real;
        d.nfft = int(N);
        d.in_place = false;
        d.batch = 1;
        d.stride_in = 1;
        d.stride_out = 1;
        plan = MakeFftPlan(d);
    }
};

int main(int argc, char** argv) {
    const size_t H = argc > 1 ? std::strtoul(argv[1], nullptr, 10) : 256;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 200;
    const size_t N = argc > 3 ? std::strtoul(argv[3], nullptr, 10) : 1024, T = 48000;
    const double sr = 48000.0;
    std::vector<float> x(T);
    for (size_t i = 0; i < T; ++i) {
        const double t = double(i) / sr;
        x[i] = 0.5f * std::sin(2.0 * M_PI * 440.0 * t) + 0.3f * std::sin(2.0 * M_PI * 880.0 * t) +
               0.2f * std::sin(2.0 * M_PI * 1320.0 * t);
    }
    try {
        Pipeline p(N, H);
        std::vector<float> frame(N), processed(N), output(T + N);
        std::vector<std::complex<float>> spectrum(N / 2 + 1);
        std::vector<double> t_pop, t_fwd, t_inv, t_push, t_prod;
        size_t frames = 0;
        // one iteration; returns its time (us) without the reset that re-arms the
        // objects for the next one (the reference keeps its OLA across iterations)
        auto streaming_iteration = [&](bool record, std::vector<float>* out) {
            size_t produced = 0;
            float* ch_out[1] = {output.data()};
            const auto t_begin = clk::now();
            p.framer.push(x.data(), T);
            size_t k = 0;
            for (;;) {
                auto t0 = clk::now();
                if (!p.framer.pop(frame.data())) break;
                for (size_t i = 0; i < N; ++i) processed[i] = frame[i] * p.window[i];
                auto t1 = clk::now();
                p.plan->forward(processed.data(), spectrum.data());
                auto t2 = clk::now();
                p.plan->inverse(spectrum.data(), processed.data());
                auto t3 = clk::now();
                p.ola->push_frame_AoS(processed.data(), nullptr, k * H, 0, N, 1.0f);
                auto t4 = clk::now();
                ch_out[0] = output.data() + produced;
                produced += p.ola->produce(ch_out, H);
                auto t5 = clk::now();
                if (record) {
                    t_pop.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
                    t_fwd.push_back(std::chrono::duration<double, std::micro>(t2 - t1).count());
                    t_inv.push_back(std::chrono::duration<double, std::micro>(t3 - t2).count());
                    t_push.push_back(std::chrono::duration<double, std::micro>(t4 - t3).count());
                    t_prod.push_back(std::chrono::duration<double, std::micro>(t5 - t4).count());
                }
                ++k;
            }
            const double us = us_since(t_begin);
            frames = k;
            if (out) out->assign(output.begin(), output.begin() + std::min(produced, T));
            p.ola->reset();
            p.ola->set_window(p.window, int(N));
            p.framer.reset();
            return us;
        };
        // warm-up (launches the call kernels), then the timed iterations
        for (int w = 0; w < 3; ++w) streaming_iteration(false, nullptr);
        std::vector<double> it_us;
        for (int it = 0; it < iters; ++it) it_us.push_back(streaming_iteration(it % 4 == 0, nullptr));
        std::vector<float> y;
        streaming_iteration(false, &y);
        y.resize(T, 0.0f);
        const double snr = calculate_snr(x, y), delay = calculate_delay(x, y, sr);

        // the spectral step on the host between the transforms: frame k's bins
        // scaled by masks[k % masks.size()] (one mask: a fixed per-bin gain)
        struct SpecRun {
            std::vector<double> it, fwd, inv, push, prod;
        };
        auto spectral_loop = [&](const std::vector<std::vector<float>>& masks) {
            SpecRun r;
            for (int it = -3; it < std::max(iters / 2, 20); ++it) {
                size_t produced = 0, k = 0;
                float* ch_out[1] = {output.data()};
                const auto t_begin = clk::now();
                p.framer.push(x.data(), T);
                while (p.framer.pop(frame.data())) {
                    for (size_t i = 0; i < N; ++i) processed[i] = frame[i] * p.window[i];
                    auto t1 = clk::now();
                    p.plan->forward(processed.data(), spectrum.data());
                    auto t2 = clk::now();
                    const std::vector<float>& g = masks[k % masks.size()];
                    for (size_t b = 0; b <= N / 2; ++b) spectrum[b] *= g[b];
                    p.plan->inverse(spectrum.data(), processed.data());
                    auto t3 = clk::now();
                    p.ola->push_frame_AoS(processed.data(), nullptr, k * H, 0, N, 1.0f);
                    auto t4 = clk::now();
                    ch_out[0] = output.data() + produced;
                    produced += p.ola->produce(ch_out, H);
                    auto t5 = clk::now();
                    if (it >= 0 && it % 4 == 0) {
                        r.fwd.push_back(std::chrono::duration<double, std::micro>(t2 - t1).count());
                        r.inv.push_back(std::chrono::duration<double, std::micro>(t3 - t2).count());
                        r.push.push_back(std::chrono::duration<double, std::micro>(t4 - t3).count());
                        r.prod.push_back(std::chrono::duration<double, std::micro>(t5 - t4).count());
                    }
                    ++k;
                }
                if (it >= 0) r.it.push_back(us_since(t_begin));
                p.ola->reset();
                p.ola->set_window(p.window, int(N));
                p.framer.reset();
            }
            return r;
        };
        std::vector<float> bin_gain(N / 2 + 1);
        for (size_t k = 0; k <= N / 2; ++k) bin_gain[k] = float(0.5 + 0.5 * std::cos(M_PI * double(k) / double(N / 2)));
        const SpecRun gain_run = spectral_loop({bin_gain});
        // a time-varying mask (a noise suppressor's shape): eight masks in turn,
        // 0.5 + 0.5 cos(pi k / (N/2) + 0.7 j) -- no fixed gain to learn
        std::vector<std::vector<float>> masks(8, std::vector<float>(N / 2 + 1));
        for (size_t j = 0; j < masks.size(); ++j)
            for (size_t k = 0; k <= N / 2; ++k)
                masks[j][k] = float(0.5 + 0.5 * std::cos(M_PI * double(k) / double(N / 2) + 0.7 * double(j)));
        const SpecRun mask_run = spectral_loop(masks);

        // the harness's literal order: every push, then the produce loop (ring aliasing, Q3)
        std::vector<double> ho_us, ho_frames_us, ho_produce_us;
        int64_t st0[11] = {0}, st1[11] = {0};
        (void)crlot_call_speculation_stats_ex(st0, 11);
        for (int it = 0; it < std::max(iters / 4, 10); ++it) {
            auto t0 = clk::now();
            p.framer.push(x.data(), T);
            size_t k = 0;
            while (p.framer.pop(frame.data())) {
                for (size_t i = 0; i < N; ++i) processed[i] = frame[i] * p.window[i];
                p.plan->forward(processed.data(), spectrum.data());
                p.plan->inverse(spectrum.data(), processed.data());
                p.ola->push_frame_AoS(processed.data(), nullptr, k * H, 0, N, 1.0f);
                ++k;
            }
            const auto t1 = clk::now();
            size_t got = 0;
            float* ch_out[1] = {output.data()};
            while (got < T) {
                ch_out[0] = output.data() + got;
                const size_t s = p.ola->produce(ch_out, T - got);
                if (s == 0) break;
                got += s;
            }
            ho_us.push_back(us_since(t0));  // the reset below re-arms the objects, untimed
            ho_frames_us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
            ho_produce_us.push_back(us_since(t1));
            p.ola->reset();
            p.ola->set_window(p.window, int(N));
            p.framer.reset();
        }
        (void)crlot_call_speculation_stats_ex(st1, 11);

        // FFT1024Performance (:187-205): forward alone
        std::vector<double> f_us;
        for (size_t i = 0; i < N; ++i) processed[i] = x[i] * p.window[i];
        for (int i = 0; i < 10000; ++i) {
            auto t0 = clk::now();
            p.plan->forward(processed.data(), spectrum.data());
            f_us.push_back(us_since(t0));
        }

        const double it_p50 = p50(it_us), ho_p50 = p50(ho_us);
        std::printf(
            "{\"harness\": \"e2e_bench\", \"reference\": \"bench/e2e_benchmark.cc\", \"frame\": %zu, \"hop\": %zu, "
            "\"samples\": %zu, \"frames_per_iteration\": %zu, \"iterations\": %d, "
            "\"full_pipeline\": {\"order\": \"streaming-interleaved\", \"ms_p50\": %.4f, \"x_realtime\": %.2f, "
            "\"reference_reporter_value\": %.1f, \"us_per_frame\": %.3f, \"msamples_s\": %.3f}, "
            "\"harness_order\": {\"ms_p50\": %.4f, \"x_realtime\": %.2f, \"us_per_frame\": %.3f, "
            "\"frames_loop_us_p50\": %.1f, \"produce_loop_us_p50\": %.1f, \"speculation_delta\": "
            "{\"starts\": %lld, \"forwards\": %lld, \"inverses\": %lld, \"pushes\": %lld, \"produces\": %lld, "
            "\"rebuilds\": %lld, \"windows\": %lld, \"declined\": %lld}}, "
            "\"per_call_us_p50\": {\"pop_window\": %.3f, \"forward\": %.3f, \"inverse\": %.3f, \"push_frame_AoS\": "
            "%.3f, \"produce\": %.3f}, "
            "\"forward_us_p10_p90\": [%.3f, %.3f], \"inverse_us_p10_p90\": [%.3f, %.3f], "
            "\"fft_forward_us_p50\": %.3f, "
            "\"spectral_gain\": {\"order\": \"streaming-interleaved\", \"ms_p50\": %.4f, \"us_per_frame\": %.3f, "
            "\"per_call_us_p50\": {\"forward\": %.3f, \"gain_and_inverse\": %.3f, \"push_frame_AoS\": %.3f, "
            "\"produce\": %.3f}}, "
            "\"spectral_mask\": {\"order\": \"streaming-interleaved\", \"masks\": 8, \"ms_p50\": %.4f, "
            "\"us_per_frame\": %.3f, \"per_call_us_p50\": {\"forward\": %.3f, \"mask_and_inverse\": %.3f, "
            "\"push_frame_AoS\": %.3f, \"produce\": %.3f}}, "
            "\"quality\": {\"snr_db\": %.4f, \"delay_ms\": %.4f}}\n",
            // 1 s of audio per iteration: x real-time = 1 s / iteration time; the
            // reference's reporter prints (48000 / ms) * 1000 under that name (:311-317)
            N, H, T, frames, iters, it_p50 / 1e3, 1e6 / it_p50, 48000.0 / (it_p50 / 1e3) * 1000.0,
            it_p50 / double(frames), double(T) / it_p50, ho_p50 / 1e3, 1e6 / ho_p50, ho_p50 / double(frames),
            p50(ho_frames_us), p50(ho_produce_us), (long long)(st1[0] - st0[0]), (long long)(st1[1] - st0[1]),
            (long long)(st1[2] - st0[2]), (long long)(st1[3] - st0[3]), (long long)(st1[4] - st0[4]),
            (long long)(st1[5] - st0[5]), (long long)(st1[7] - st0[7]), (long long)(st1[8] - st0[8]), p50(t_pop),
            p50(t_fwd), p50(t_inv), p50(t_push), p50(t_prod), pct(t_fwd, 0.1), pct(t_fwd, 0.9), pct(t_inv, 0.1),
            pct(t_inv, 0.9), p50(f_us), p50(gain_run.it) / 1e3, p50(gain_run.it) / double(frames), p50(gain_run.fwd),
            p50(gain_run.inv), p50(gain_run.push), p50(gain_run.prod), p50(mask_run.it) / 1e3,
            p50(mask_run.it) / double(frames), p50(mask_run.fwd), p50(mask_run.inv), p50(mask_run.push),
            p50(mask_run.prod), snr, delay);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "exception: %s\n", e.what());
        return 4;
    }
    return 0;
}
