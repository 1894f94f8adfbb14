// pipeline_bench: counterpart of the reference's integrated pipeline,
// bench/performance_benchmark.cc:174-246 (IntegratedPipelinePerformance),
// written against the drop-in classes of include/crlot_dsp.hpp as the
// reference writes it against dsp::*: per iteration
//   FrameQueue(x, 16384, 1024, 512, center = true)        (:181)
//   WindowLUT::GetWindowSafe(HANN, 1024); OLAAccumulator(apply_window_inside)
//   MakeFftPlan(Real, 1024)
//   per frame: copy -> forward -> inverse -> add_frame_SoA(window, i*hop)  (:213-229)
//   produce(hop) until 16384 samples                                       (:232-240)
// The reference pushes every frame before producing, which aliases its ring
// once 16384 + 512 > ring; this counterpart times that literal
// order ("literal") and the streaming-interleaved one ("interleaved": produce
// after each add, the semantics the batched engine implements).
// Usage: pipeline_bench [iterations=200]
#include <algorithm>
#include <chrono>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../include/crlot_dsp.hpp"

using namespace crlot::dsp;
using namespace crlot::dsp::fft;
using clk = std::chrono::steady_clock;

static double p50(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[v.size() / 2];
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 200;
    const size_t L = 16384, N = 1024, H = 512;
    std::vector<float> x(L);
    std::mt19937 gen(42);
    std::normal_distribution<float> dist(0.0f, 1.0f);
    for (auto& v : x) v = dist(gen);
    struct Times {
        double total_us, loop_us;
        size_t frames;
        double fq_us, ola_us, first_fwd_us;  // construction of the FrameQueue / the OLA object; frame 0's forward
        double part_us[5];                   // loop totals: getFrame + copy, forward (frames >= 1), inverse, add, produce
        double destroy_us;                   // the objects' destruction (inside total_us)
    };
    try {
        auto run_objects = [&](bool interleaved, clk::time_point t0) -> Times {
            FrameQueue frames(x.data(), L, N, H, true);
            const auto t_fq = clk::now();
            auto window = WindowLUT::getInstance().GetWindowSafe(WindowType::HANN, N);
            OLAConfig config;
            config.sample_rate = 48000;
            config.frame_size = N;
            config.hop_size = H;
            config.channels = 1;
            config.eps = 1e-8f;
            config.apply_window_inside = true;
            OLAAccumulator ola(config);
            ola.set_window(window.get(), int(N));
            const auto t_ola = clk::now();
            FftPlanDesc desc{FftDomain::Real, int(N), false, 1, 1, 1};
            auto fft_plan = MakeFftPlan(desc);
            std::vector<std::complex<float>> spectrum(N / 2 + 1);
            std::vector<float> processed(N), output(L + N);
            const auto t_loop = clk::now();
            double first_fwd = 0.0, part[5] = {0, 0, 0, 0, 0};
            auto lap = [](clk::time_point& t, double& acc) {
                const auto n = clk::now();
                acc += std::chrono::duration<double, std::micro>(n - t).count();
                t = n;
            };
            size_t total = 0;
            float* ch_out[1] = {output.data()};
            for (size_t i = 0; i < frames.getNumFrames(); ++i) {
                auto tp = clk::now();
                const float* frame = frames.getFrame(i);
                std::copy(frame, frame + N, processed.begin());
                lap(tp, part[0]);
                fft_plan->forward(processed.data(), spectrum.data());
                if (i == 0) {
                    first_fwd = std::chrono::duration<double, std::micro>(clk::now() - tp).count();
                    tp = clk::now();
                } else {
                    lap(tp, part[1]);
                }
                fft_plan->inverse(spectrum.data(), processed.data());
                lap(tp, part[2]);
                const float* ch_frames[1] = {processed.data()};
                ola.add_frame_SoA(ch_frames, window.get(), i * H, 0, N, 1.0f);
                lap(tp, part[3]);
                if (interleaved && total < L) {
                    ch_out[0] = output.data() + total;
                    total += ola.produce(ch_out, H);
                }
                lap(tp, part[4]);
            }
            while (total < L) {
                ch_out[0] = output.data() + total;
                const size_t s = ola.produce(ch_out, H);
                if (s == 0) break;
                total += s;
            }
            const auto t1 = clk::now();
            auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
            return Times{us(t0, t1), us(t_loop, t1), frames.getNumFrames(), us(t0, t_fq), us(t_fq, t_ola), first_fwd,
                         {part[0], part[1], part[2], part[3], part[4]}, 0.0};
        };
        // the reference's iteration ends with its objects' destruction (the loop
        // body's scope, performance_benchmark.cc:179-243): timed too
        auto run = [&](bool interleaved) -> Times {
            const auto t0 = clk::now();
            Times t = run_objects(interleaved, t0);
            const double end = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
            t.destroy_us = end - t.total_us;
            t.total_us = end;
            return t;
        };
        for (int w = 0; w < 5; ++w) run(true);
        std::vector<double> lit, ilv, lit_loop, ilv_loop, fq, olac, ff, part[5], dst;
        size_t F = 0;
        for (int i = 0; i < iters; ++i) {
            const Times a = run(false), b = run(true);
            lit.push_back(a.total_us);
            ilv.push_back(b.total_us);
            lit_loop.push_back(a.loop_us);
            ilv_loop.push_back(b.loop_us);
            fq.push_back(b.fq_us);
            olac.push_back(b.ola_us);
            ff.push_back(b.first_fwd_us);
            for (int q = 0; q < 5; ++q) part[q].push_back(b.part_us[q]);
            dst.push_back(b.destroy_us);
            F = a.frames;
        }
        // what the batched speculation served per interleaved iteration (batches,
        // forwards, inverses, pushes, produces, ring rebuilds; crlot_call_speculation_stats)
        int64_t s0[6], s1[6];
        crlot_call_speculation_stats(s0);
        for (int i = 0; i < 10; ++i) run(true);
        crlot_call_speculation_stats(s1);
        // total: the reference's iteration (object construction and destruction
        // included, :179-243);
        // loop: the per-frame calls and the produce loop only
        std::printf("{\"harness\": \"pipeline_bench\", \"reference\": \"bench/performance_benchmark.cc:174-246\", "
                    "\"input_length\": %zu, \"frame\": %zu, \"hop\": %zu, \"frames\": %zu, \"iterations\": %d, "
                    "\"literal\": {\"total_us_p50\": %.2f, \"loop_us_p50\": %.2f, \"loop_us_per_frame\": %.3f}, "
                    "\"interleaved\": {\"total_us_p50\": %.2f, \"loop_us_p50\": %.2f, \"loop_us_per_frame\": %.3f, "
                    "\"served_per_iteration\": {\"batches\": %.1f, \"forwards\": %.1f, \"inverses\": %.1f, "
                    "\"pushes\": %.1f, \"produces\": %.1f, \"rebuilds\": %.1f}, "
                    "\"framequeue_us_p50\": %.2f, \"ola_object_us_p50\": %.2f, \"first_forward_us_p50\": %.2f, "
                    "\"loop_parts_us_p50\": {\"get_copy\": %.2f, \"forward_rest\": %.2f, \"inverse\": %.2f, "
                    "\"add\": %.2f, \"produce\": %.2f}, \"destroy_us_p50\": %.2f}}\n",
                    L, N, H, F, iters, p50(lit), p50(lit_loop), p50(lit_loop) / double(F), p50(ilv), p50(ilv_loop),
                    p50(ilv_loop) / double(F), (s1[0] - s0[0]) / 10.0, (s1[1] - s0[1]) / 10.0,
                    (s1[2] - s0[2]) / 10.0, (s1[3] - s0[3]) / 10.0, (s1[4] - s0[4]) / 10.0, (s1[5] - s0[5]) / 10.0,
                    p50(fq), p50(olac), p50(ff), p50(part[0]), p50(part[1]), p50(part[2]), p50(part[3]),
                    p50(part[4]), p50(dst));
    } catch (const std::exception& e) {
        std::fprintf(stderr, "exception: %s\n", e.what());
        return 4;
    }
    return 0;
}
