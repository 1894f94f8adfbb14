// e2e_loop: the reference harness's pipeline (bench/e2e_benchmark.cc:42-76 set-up,
// :138-186 loop) written against the reference's own headers (include/ref/dsp/...: the
// drop-in classes of include/crlot_dsp.hpp under the names dsp::*), in the streaming-interleaved
// order (push frame k, then produce(H)):
//
//   Framer::push(x, T) -> while pop(frame): p = frame * w -> IFftPlan::forward
//   -> IFftPlan::inverse -> OLAAccumulator::push_frame_AoS(p, nullptr, k*H, 0, N, 1)
//   -> produce(ch_out, H)
//
// with C interleaved channels (Framer(N, H, C); one forward plan reading stride
// C, one inverse plan writing stride C, so the OLA gets the interleaved frame).
// Usage: e2e_loop x.f32 T C N H zpad|drop y.f32 frames.f32
//   x.f32       T*C interleaved floats
//   y.f32       written: [C][F*H] produced samples, channel-major
//   frames.f32  written: [F][N*C] the push_frame_AoS inputs (for the bit-exact
//               OLA check against the oracle)
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

// The reference harness's own includes and using-directives (bench/e2e_benchmark.cc:8-15),
// resolved by the drop-in headers under include/ref (-I include/ref): no source edit.
#include "dsp/ola/OLAAccumulator.h"
#include "dsp/window/WindowLUT.h"
#include "dsp/frame/framer.h"
#include "dsp/fft/api/fft_api.h"
#include "io/wav.h"

using namespace dsp;
using namespace dsp::fft;

static std::vector<float> read_f32(const char* path, size_t n) {
    std::vector<float> v(n);
    FILE* f = std::fopen(path, "rb");
    if (!f || std::fread(v.data(), sizeof(float), n, f) != n) {
        std::fprintf(stderr, "cannot read %zu floats from %s\n", n, path);
        std::exit(2);
    }
    std::fclose(f);
    return v;
}

static void write_f32(const char* path, const std::vector<float>& v) {
    FILE* f = std::fopen(path, "wb");
    if (!f || std::fwrite(v.data(), sizeof(float), v.size(), f) != v.size()) std::exit(3);
    std::fclose(f);
}

int main(int argc, char** argv) {
    if (argc != 9) {
        std::fprintf(stderr, "usage: e2e_loop x.f32 T C N H zpad|drop y.f32 frames.f32\n");
        return 1;
    }
    const size_t T = std::strtoull(argv[2], nullptr, 10), C = std::strtoull(argv[3], nullptr, 10);
    const size_t N = std::strtoull(argv[4], nullptr, 10), H = std::strtoull(argv[5], nullptr, 10);
    const BoundaryMode mode = std::string(argv[6]) == "drop" ? BoundaryMode::DROP : BoundaryMode::ZERO_PAD;
    const std::vector<float> x = read_f32(argv[1], T * C);
    try {
        // e2e_benchmark.cc:42-76
        Framer framer;
        framer.set_params(N, H, C, mode);
        WindowLUT& lut = WindowLUT::getInstance();
        auto safe_window = lut.GetWindowSafe(WindowType::HANN, N);
        const float* window = safe_window.get();
        OLAConfig ola_config;
        ola_config.sample_rate = 48000;
        ola_config.frame_size = N;
        ola_config.hop_size = H;
        ola_config.channels = C;
        ola_config.apply_window_inside = true;
        auto ola = std::make_unique<OLAAccumulator>(ola_config);
        ola->set_window(window, int(N));
        FftPlanDesc fwd_desc{FftDomain::Real, int(N), false, 1, int(C), 1};
        FftPlanDesc inv_desc{FftDomain::Real, int(N), false, 1, 1, int(C)};
        auto fwd = MakeFftPlan(fwd_desc);
        auto inv = MakeFftPlan(inv_desc);

        // e2e_benchmark.cc:138-186, streaming-interleaved
        framer.push(x.data(), T);
        std::vector<float> frame(N * C), processed(N * C), synth(N * C);
        std::vector<std::complex<float>> spectrum(N / 2 + 1);
        std::vector<std::vector<float>> out(C);
        std::vector<float> pushed;
        std::vector<float> hop(H * C);
        std::vector<float*> ch_out(C);
        for (size_t c = 0; c < C; ++c) ch_out[c] = hop.data() + c * H;
        size_t k = 0;
        while (framer.pop(frame.data())) {
            for (size_t i = 0; i < N; ++i)
                for (size_t c = 0; c < C; ++c) processed[i * C + c] = frame[i * C + c] * window[i];
            for (size_t c = 0; c < C; ++c) {
                fwd->forward(processed.data() + c, spectrum.data());
                inv->inverse(spectrum.data(), synth.data() + c);
            }
            ola->push_frame_AoS(synth.data(), nullptr, k * H, 0, N, 1.0f);
            pushed.insert(pushed.end(), synth.begin(), synth.end());
            const size_t got = ola->produce(ch_out.data(), H);
            for (size_t c = 0; c < C; ++c) out[c].insert(out[c].end(), ch_out[c], ch_out[c] + got);
            ++k;
        }
        std::vector<float> y;
        for (size_t c = 0; c < C; ++c) y.insert(y.end(), out[c].begin(), out[c].end());
        write_f32(argv[7], y);
        write_f32(argv[8], pushed);
        std::printf("frames %zu produced %zu peak %.9g\n", k, out[0].size(), double(ola->meter_peak()));
    } catch (const std::exception& e) {
        std::fprintf(stderr, "exception: %s\n", e.what());
        return 4;
    }
    return 0;
}
