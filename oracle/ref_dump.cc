// ref_dump.cc -- fixture generator linked against the REFERENCE's own sources.
//
// TEST INFRASTRUCTURE ONLY.  Built by oracle/Makefile (target `ref`) from
// /root/reference/dsp/window/WindowLUT.cc, dsp/ola/norm_builder.cc,
// dsp/frame/framer.cc, dsp/frame/FrameQueue.cc, dsp/ola/kernels.cc (its scalar
// kernels; the Highway dispatchers are dropped by --gc-sections, nothing stands
// in for them), dsp/ring/ring_buffer.cc, dsp/ola/aos_to_soa.cc and
// dsp/base/aligned_alloc.cc compiled unchanged with the reference's release flags
// (-std=c++17 -O3 -DNDEBUG -march=native, scripts/run_all.sh:12).  No stand-in
// headers or libraries are involved: those translation units need only
// the C++ standard library.  Output goes to a directory of raw little-endian
// float32 / uint64 files plus a manifest consumed by tests/golden/make_golden.py.
//
// The reference OLAAccumulator (needs Highway via kernels_hwy.cc) and the
// kissfft adapter (needs the absent kissfft submodule) are NOT built here.
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include <random>

#include "dsp/frame/FrameQueue.h"
#include "dsp/frame/framer.h"
#include "dsp/ola/aos_to_soa.h"
#include "dsp/ola/kernels.h"
#include "dsp/ola/norm_builder.h"
#include "dsp/ring/ring_buffer.h"
#include "dsp/window/WindowLUT.h"

static std::string g_dir;
static FILE* g_manifest = nullptr;

static void dump_f32(const std::string& name, const float* p, size_t n) {
    std::string path = g_dir + "/" + name + ".f32";
    FILE* f = std::fopen(path.c_str(), "wb");
    if (n) std::fwrite(p, sizeof(float), n, f);
    std::fclose(f);
    std::fprintf(g_manifest, "%s f32 %zu\n", name.c_str(), n);
}

static void dump_u64(const std::string& name, const std::vector<uint64_t>& v) {
    std::string path = g_dir + "/" + name + ".u64";
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!v.empty()) std::fwrite(v.data(), sizeof(uint64_t), v.size(), f);
    std::fclose(f);
    std::fprintf(g_manifest, "%s u64 %zu\n", name.c_str(), v.size());
}

static void windows() {
    const dsp::WindowType types[] = {dsp::WindowType::HANN, dsp::WindowType::HAMMING,
                                     dsp::WindowType::BLACKMAN, dsp::WindowType::RECT};
    const char* tnames[] = {"hann", "hamming", "blackman", "rect"};
    const size_t sizes[] = {1, 2, 7, 128, 512, 1000, 1024, 4096};
    const dsp::NormalizationType norms[] = {dsp::NormalizationType::NONE,
                                            dsp::NormalizationType::SUM_TO_ONE,
                                            dsp::NormalizationType::L2_NORM,
                                            dsp::NormalizationType::OLA_UNITY_GAIN,
                                            dsp::NormalizationType::OLA_SUM_WSQ};
    for (int t = 0; t < 4; ++t)
        for (int per = 0; per < 2; ++per)
            for (size_t n : sizes)
                for (int nm = 0; nm < 5; ++nm) {
                    if (nm > 0 && n != 1024 && n != 7) continue;  // keep the fixture small
                    dsp::WindowLUT lut(n, types[t], per != 0, norms[nm]);
                    char name[128];
                    std::snprintf(name, sizeof name, "window_%s_p%d_n%zu_norm%d", tnames[t], per, n,
                                  nm);
                    dump_f32(name, lut.data(), n);
                }
    // GetWindowSafe (the e2e harness path, e2e_benchmark.cc:51-53) must equal the ctor path
    auto safe = dsp::WindowLUT::getInstance().GetWindowSafe(dsp::WindowType::HANN, 1024);
    dump_f32("window_getsafe_hann_1024", safe.get(), 1024);
}

static void norms() {
    struct C { size_t n, h; } cases[] = {{1024, 256}, {4096, 1024}, {512, 128}, {1024, 512},
                                         {256, 64},   {2048, 256},  {1000, 300}, {64, 16}};
    for (auto c : cases) {
        // OLAAccumulator::calculate_ring_size formula (OLAAccumulator.cc:249-258)
        size_t ring = ((c.n + c.h - 1) / c.h + 20) * c.h;
        for (int per = 0; per < 2; ++per) {
            dsp::WindowLUT lut(c.n, dsp::WindowType::HANN, per != 0);
            std::vector<float> norm(ring);
            dsp::ola::build_norm_linear(norm.data(), lut.data(), ring, c.n, c.h);
            char name[128];
            std::snprintf(name, sizeof name, "norm_hann_p%d_n%zu_h%zu_r%zu", per, c.n, c.h, ring);
            dump_f32(name, norm.data(), ring);
        }
    }
    // the reference's own norm_builder_test parameter grid (norm_builder_test.cc:87-93)
    struct G { size_t n, h, ring; } grid[] = {
        {128, 32, 512}, {512, 128, 2048}, {256, 64, 1024}, {64, 16, 256}, {1024, 256, 4096}};
    for (auto g : grid) {
        dsp::WindowLUT lut(g.n, dsp::WindowType::HANN, false);
        std::vector<float> norm(g.ring);
        dsp::ola::build_norm_linear(norm.data(), lut.data(), g.ring, g.n, g.h);
        char name[128];
        std::snprintf(name, sizeof name, "normgrid_n%zu_h%zu_r%zu", g.n, g.h, g.ring);
        dump_f32(name, norm.data(), g.ring);
    }
}

// Run a Framer over input x (T samples x C channels), pushing in chunks of
// `chunk` frames (0 = whole), popping after every push; dump the popped frames.
static void framer_case(const std::string& tag, const std::vector<float>& x, size_t T, size_t C,
                        size_t N, size_t H, dsp::BoundaryMode mode, size_t chunk) {
    dsp::Framer fr;
    fr.set_params(N, H, C, mode);
    std::vector<float> frames, buf(N * C);
    std::vector<uint64_t> avail_trace;
    size_t pos = 0;
    if (chunk == 0) chunk = T;
    while (pos < T) {
        size_t n = std::min(chunk, T - pos);
        fr.push(x.data() + pos * C, n);
        pos += n;
        avail_trace.push_back(fr.available_frames());
        while (fr.pop(buf.data())) frames.insert(frames.end(), buf.begin(), buf.end());
    }
    dump_f32("framer_" + tag, frames.data(), frames.size());
    dump_u64("framer_" + tag + "_avail", avail_trace);
}

static void framers() {
    // ramp 1..20, N=8 H=2 (SURVEY Appendix A probe)
    std::vector<float> ramp(20);
    for (int i = 0; i < 20; ++i) ramp[i] = float(i + 1);
    for (int m = 0; m < 2; ++m) {
        auto mode = m ? dsp::BoundaryMode::DROP : dsp::BoundaryMode::ZERO_PAD;
        const char* mn = m ? "drop" : "zpad";
        for (size_t chunk : {size_t(0), size_t(2), size_t(3), size_t(7)}) {
            framer_case(std::string("ramp20_n8_h2_") + mn + "_c" + std::to_string(chunk), ramp, 20,
                        1, 8, 2, mode, chunk);
        }
        // stereo interleaved ramp: 10 frames x 2 ch
        framer_case(std::string("ramp20_st_n4_h2_") + mn, ramp, 10, 2, 4, 2, mode, 0);
        // edge lengths around N for N=1024 H=256
        for (size_t T : {size_t(1), size_t(255), size_t(1023), size_t(1024), size_t(1025),
                         size_t(4096 + 77)}) {
            std::vector<float> x(T);
            for (size_t i = 0; i < T; ++i) x[i] = float(i % 1000) / 1024.0f - 0.5f;  // exact in float
            framer_case(std::string("edge_t") + std::to_string(T) + "_" + mn, x, T, 1, 1024, 256,
                        mode, 0);
        }
        // hop that does not divide N, chunked by hop (config-4 style per-hop pushes)
        std::vector<float> x(3000);
        for (size_t i = 0; i < x.size(); ++i) x[i] = float(i);
        framer_case(std::string("n512_h128_perhop_") + mn, x, 3000, 1, 512, 128, mode, 128);
        framer_case(std::string("n100_h30_") + mn, x, 1000, 1, 100, 30, mode, 0);
    }
}

// FrameQueue (FrameQueue.cc:9-115, Indexing.h:18-70): every pad mode, center
// on/off, signals shorter than the pad (multi-bounce reflect101), odd sizes.
static void framequeues() {
    const dsp::PadMode modes[] = {dsp::PadMode::CONSTANT, dsp::PadMode::REFLECT, dsp::PadMode::EDGE};
    const char* mnames[] = {"constant", "reflect", "edge"};
    struct Case {
        size_t T, N, H;
    };
    const Case cases[] = {{20, 8, 2},   {5, 8, 2},      {1, 8, 4},      {2, 16, 4},  {3, 16, 16},
                          {0, 8, 2},    {1000, 100, 30}, {3000, 512, 128}, {4100, 1024, 256},
                          {9000, 1024, 512}, {6000, 4096, 1024}, {7, 6, 9}};
    for (const Case& c : cases) {
        std::vector<float> x(c.T);
        for (size_t i = 0; i < c.T; ++i) x[i] = float(i % 1000) / 1024.0f - 0.5f + float(i / 1000);
        for (int center = 0; center < 2; ++center)
            for (int m = 0; m < 3; ++m) {
                if (!center && m > 0) continue;  // padding is never consulted without center
                dsp::FrameQueue fq(c.T ? x.data() : nullptr, c.T, c.N, c.H, center != 0, modes[m]);
                char name[160];
                std::snprintf(name, sizeof name, "fq_t%zu_n%zu_h%zu_c%d_%s", c.T, c.N, c.H, center,
                              mnames[m]);
                dump_u64(std::string(name) + "_meta",
                         {uint64_t(c.T), uint64_t(c.N), uint64_t(c.H), uint64_t(center), uint64_t(m),
                          uint64_t(fq.getNumFrames())});
                dump_f32(std::string(name) + "_x", x.data(), x.size());
                dump_f32(std::string(name) + "_frames", fq.getAllFrames().data(),
                         fq.getAllFrames().size());
            }
    }
}

// The OLA stage's arithmetic (kernels.cc:18-36 scalar kernels, the ones
// kernels_test.cc pins the Highway versions to within 1 ULP), RingBuffer::split
// (ring_buffer.cc:44-85) and deinterleave_to_scratch (aos_to_soa.cc:7-18) on
// seeded data: inputs and outputs, so the oracle's restatements are pinned bit
// for bit to the reference's own compiled code.
static void ola_primitives() {
    std::mt19937 rng(42);  // kernels_test.cc:219
    std::uniform_real_distribution<float> u(-10.0f, 10.0f);
    const size_t sizes[] = {0, 1, 7, 16, 255, 1024, 4097};
    const float gains[] = {1.0f, 0.5f, -1.25f, 3.0e-5f};
    for (size_t n : sizes)
        for (int gi = 0; gi < 4; ++gi) {
            std::vector<float> dst(n), src(n), win(n);
            for (size_t i = 0; i < n; ++i) dst[i] = u(rng), src[i] = u(rng), win[i] = u(rng) * 0.1f;
            char name[96];
            std::snprintf(name, sizeof name, "k_n%zu_g%d", n, gi);
            dump_f32(std::string(name) + "_dst", dst.data(), n);
            dump_f32(std::string(name) + "_src", src.data(), n);
            dump_f32(std::string(name) + "_win", win.data(), n);
            dump_f32(std::string(name) + "_gain", &gains[gi], 1);
            std::vector<float> a = dst, w = dst;
            dsp::axpy_scalar(a.data(), src.data(), gains[gi], n);
            dsp::axpy_windowed_scalar(w.data(), src.data(), win.data(), gains[gi], n);
            dump_f32(std::string(name) + "_axpy", a.data(), n);
            dump_f32(std::string(name) + "_axpyw", w.data(), n);
            // normalize_and_clear: norm around eps (both sides of the guard) and large
            const float eps = gi == 3 ? 1e-8f : 1e-3f;
            std::vector<float> acc = dst, norm(n), out(n);
            for (size_t i = 0; i < n; ++i) {
                const float r = std::fabs(u(rng));
                norm[i] = (i % 3 == 0) ? eps * r * 0.1f : (i % 3 == 1 ? eps * (1.0f + r) : r);
            }
            dump_f32(std::string(name) + "_norm", norm.data(), n);
            dump_f32(std::string(name) + "_eps", &eps, 1);
            dsp::normalize_and_clear_scalar(out.data(), acc.data(), norm.data(), eps, n);
            dump_f32(std::string(name) + "_out", out.data(), n);
            dump_f32(std::string(name) + "_acc", acc.data(), n);
        }
    // RingBuffer::split spans, as (first offset, first len, second offset, second len)
    const size_t caps[] = {1, 8, 100, 6144, 11264};
    std::vector<uint64_t> rows;
    for (size_t cap : caps) {
        dsp::ring::RingBuffer<float> rb(cap);
        const float* base = rb.split(0, 1).first.data();
        const size_t starts[] = {0, 1, cap - 1, cap, cap + 3, 7 * cap + cap / 2, 123457};
        const size_t lens[] = {0, 1, cap / 2, cap - 1, cap, cap + 1, 3 * cap};
        for (size_t s : starts)
            for (size_t l : lens) {
                const auto sp = rb.split(s, l);
                rows.push_back(cap), rows.push_back(s), rows.push_back(l);
                rows.push_back(sp.first.size() ? uint64_t(sp.first.data() - base) : 0);
                rows.push_back(sp.first.size());
                rows.push_back(sp.second.size() ? uint64_t(sp.second.data() - base) : 0);
                rows.push_back(sp.second.size());
            }
    }
    dump_u64("ring_split_rows", rows);
    // deinterleave_to_scratch
    for (size_t c : {1, 2, 3, 5, 16}) {
        const size_t n = 1000 + c;
        std::vector<float> x(n * c), s(n * c, -1.0f);
        for (float& v : x) v = u(rng);
        dsp::ola::deinterleave_to_scratch(x.data(), n, c, s.data());
        char name[64];
        std::snprintf(name, sizeof name, "deint_c%zu", c);
        dump_f32(std::string(name) + "_x", x.data(), x.size());
        dump_f32(std::string(name) + "_s", s.data(), s.size());
    }
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: ref_dump OUTDIR\n");
        return 2;
    }
    g_dir = argv[1];
    g_manifest = std::fopen((g_dir + "/manifest.txt").c_str(), "w");
    if (!g_manifest) return 1;
    windows();
    norms();
    framers();
    framequeues();
    ola_primitives();
    std::fclose(g_manifest);
    return 0;
}
