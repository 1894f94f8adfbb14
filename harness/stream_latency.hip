// stream_latency: per-hop latency of the config-4 streaming path (BASELINE
// config 4: 64 channels, N = 512, H = 128, DROP) measured from C++ so the
// numbers carry no Python overhead, next to the floor of the same launch
// machinery (an empty kernel, and an empty kernel plus the hop copies).
// Usage: stream_latency [hops=3750] [channels=64] [N=512] [H=128]
// Prints one JSON line.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/crlot_dsp.h"

#define HIPCHECK(x)                                                                      \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(2);                                                                \
        }                                                                                \
    } while (0)
#define CRCHECK(x)                                                                         \
    do {                                                                                   \
        int r_ = (x);                                                                      \
        if (r_ != 0) {                                                                     \
            std::fprintf(stderr, "%s:%d rc=%d %s\n", __FILE__, __LINE__, r_, crlot_last_error()); \
            std::exit(3);                                                                  \
        }                                                                                  \
    } while (0)

__global__ void k_empty(float* p) {
    if (p && threadIdx.x == 0 && blockIdx.x == 0xFFFFFFF) p[0] = 1.f;
}

using clk = std::chrono::steady_clock;

// [rows][cols] -> [cols][rows]
static void transpose(const float* src, float* dst, int rows, int cols) {
    for (int r = 0; r < rows; ++r)
        for (int c = 0; c < cols; ++c) dst[size_t(c) * rows + r] = src[size_t(r) * cols + c];
}

struct Stat {
    std::vector<double> v;
    void add(double x) { v.push_back(x); }
    double pct(double q) {
        std::sort(v.begin(), v.end());
        return v.empty() ? 0 : v[std::min(v.size() - 1, size_t(q * (v.size() - 1) + 0.5))];
    }
};

static void print_stat(const char* name, Stat& s, bool last = false) {
    std::printf("\"%s\": {\"p50\": %.2f, \"p99\": %.2f}%s", name, s.pct(0.5), s.pct(0.99), last ? "" : ", ");
}

int main(int argc, char** argv) {
    const int hops = argc > 1 ? std::atoi(argv[1]) : 3750;
    const int C = argc > 2 ? std::atoi(argv[2]) : 64;
    const int N = argc > 3 ? std::atoi(argv[3]) : 512;
    const int H = argc > 4 ? std::atoi(argv[4]) : 128;
    HIPCHECK(hipSetDeviceFlags(hipDeviceScheduleSpin));
    HIPCHECK(hipSetDevice(0));
    hipStream_t s;
    HIPCHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    HIPCHECK(hipEventCreate(&e0));
    HIPCHECK(hipEventCreate(&e1));
    const size_t hop_floats = size_t(C) * H;
    float *d_in, *d_out, *h_in, *h_out;
    HIPCHECK(hipMalloc(&d_in, sizeof(float) * hop_floats * hops));
    HIPCHECK(hipMalloc(&d_out, sizeof(float) * hop_floats));
    HIPCHECK(hipHostMalloc(&h_in, sizeof(float) * hop_floats * hops));
    HIPCHECK(hipHostMalloc(&h_out, sizeof(float) * hop_floats));
    uint32_t r = 12345;
    for (size_t i = 0; i < hop_floats * hops; ++i) {
        r = r * 1664525u + 1013904223u;
        h_in[i] = (float(r >> 8) / 16777216.0f - 0.5f);
    }
    HIPCHECK(hipMemcpy(d_in, h_in, sizeof(float) * hop_floats * hops, hipMemcpyHostToDevice));

    // floor 1: empty kernel, launch + synchronize (wall) and event-to-event (device)
    Stat fw, fd, cw;
    for (int i = 0; i < 200 + hops; ++i) {
        auto t0 = clk::now();
        HIPCHECK(hipEventRecord(e0, s));
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, nullptr);
        HIPCHECK(hipEventRecord(e1, s));
        HIPCHECK(hipStreamSynchronize(s));
        auto t1 = clk::now();
        float ms;
        HIPCHECK(hipEventElapsedTime(&ms, e0, e1));
        if (i >= 200) {
            fw.add(std::chrono::duration<double, std::micro>(t1 - t0).count());
            fd.add(ms * 1e3);
        }
    }
    // floor 2: host hop in -> empty kernel -> host hop out
    for (int i = 0; i < 200 + hops; ++i) {
        const int q = i % hops;
        auto t0 = clk::now();
        HIPCHECK(hipMemcpyAsync(d_in, h_in + q * hop_floats, sizeof(float) * hop_floats, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, nullptr);
        HIPCHECK(hipMemcpyAsync(h_out, d_out, sizeof(float) * hop_floats, hipMemcpyDeviceToHost, s));
        HIPCHECK(hipStreamSynchronize(s));
        auto t1 = clk::now();
        if (i >= 200) cw.add(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    HIPCHECK(hipMemcpy(d_in, h_in, sizeof(float) * hop_floats * hops, hipMemcpyHostToDevice));

    crlot_plan_desc d = {};
    d.window_type = CRLOT_WIN_HANN;
    d.analysis_window = 1;
    d.apply_window_inside = 1;
    d.device = -1;
    d.frame_size = N;
    d.hop_size = H;
    d.boundary_mode = CRLOT_DROP;
    crlot_plan* plan;
    CRCHECK(crlot_plan_create(&d, &plan));
    crlot_stream* st;
    CRCHECK(crlot_stream_create(plan, C, &st));
    CRCHECK(crlot_stream_set_layout(st, 1));
    // device-resident hop buffers (per-hop launch: crlot_stream_push_hop)
    const int64_t nb = N / H;
    std::vector<float> ref(hop_floats * hops, 0.0f);
    Stat dw, dd;
    for (int pass = 0; pass < 2; ++pass) {
        CRCHECK(crlot_stream_reset(st));
        for (int q = 0; q < hops; ++q) {
            int32_t em = 0;
            auto t0 = clk::now();
            HIPCHECK(hipEventRecord(e0, s));
            CRCHECK(crlot_stream_push_hop(st, d_in + q * hop_floats, d_out, &em, s));
            HIPCHECK(hipEventRecord(e1, s));
            HIPCHECK(hipStreamSynchronize(s));
            auto t1 = clk::now();
            float ms;
            HIPCHECK(hipEventElapsedTime(&ms, e0, e1));
            if (pass == 1) {
                dw.add(std::chrono::duration<double, std::micro>(t1 - t0).count());
                dd.add(ms * 1e3);
                if (em) HIPCHECK(hipMemcpy(ref.data() + q * hop_floats, d_out, sizeof(float) * hop_floats,
                                           hipMemcpyDeviceToHost));
            }
        }
    }
    // back to back (no per-hop sync)
    CRCHECK(crlot_stream_reset(st));
    HIPCHECK(hipStreamSynchronize(s));
    auto tb = clk::now();
    for (int q = 0; q < hops; ++q) CRCHECK(crlot_stream_push_hop(st, d_in + q * hop_floats, d_out, nullptr, s));
    HIPCHECK(hipStreamSynchronize(s));
    const double b2b = std::chrono::duration<double>(clk::now() - tb).count();

    // resident kernel, hops in host memory (crlot_stream_rt_push_hop: copy in,
    // doorbell, wait, copy out), then the zero-copy form (caller writes the slot)
    crlot_stream_rt* rt;
    CRCHECK(crlot_stream_rt_create(plan, C, 1, 4, &rt));
    Stat rw, rd, zw;
    std::vector<float> out(hop_floats);
    int64_t mismatches = 0;
    for (int pass = 0; pass < 2; ++pass) {
        CRCHECK(crlot_stream_rt_reset(rt));
        for (int q = 0; q < hops; ++q) {
            int32_t em = 0;
            auto t0 = clk::now();
            CRCHECK(crlot_stream_rt_push_hop(rt, h_in + q * hop_floats, out.data(), &em));
            auto t1 = clk::now();
            double ns = 0;
            CRCHECK(crlot_stream_rt_info(rt, nullptr, &ns, nullptr));
            if (pass == 1) {
                rw.add(std::chrono::duration<double, std::micro>(t1 - t0).count());
                if (em) rd.add(ns * 1e-3);
                if ((em != 0) != (q >= nb - 1)) ++mismatches;
                if (em && std::memcmp(out.data(), ref.data() + q * hop_floats, sizeof(float) * hop_floats))
                    ++mismatches;
            }
        }
    }
    CRCHECK(crlot_stream_rt_reset(rt));
    for (int q = 0; q < hops; ++q) {
        auto t0 = clk::now();
        float* slot = crlot_stream_rt_input_slot(rt);
        if (!slot) CRCHECK(-1);
        transpose(h_in + q * hop_floats, slot, H, C);  // interleaved PCM -> [C][H] slot
        int64_t qi;
        CRCHECK(crlot_stream_rt_submit(rt, &qi));
        const float* o;
        int32_t em;
        CRCHECK(crlot_stream_rt_wait(rt, qi, &o, &em));
        auto t1 = clk::now();
        zw.add(std::chrono::duration<double, std::micro>(t1 - t0).count());
        if (em) {
            transpose(o, out.data(), C, H);
            if (std::memcmp(out.data(), ref.data() + q * hop_floats, sizeof(float) * hop_floats)) ++mismatches;
        }
    }
    // zero-copy with a channel-major caller (no transposes): the path's floor
    Stat cz;
    std::vector<float> xcm(hop_floats * hops);
    for (int q = 0; q < hops; ++q) transpose(h_in + q * hop_floats, xcm.data() + q * hop_floats, H, C);
    CRCHECK(crlot_stream_rt_reset(rt));
    for (int q = 0; q < hops; ++q) {
        auto t0 = clk::now();
        float* slot = crlot_stream_rt_input_slot(rt);
        if (!slot) CRCHECK(-1);
        std::memcpy(slot, xcm.data() + q * hop_floats, sizeof(float) * hop_floats);
        int64_t qi;
        CRCHECK(crlot_stream_rt_submit(rt, &qi));
        const float* o;
        int32_t em;
        CRCHECK(crlot_stream_rt_wait(rt, qi, &o, &em));
        if (em) std::memcpy(out.data(), o, sizeof(float) * hop_floats);
        auto t1 = clk::now();
        cz.add(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    // pipelined: keep `depth` hops in flight, sustained rate
    CRCHECK(crlot_stream_rt_reset(rt));
    auto tp = clk::now();
    for (int q = 0; q < hops; ++q) {
        float* slot = crlot_stream_rt_input_slot(rt);
        if (!slot) CRCHECK(-1);
        transpose(h_in + q * hop_floats, slot, H, C);
        CRCHECK(crlot_stream_rt_submit(rt, nullptr));
    }
    CRCHECK(crlot_stream_rt_wait(rt, hops - 1, nullptr, nullptr));
    const double piped = std::chrono::duration<double>(clk::now() - tp).count();
    double ph[8];
    CRCHECK(crlot_stream_rt_phases(rt, ph));
    crlot_stream_rt_destroy(rt);

    std::printf("{\"config\": \"%d ch, N=%d H=%d DROP, interleaved, %d hops\", ", C, N, H, hops);
    print_stat("empty_kernel_wall_us", fw);
    print_stat("empty_kernel_event_us", fd);
    print_stat("empty_kernel_with_hop_copies_wall_us", cw);
    print_stat("push_hop_device_buffers_wall_us", dw);
    print_stat("push_hop_event_us", dd);
    std::printf("\"back_to_back_us_per_hop\": %.2f, ", b2b / hops * 1e6);
    print_stat("resident_push_hop_host_buffers_wall_us", rw);
    print_stat("resident_device_us", rd);
    print_stat("resident_zero_copy_interleaved_caller_wall_us", zw);
    print_stat("resident_zero_copy_channel_major_wall_us", cz);
    std::printf("\"resident_pipelined_us_per_hop\": %.2f, \"resident_realtime_factor_pipelined\": %.1f, "
                "\"resident_bit_mismatches_vs_push_hop\": %lld}\n",
                piped / hops * 1e6, double(hops) * H / 48000.0 / piped, (long long)mismatches);
    std::fprintf(stderr, "phases_ns_wg0_last_hop: %.0f %.0f %.0f %.0f %.0f %.0f %.0f\n", ph[0], ph[1], ph[2], ph[3],
                 ph[4], ph[5], ph[6]);
    if (mismatches) return 4;
    crlot_stream_destroy(st);
    crlot_plan_destroy(plan);
    return 0;
}
