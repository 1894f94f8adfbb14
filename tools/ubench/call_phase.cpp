// call_phase: where the time of one resident-call request goes (OLA add with
// a speculated produce, as push_frame_AoS + produce(H) issue it; and a bare
// 4 KB forward-sized request).  Built with the call-server sources and
// -DCRLOT_CALL_PHASES (make -C tools/ubench call_phase): the kernel stamps its
// phases (descriptor + input fetched, compute, fences) into host memory.
// Prints host round trip p50 and the device phase p50s (us).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#include "call.h"

using namespace crlot;
static double p50(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main() {
    const int64_t N = 1024, H = 256, R = 6144;
    float *ring, *den;
    if (hipMalloc(&ring, R * 4) || hipMalloc(&den, R * 4)) return 2;
    std::vector<float> ones(R, 2.0f);
    (void)hipMemcpy(den, ones.data(), R * 4, hipMemcpyHostToDevice);
    (void)hipMemset(ring, 0, R * 4);
    CallServer* sv = nullptr;
    if (CallServer::create(0, 0, 8, N + N, N, N, &sv) != CRLOT_OK) return 3;
    std::vector<float> frame(N, 0.25f);
    const double tick = 10e-3;  // us per 100 MHz tick
    for (int mode = 0; mode < 2; ++mode) {
        std::vector<double> rtt, ph[4];
        for (int it = 0; it < 3000; ++it) {
            CallSlot sl;
            if (sv->next_slot(&sl) != CRLOT_OK) return 4;
            const auto t0 = std::chrono::steady_clock::now();
            sv->put(sl.in, frame.data(), size_t(N));
            CallReq r{};
            r.op = kCallOlaAdd;
            r.channels = 1;
            r.win_off = -1;
            r.p1 = den;
            r.p2 = ring;
            r.i[0] = R;
            r.i[1] = (it * H) % R;
            r.i[2] = mode == 0 ? N : 64;  // mode 1: a small add
            r.i[4] = (it * H) % R;
            r.i[5] = H;
            r.f0 = 1.0f;
            r.flags = kCallSpec;
            if (sv->submit(r, sl) != CRLOT_OK) return 5;
            if (sv->wait_spec(sl.index) != CRLOT_OK) return 6;
            rtt.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
            const CallHostCtl* h = sv->host_ctl();
            for (int i = 0; i < 4; ++i) ph[i].push_back(double(__atomic_load_n(&h->ph[i], __ATOMIC_ACQUIRE)) * tick);
            // clear the block, as the produce's commit does
            CallSlot s2;
            if (sv->next_slot(&s2) != CRLOT_OK) return 7;
            CallReq c{};
            c.op = kCallOlaProduce;
            c.flags = kCallClearOnly;
            c.channels = 1;
            c.win_off = -1;
            c.p1 = den;
            c.p2 = ring;
            c.i[0] = R;
            c.i[1] = (it * H) % R;
            c.i[2] = H;
            if (sv->submit(c, s2) != CRLOT_OK || sv->wait(s2.index) != CRLOT_OK) return 8;
        }
        std::printf("{\"add_len\": %d, \"host_rtt_us_p50\": %.2f, \"dev_compute_us\": %.2f, \"dev_spec_end_us\": "
                    "%.2f, \"dev_fence_end_us\": %.2f}\n",
                    mode == 0 ? 1024 : 64, p50(rtt), p50(ph[0]), p50(ph[2]), p50(ph[3]));
    }
    delete sv;

    // the shared E = 8 server (N = 1024): a forward real FFT with its speculated
    // inverse, as IFftPlan::forward issues it
    int rc = 0;
    SharedServer* sh = shared_server(0, 8, &rc);
    if (!sh) return 9;
    CallServer* fs = sh->srv;
    std::vector<float> x(N);
    for (int64_t i = 0; i < N; ++i) x[size_t(i)] = float((i * 37) % 101) / 101.0f - 0.5f;
    std::vector<double> rtt, rtt_spec, ph[4];
    for (int it = 0; it < 3000; ++it) {
        CallSlot sl;
        if (fs->next_slot(&sl) != CRLOT_OK) return 10;
        const auto t0 = std::chrono::steady_clock::now();
        fs->put(sl.in, x.data(), size_t(N));
        CallReq r{};
        r.op = kCallRfft;
        r.batch = 1;
        r.win_off = -1;
        r.p0 = sh->d_tw;
        r.p1 = sh->d_st;
        r.f0 = 1.0f / float(N);
        r.flags = kCallSpec;
        if (fs->submit(r, sl) != CRLOT_OK || fs->wait(sl.index) != CRLOT_OK) return 11;
        const auto t1 = std::chrono::steady_clock::now();
        if (fs->wait_spec(sl.index) != CRLOT_OK) return 12;
        const auto t2 = std::chrono::steady_clock::now();
        rtt.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        rtt_spec.push_back(std::chrono::duration<double, std::micro>(t2 - t0).count());
        const CallHostCtl* h = fs->host_ctl();
        for (int i = 0; i < 4; ++i) ph[i].push_back(double(__atomic_load_n(&h->ph[i], __ATOMIC_ACQUIRE)) * tick);
    }
    std::printf("{\"rfft1024_spec\": {\"host_done_us_p50\": %.2f, \"host_spec_us_p50\": %.2f, \"dev_compute_us\": %.2f, "
                "\"dev_fence_end_us\": %.2f, \"dev_spec_end_us\": %.2f, \"dev_spec_fence_end_us\": %.2f}}\n",
                p50(rtt), p50(rtt_spec), p50(ph[0]), p50(ph[1]), p50(ph[2]), p50(ph[3]));
    return 0;
}
