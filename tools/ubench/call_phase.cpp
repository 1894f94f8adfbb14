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
    // the any-size server (K_call<-1>, fft_any.h passes): the same request at 20 ms frames
    for (int n : {960, 882, 1920}) {
        SharedServer* sa = shared_server(0, -(n / 2), &rc);
        if (!sa) return 13;
        CallServer* as = sa->srv;
        std::vector<float> xa(static_cast<size_t>(n));
        for (int i = 0; i < n; ++i) xa[size_t(i)] = float((i * 37) % 101) / 101.0f - 0.5f;
        std::vector<double> ra, rs, pa[4];
        for (int it = 0; it < 2000; ++it) {
            CallSlot sl;
            if (as->next_slot(&sl) != CRLOT_OK) return 14;
            const auto t0 = std::chrono::steady_clock::now();
            as->put(sl.in, xa.data(), size_t(n));
            CallReq r{};
            r.op = kCallRfft;
            r.batch = 1;
            r.win_off = -1;
            r.p0 = sa->d_tw;
            r.p1 = sa->d_st;
            r.p5 = sa->d_plan;
            r.f0 = 1.0f / float(n);
            r.flags = kCallSpec;
            if (as->submit(r, sl) != CRLOT_OK || as->wait(sl.index) != CRLOT_OK) return 15;
            const auto t1 = std::chrono::steady_clock::now();
            if (as->wait_spec(sl.index) != CRLOT_OK) return 16;
            const auto t2 = std::chrono::steady_clock::now();
            ra.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
            rs.push_back(std::chrono::duration<double, std::micro>(t2 - t0).count());
            const CallHostCtl* h = as->host_ctl();
            for (int i = 0; i < 4; ++i) pa[i].push_back(double(__atomic_load_n(&h->ph[i], __ATOMIC_ACQUIRE)) * tick);
        }
        std::printf("{\"rfft%d_any_spec\": {\"host_done_us_p50\": %.2f, \"host_spec_us_p50\": %.2f, "
                    "\"dev_compute_us\": %.2f, \"dev_fence_end_us\": %.2f, \"dev_spec_end_us\": %.2f, "
                    "\"dev_spec_fence_end_us\": %.2f}}\n",
                    n, p50(ra), p50(rs), p50(pa[0]), p50(pa[1]), p50(pa[2]), p50(pa[3]));
    }
    // the e2e loop's rhythm on the any-size server: a chained forward (spec inverse
    // + the produce block of pushing it), the push and the produce's clear deferred
    // onto the next forward
    for (int cfg = 0; cfg < 4; ++cfg) {
        const int n = cfg & 1 ? 1024 : 960;
        const bool use_win = cfg >= 2;
        const int e = n == 1024 ? 8 : -(n / 2);
        SharedServer* sa = shared_server(0, e, &rc);
        if (!sa) return 17;
        CallServer* as = sa->srv;
        const int64_t Hh = n / 4, Rr = int64_t(n) * 6;
        float *rg, *dn, *wn;
        if (hipMalloc(&rg, Rr * 4) || hipMalloc(&dn, Rr * 4) || hipMalloc(&wn, n * 4)) return 18;
        (void)hipMemcpy(wn, std::vector<float>(size_t(n), 0.5f).data(), n * 4, hipMemcpyHostToDevice);
        std::vector<float> two(size_t(Rr), 2.0f);
        (void)hipMemcpy(dn, two.data(), Rr * 4, hipMemcpyHostToDevice);
        (void)hipMemset(rg, 0, Rr * 4);
        std::vector<float> xa(static_cast<size_t>(n));
        for (int i = 0; i < n; ++i) xa[size_t(i)] = float((i * 37) % 101) / 101.0f - 0.5f;
        if (as->grow(size_t(n), size_t(n) + 2, size_t(n) + size_t(Hh)) != CRLOT_OK) return 19;
        std::vector<double> ra, pa[6];
        for (int it = 0; it < 2000; ++it) {
            CallSlot sl;
            if (as->next_slot(&sl) != CRLOT_OK) return 20;
            const auto t0 = std::chrono::steady_clock::now();
            as->put(sl.in, xa.data(), size_t(n));
            CallReq r{};
            r.op = kCallRfft;
            r.batch = 1;
            r.win_off = -1;
            r.p0 = sa->d_tw;
            r.p1 = sa->d_st;
            r.p5 = sa->d_plan;
            r.f0 = 1.0f / float(n);
            r.flags = kCallSpec | kCallChain;
            r.p2 = rg;
            r.p3 = dn;
            r.p4 = use_win ? wn : nullptr;
            r.j[0] = Rr;
            r.j[1] = (int64_t(it) * Hh) % Rr;
            r.j[2] = (int64_t(it) * Hh) % Rr;
            r.j[3] = Hh;
            r.f1 = 1.0f;
            if (as->submit(r, sl) != CRLOT_OK || as->wait(sl.index) != CRLOT_OK) return 21;
            ra.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
            const CallHostCtl* h = as->host_ctl();
            for (int i = 0; i < 6; ++i) pa[i].push_back(double(__atomic_load_n(&h->ph[i < 4 ? i : i], __ATOMIC_ACQUIRE)) * tick);
            if (as->wait_chain(sl.index) != CRLOT_OK) return 22;
            CallReq::Pend pe{};
            pe.flags = kPendCommit | kPendClear;
            pe.ring = rg;
            pe.win = use_win ? wn : nullptr;
            pe.R = Rr;
            pe.start = r.j[1];
            pe.len = n;
            pe.gain = 1.0f;
            pe.rp = r.j[2];
            pe.n = Hh;
            pe.src_index = sl.index;     // the frame this request kept in LDS (the e2e loop's case)
            pe.src_off = sl.spec_off;
            if (as->defer(pe) != CRLOT_OK) return 23;
        }
        std::printf("{\"chained_rfft%d\": {\"window\": %d, \"host_done_us_p50\": %.2f, \"dev_pend_end_us\": %.2f, "
                    "\"dev_compute_end_us\": %.2f, \"dev_fence_end_us\": %.2f}}\n",
                    n, int(use_win), p50(ra), p50(pa[4]), p50(pa[0]), p50(pa[1]));
        (void)as->drain();
    }
    return 0;
}
