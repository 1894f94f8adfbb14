// call.cpp -- host side of K_call (call_rt.hip): the resident server that runs
// the reference's host-pointer calls one at a time (IFftPlan::forward /
// inverse, OLAAccumulator add / push / produce, dsp::axpy / axpy_windowed /
// normalize_and_clear) without a kernel launch or a copy-engine transfer per
// call.
//
// Memory: a fine-grained DEVICE block [CallCtl][depth descriptors][input
// arena] that the host writes through the BAR (write-combined stores, then an
// sfence before and after the doorbell), and a pinned HOST block
// [CallHostCtl][output arena][speculation arena] that the kernel writes.  Request q uses
// slot q % depth of each arena; a slot is reused only after request q - depth
// (and its speculation) completed.  If the device block cannot be allocated
// host-visible, the input side falls back to pinned host memory (the kernel's
// system-scope loads read either).
#include "call.h"
#include "ab.h"

#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <vector>

namespace crlot {
int set_error(int code, const std::string& msg);  // abi.cpp

namespace {
int fail(int code, const std::string& msg) { return set_error(code, msg); }
int hip_fail(hipError_t e, const char* what) { return fail(CRLOT_EHIP, std::string(what) + ": " + hipGetErrorString(e)); }

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (dev >= 0 && dev != prev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// write-combined copy into BAR-mapped device memory: 16-byte streaming stores
// (dst 16-byte aligned), scalar tail
void copy_wc(float* dst, const float* src, size_t n) {
    size_t i = 0;
    if ((reinterpret_cast<uintptr_t>(dst) & 15u) == 0) {
        for (; i + 4 <= n; i += 4)
            _mm_stream_ps(dst + i, _mm_loadu_ps(src + i));
    }
    for (; i < n; ++i) dst[i] = src[i];
}

inline uint64_t load_acq(const uint64_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }

constexpr size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }
}  // namespace

CallServer::~CallServer() { release(); }

void CallServer::release() {
    DeviceGuard g(device_);
    (void)stop();
    if (dblk_) (void)hipFree(dblk_);
    if (dhost_) (void)hipHostFree(dhost_);
    if (hblk_) (void)hipHostFree(hblk_);
    dblk_ = nullptr;
    dhost_ = nullptr;
    hblk_ = nullptr;
    if (ev_) (void)hipEventDestroy(ev_);
    if (s_) (void)hipStreamDestroy(s_);
    ev_ = nullptr;
    s_ = nullptr;
}

int CallServer::create(int device, int e, int depth, size_t in_cap, size_t out_cap, size_t spec_cap,
                       CallServer** out) {
    *out = nullptr;
    if (call_lds_bytes(e) == 0) return fail(CRLOT_EUNSUPPORTED, "call server: no instantiation for this size");
    CallServer* sv = new CallServer();
    sv->device_ = device;
    sv->e_ = e;
    sv->depth_ = depth;
    DeviceGuard g(device);
    hipError_t err;
    if ((err = hipStreamCreateWithFlags(&sv->s_, hipStreamNonBlocking)) ||
        (err = hipEventCreateWithFlags(&sv->ev_, hipEventDisableTiming))) {
        delete sv;
        return hip_fail(err, "call server stream");
    }
    int khz = 100000;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || khz <= 0) khz = 100000;
    sv->tick_ns_ = 1e6 / double(khz);
    sv->idle_ticks_ = uint64_t(20.0e6 / sv->tick_ns_);  // 20 ms without a call
    const int rc = sv->alloc(in_cap, out_cap, spec_cap);
    if (rc != CRLOT_OK) {
        delete sv;
        return rc;
    }
    *out = sv;
    return CRLOT_OK;
}

int CallServer::alloc(size_t in_cap, size_t out_cap, size_t spec_cap) {
    // >= 1024 floats: the kernel fetches the first 4 KB of a slot with its descriptor
    ++gen_;
    in_cap_ = align_up(std::max<size_t>(in_cap, 1024), 32);
    out_cap_ = align_up(std::max<size_t>(out_cap, 64), 32);
    spec_cap_ = align_up(spec_cap, 32);
    const size_t dbytes = sizeof(CallCtl) + sizeof(CallReq) * size_t(depth_) + sizeof(float) * in_cap_ * depth_;
    const size_t hbytes =
        sizeof(CallHostCtl) + sizeof(float) * (out_cap_ + spec_cap_) * size_t(depth_);
    hipError_t err;
    const unsigned fl = hipHostMallocCoherent | hipHostMallocMapped;
    static const bool host_inputs = [] {
        const char* v = ab_env("CRLOT_CALL_HOST_INPUTS");  // A/B: inputs in pinned host memory
        return v && v[0] == '1';
    }();
    void* d = nullptr;
    if (!host_inputs && hipExtMallocWithFlags(&d, dbytes, hipDeviceMallocFinegrained) == hipSuccess) {
        dblk_ = static_cast<char*>(d);
        wc_inputs_ = true;
        ddev_ = dblk_;
    } else {
        if ((err = hipHostMalloc(reinterpret_cast<void**>(&dhost_), dbytes, fl)) != hipSuccess)
            return hip_fail(err, "call server input block");
        void* dp = nullptr;
        if ((err = hipHostGetDevicePointer(&dp, dhost_, 0)) != hipSuccess) return hip_fail(err, "call server map");
        ddev_ = static_cast<char*>(dp);
        wc_inputs_ = false;
    }
    char* hin = dblk_ ? dblk_ : dhost_;  // host view of the input block
    if ((err = hipHostMalloc(reinterpret_cast<void**>(&hblk_), hbytes, fl)) != hipSuccess)
        return hip_fail(err, "call server output block");
    void* hdp = nullptr;
    if ((err = hipHostGetDevicePointer(&hdp, hblk_, 0)) != hipSuccess) return hip_fail(err, "call server map");
    hctl_dev_ = static_cast<char*>(hdp);
    ctl_ = reinterpret_cast<CallCtl*>(hin);
    reqs_ = reinterpret_cast<CallReq*>(hin + sizeof(CallCtl));
    in_ = reinterpret_cast<float*>(hin + sizeof(CallCtl) + sizeof(CallReq) * size_t(depth_));
    hctl_ = reinterpret_cast<CallHostCtl*>(hblk_);
    out_ = reinterpret_cast<float*>(hblk_ + sizeof(CallHostCtl));
    std::memset(hblk_, 0, sizeof(CallHostCtl));
    CallCtl zero{};
    copy_wc(reinterpret_cast<float*>(ctl_), reinterpret_cast<const float*>(&zero), sizeof(CallCtl) / 4);
    _mm_sfence();
    q_ = 0;
    spec_req_.assign(size_t(depth_), 0);
    slot_rings_.assign(2 * size_t(depth_), nullptr);
    return CRLOT_OK;
}

int CallServer::grow(size_t in_cap, size_t out_cap, size_t spec_cap) {
    if (in_cap <= in_cap_ && out_cap <= out_cap_ && spec_cap <= spec_cap_) return CRLOT_OK;
    DeviceGuard g(device_);
    int rc = drain();
    if (rc == CRLOT_OK) rc = stop();
    if (rc != CRLOT_OK) return rc;
    if (dblk_) (void)hipFree(dblk_);
    if (dhost_) (void)hipHostFree(dhost_);
    if (hblk_) (void)hipHostFree(hblk_);
    dblk_ = dhost_ = hblk_ = nullptr;
    // request numbers stay monotonic across the reallocation (a speculation
    // recorded before it can never match a later request)
    const uint64_t q = q_;
    rc = alloc(std::max(in_cap, in_cap_), std::max(out_cap, out_cap_), std::max(spec_cap, spec_cap_));
    if (rc != CRLOT_OK) return rc;
    q_ = q;
    hctl_->done = hctl_->spec_done = hctl_->chain_done = hctl_->ring_done = q;
    store_ctl(&ctl_->seq, q);
    return CRLOT_OK;
}

bool CallServer::running() { return launched_ && hipEventQuery(ev_) == hipErrorNotReady; }

int CallServer::launch() {
    CallArgs a;
    a.ctl = reinterpret_cast<CallCtl*>(ddev_);
    a.hctl = reinterpret_cast<CallHostCtl*>(hctl_dev_);
    a.reqs = reinterpret_cast<const CallReq*>(ddev_ + sizeof(CallCtl));
    a.in_arena = reinterpret_cast<const float*>(ddev_ + sizeof(CallCtl) + sizeof(CallReq) * size_t(depth_));
    a.out_arena = reinterpret_cast<float*>(hctl_dev_ + sizeof(CallHostCtl));
    a.depth = depth_;
    a.in_cap = int64_t(in_cap_);
    a.first = load_acq(&hctl_->done);
    a.idle_ticks = idle_ticks_;
    store_ctl(&ctl_->stop, 0);
    hipError_t e = launch_call(e_, a, s_);
    if (e == hipSuccess) e = hipEventRecord(ev_, s_);
    if (e != hipSuccess) return hip_fail(e, "call server launch");
    launched_ = true;
    return CRLOT_OK;
}

void CallServer::store_ctl(uint64_t* p, uint64_t v) {
    if (wc_inputs_) {
        _mm_sfence();
        *reinterpret_cast<volatile uint64_t*>(p) = v;
        _mm_sfence();  // out of the write-combining buffer now
    } else {
        __atomic_store_n(p, v, __ATOMIC_RELEASE);
    }
}

int CallServer::stop() {
    if (!launched_) return CRLOT_OK;
    store_ctl(&ctl_->stop, 1);
    hipError_t e = hipStreamSynchronize(s_);
    launched_ = false;
    return e == hipSuccess ? CRLOT_OK : hip_fail(e, "call server");
}

namespace {
// crlot_test_inject(CRLOT_INJECT_CALL_TIMEOUT, k): the next k waits take the
// timeout path at their first check (the request itself completes normally)
std::atomic<int> g_timeout_inject{0};
}  // namespace
bool test_timeout_now() {
    int v = g_timeout_inject.load(std::memory_order_relaxed);
    while (v > 0)
        if (g_timeout_inject.compare_exchange_weak(v, v - 1, std::memory_order_relaxed)) return true;
    return false;
}
void test_inject_timeouts(int count) { g_timeout_inject.store(count, std::memory_order_relaxed); }

int CallServer::wait_counter(const uint64_t* ctr, uint64_t target) {
    if (test_timeout_now()) {  // (test-only: the timeout path below, taken at once)
        timed_out(std::min(done(), target - 1));
        return fail(CRLOT_EHIP, "call server: request timed out (server paused)");
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0;; ++spin) {
        if (load_acq(ctr) >= target) return CRLOT_OK;
        if ((spin & 1023) == 1023) {
            if (!running()) {
                if (launched_) {
                    hipError_t e = hipEventSynchronize(ev_);
                    if (e != hipSuccess) return hip_fail(e, "call server");
                    launched_ = false;
                }
                if (load_acq(ctr) >= target) return CRLOT_OK;
                // exited idle just as the request arrived: relaunch (it resumes at done)
                int rc = launch();
                if (rc != CRLOT_OK) return rc;
            }
            const auto us =
                std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
            if (us > 5000000) {
                // the request is still in flight in the resident kernel: no later call
                // may read a slot or speculation it could still write -- until every
                // request submitted so far has completed (submit re-checks)
                timed_out(load_acq(ctr) < target ? std::min(done(), target - 1) : done());
                return fail(CRLOT_EHIP, "call server: request timed out (server paused)");
            }
        }
        _mm_pause();
    }
}

// A request timed out while still in flight: pause the server until every
// request submitted so far has completed.  The OLA rings those requests change
// (an add / produce, a chained produce, deferred push / clear work) are
// poisoned: the host's bookkeeping of their objects no longer matches what the
// device does (a produce that failed here still clears its slots there), so
// those objects' calls fail loudly until reset() instead of reading a ring the
// host cannot account for.  Stateless requests (FFTs) resume.
void CallServer::timed_out(uint64_t done_seen) {
    broken_ = true;
    broken_at_ = q_;
    // requests (done_seen, q_] are in flight, at most depth_ of them (next_slot), so
    // each still owns its slot's record
    for (uint64_t i = done_seen + 1; i <= q_; ++i) {
        const size_t k = size_t((i - 1) % uint64_t(depth_));
        for (int j = 0; j < 2; ++j) {
            const float* r = slot_rings_[2 * k + size_t(j)];
            if (r && !poisoned(r) && ola_ring_live(r)) poisoned_.push_back(r);
        }
    }
}

bool CallServer::poisoned(const float* ring) const {
    return std::find(poisoned_.begin(), poisoned_.end(), ring) != poisoned_.end();
}

void CallServer::unpoison(const float* ring) {
    poisoned_.erase(std::remove(poisoned_.begin(), poisoned_.end(), ring), poisoned_.end());
}

int CallServer::defer(const CallReq::Pend& p) {
    const bool merge = pend_.flags == 0 ||
                       (p.flags == kPendClear && pend_.flags == kPendCommit && pend_.ring == p.ring && pend_.R == p.R);
    if (!merge) {
        int rc = flush();
        if (rc != CRLOT_OK) return rc;
    }
    if (pend_.flags == 0) {
        pend_ = p;
    } else {  // a clear behind the pending commit of the same ring
        pend_.flags |= kPendClear;
        pend_.rp = p.rp;
        pend_.n = p.n;
    }
    return CRLOT_OK;
}

int CallServer::flush() {
    if (pend_.flags == 0) return CRLOT_OK;
    CallSlot sl;
    int rc = next_slot(&sl);
    if (rc != CRLOT_OK) return rc;
    CallReq r{};
    r.op = 0;
    r.win_off = -1;
    return submit(r, sl);  // carries pend_
}

int CallServer::drain() {
    int rc = flush();
    if (rc != CRLOT_OK) return rc;
    if (q_ == 0) return CRLOT_OK;
    if ((rc = wait_counter(&hctl_->done, q_)) != CRLOT_OK) return rc;
    if (last_chain_ && (rc = wait_counter(&hctl_->chain_done, last_chain_)) != CRLOT_OK) return rc;
    if (last_late_ && (rc = wait_counter(&hctl_->ring_done, last_late_)) != CRLOT_OK) return rc;
    for (int i = 0; i < depth_; ++i)
        if (spec_req_[size_t(i)]) {
            rc = wait_counter(&hctl_->spec_done, spec_req_[size_t(i)]);
            if (rc != CRLOT_OK) return rc;
        }
    return CRLOT_OK;
}

int CallServer::next_slot(CallSlot* sl) {
    // slot q % depth was last used by request q - depth + 1 (1-based): wait for it
    const int k = int(q_ % uint64_t(depth_));
    if (q_ >= uint64_t(depth_)) {
        int rc = wait_counter(&hctl_->done, q_ - uint64_t(depth_) + 1);
        if (rc != CRLOT_OK) return rc;
    }
    if (spec_req_[size_t(k)]) {
        int rc = wait_counter(&hctl_->spec_done, spec_req_[size_t(k)]);
        if (rc != CRLOT_OK) return rc;
        spec_req_[size_t(k)] = 0;
    }
    sl->index = q_ + 1;
    sl->gen = gen_;
    sl->in = in_ + size_t(k) * in_cap_;
    sl->out = out_ + size_t(k) * out_cap_;
    sl->spec = out_ + size_t(depth_) * out_cap_ + size_t(k) * spec_cap_;
    sl->in_off = int64_t(size_t(k) * in_cap_);
    sl->out_off = int64_t(size_t(k) * out_cap_);
    sl->spec_off = int64_t(size_t(depth_) * out_cap_ + size_t(k) * spec_cap_);
    return CRLOT_OK;
}

void CallServer::put(float* dst, const float* src, size_t n) {
    if (wc_inputs_)
        copy_wc(dst, src, n);
    else
        std::memcpy(dst, src, sizeof(float) * n);
}

int CallServer::submit(CallReq& r, const CallSlot& sl) {
    if (broken_) {  // a timed-out request: serve again once everything submitted has completed
        if (done() < broken_at_) return fail(CRLOT_EHIP, "call server: a timed-out request is still in flight");
        broken_ = false;
        acquire_next_ = true;  // (the kernel's view of host memory is refreshed with the next request)
    }
    r.in_off = sl.in_off;
    r.out_off = sl.out_off;
    r.spec_off = sl.spec_off;
    if (acquire_next_) {
        r.flags |= kCallAcquire;
        acquire_next_ = false;
    }
    r.pend = pend_;
    pend_ = CallReq::Pend{};
    if (r.flags & kCallChain) last_chain_ = q_ + 1;
    if (r.flags & kCallPendLate) last_late_ = q_ + 1;
    const int k = int(q_ % uint64_t(depth_));
    const bool ring_op = r.op == kCallOlaAdd || r.op == kCallOlaProduce || (r.flags & (kCallChain | kCallPendLate));
    slot_rings_[2 * size_t(k)] = ring_op ? r.p2 : nullptr;
    slot_rings_[2 * size_t(k) + 1] = r.pend.flags != 0 ? r.pend.ring : nullptr;
    if (wc_inputs_)
        copy_wc(reinterpret_cast<float*>(reqs_ + k), reinterpret_cast<const float*>(&r), sizeof(CallReq) / 4);
    else
        std::memcpy(reqs_ + k, &r, sizeof(CallReq));
    spec_req_[size_t(k)] = (r.flags & kCallSpec) ? q_ + 1 : 0;
    q_ += 1;
    store_ctl(&ctl_->seq, q_);  // sfence: payload and descriptor land before the doorbell
    if (!running()) {
        if (launched_) {
            hipError_t e = hipEventSynchronize(ev_);
            if (e != hipSuccess) return hip_fail(e, "call server");
            launched_ = false;
        }
        return launch();
    }
    return CRLOT_OK;
}

int CallServer::wait(uint64_t index) { return wait_counter(&hctl_->done, index); }
int CallServer::wait_spec(uint64_t index) { return wait_counter(&hctl_->spec_done, index); }
int CallServer::wait_chain(uint64_t index) { return wait_counter(&hctl_->chain_done, index); }

// ------------------------------------------------------------------ shared servers
// One E = 0 server per device for the free functions (dsp::axpy & co).
namespace {
std::mutex g_free_mu;
CallServer* g_free[64] = {};
}  // namespace

CallServer* free_function_server(int device, int* rc) {
    if (device < 0 || device >= 64) {
        *rc = fail(CRLOT_EINVAL, "device ordinal");
        return nullptr;
    }
    if (!g_free[device]) {
        CallServer* s = nullptr;
        *rc = CallServer::create(device, 0, 4, 3 * 4096, 2 * 4096, 0, &s);
        if (*rc != CRLOT_OK) return nullptr;
        static const bool hooked = [] { return std::atexit(stop_free_function_servers) == 0; }();
        (void)hooked;
        g_free[device] = s;
    }
    *rc = CRLOT_OK;
    return g_free[device];
}
std::mutex& free_function_mutex() { return g_free_mu; }

void stop_free_function_servers() {
    for (CallServer* s : g_free)
        if (s) (void)s->stop();
}

namespace {
std::mutex g_shared_mu;
SharedServer* g_shared[64][6] = {};  // [device][log2(E / 2)]

std::map<std::pair<int, int>, SharedServer*> g_shared_any;  // (device, P): any-size FFT servers

void stop_shared_servers() {
    for (auto& row : g_shared)
        for (SharedServer* s : row)
            if (s && s->srv) (void)s->srv->stop();
    for (auto& kv : g_shared_any)
        if (kv.second && kv.second->srv) (void)kv.second->srv->stop();
}
}  // namespace

namespace {
SharedServer* shared_server_any(int device, int P, int* rc) {
    std::lock_guard<std::mutex> lk(g_shared_mu);
    auto it = g_shared_any.find({device, P});
    if (it != g_shared_any.end() && it->second) {  // (every call after the first: no table work)
        *rc = CRLOT_OK;
        return it->second;
    }
    const int waves = call_any_waves(P);
    if (device < 0 || device >= 64 || waves == 0 || !any_supported(P)) {
        *rc = fail(CRLOT_EUNSUPPORTED, "call server slot");
        return nullptr;
    }
    SharedServer*& s = g_shared_any[{device, P}];
    if (!s) {
        static const bool hooked = [] { return std::atexit(stop_shared_servers) == 0; }();
        (void)hooked;
        DeviceGuard g(device);
        SharedServer* n = new SharedServer();
        n->e = -P;
        n->any_waves = waves;
        n->any_two = call_any_two(P);
        const std::vector<float> tw = build_any_twiddles(P);
        const std::vector<uint8_t> plan = build_any_plan_blob(P);
        std::vector<float> st(2 * size_t(P));
        for (int t = 0; t < P; ++t) {  // exp(-i pi (t/P + 1/2)), as crlot_plan_create
            const double ps = -M_PI * (double(t) / double(P) + 0.5);
            st[2 * size_t(t)] = float(std::cos(ps));
            st[2 * size_t(t) + 1] = float(std::sin(ps));
        }
        hipError_t err;
        if ((err = hipMalloc(&n->d_tw, sizeof(float) * tw.size())) ||
            (err = hipMalloc(&n->d_st, sizeof(float) * st.size())) ||
            (err = hipMalloc(&n->d_plan, plan.size())) ||
            (err = hipMemcpy(n->d_tw, tw.data(), sizeof(float) * tw.size(), hipMemcpyHostToDevice)) ||
            (err = hipMemcpy(n->d_st, st.data(), sizeof(float) * st.size(), hipMemcpyHostToDevice)) ||
            (err = hipMemcpy(n->d_plan, plan.data(), plan.size(), hipMemcpyHostToDevice))) {
            *rc = hip_fail(err, "call server tables");
            return nullptr;
        }
        const size_t row = size_t(2 * P + 2) * 2;
        *rc = CallServer::create(device, -P, 8, 4 * row, 4 * row, 4 * row, &n->srv);
        if (*rc != CRLOT_OK) return nullptr;
        s = n;
    }
    *rc = CRLOT_OK;
    return s;
}
}  // namespace

SharedServer* shared_server(int device, int e, int* rc) {
    if (e < 0) return shared_server_any(device, -e, rc);
    int lg = 0;
    while ((2 << lg) < e) ++lg;  // e = 2, 4, ..., 32 -> 0..4
    if (device < 0 || device >= 64 || lg > 5 || (2 << lg) != e) {
        *rc = fail(CRLOT_EUNSUPPORTED, "call server slot");
        return nullptr;
    }
    std::lock_guard<std::mutex> lk(g_shared_mu);
    SharedServer*& s = g_shared[device][lg];
    if (!s) {
        static const bool hooked = [] { return std::atexit(stop_shared_servers) == 0; }();
        (void)hooked;
        DeviceGuard g(device);
        SharedServer* n = new SharedServer();
        n->e = e;
        const int P = 64 * e;
        const std::vector<float> tw = build_pass_twiddles(2 * P);
        std::vector<float> st(2 * size_t(P));
        for (int t = 0; t < P; ++t) {  // exp(-i pi (t/P + 1/2)), as crlot_plan_create
            const double ps = -M_PI * (double(t) / double(P) + 0.5);
            st[2 * size_t(t)] = float(std::cos(ps));
            st[2 * size_t(t) + 1] = float(std::sin(ps));
        }
        hipError_t err;
        if ((err = hipMalloc(&n->d_tw, sizeof(float) * tw.size())) ||
            (err = hipMalloc(&n->d_st, sizeof(float) * st.size())) ||
            (err = hipMemcpy(n->d_tw, tw.data(), sizeof(float) * tw.size(), hipMemcpyHostToDevice)) ||
            (err = hipMemcpy(n->d_st, st.data(), sizeof(float) * st.size(), hipMemcpyHostToDevice))) {
            *rc = hip_fail(err, "call server tables");
            return nullptr;
        }
        const size_t row = size_t(2 * P + 2) * 2;
        *rc = CallServer::create(device, e, 8, 4 * row, 4 * row, 4 * row, &n->srv);
        if (*rc != CRLOT_OK) return nullptr;
        s = n;
    }
    *rc = CRLOT_OK;
    return s;
}

}  // namespace crlot

// ------------------------------------------------------------------ free functions (host pointers)
extern "C" {

static int free_call(uint32_t op, float* dst, float* dst2, const float* a, const float* b, const float* c, float f,
                     int64_t n) {
    using namespace crlot;
    if (n < 0) return fail(CRLOT_EINVAL, "negative size");
    if (n == 0) return CRLOT_OK;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return fail(CRLOT_EHIP, "no HIP device");
    std::lock_guard<std::mutex> lk(free_function_mutex());
    int rc = CRLOT_OK;
    CallServer* sv = free_function_server(dev, &rc);
    if (!sv) return rc;
    const int nin = c ? 3 : 2, nout = dst2 ? 2 : 1;
    if ((rc = sv->grow(size_t(nin) * size_t(n), size_t(nout) * size_t(n), 0)) != CRLOT_OK) return rc;
    CallSlot sl;
    if ((rc = sv->next_slot(&sl)) != CRLOT_OK) return rc;
    sv->put(sl.in, a, size_t(n));
    sv->put(sl.in + n, b, size_t(n));
    if (c) sv->put(sl.in + 2 * n, c, size_t(n));
    CallReq r{};
    r.op = op;
    r.win_off = -1;
    r.i[0] = n;
    r.f0 = f;
    if ((rc = sv->submit(r, sl)) != CRLOT_OK) return rc;
    if ((rc = sv->wait(sl.index)) != CRLOT_OK) return rc;
    std::memcpy(dst, sl.out, sizeof(float) * size_t(n));
    if (dst2) std::memcpy(dst2, sl.out + n, sizeof(float) * size_t(n));
    return CRLOT_OK;
}

int crlot_call_axpy(float* dst, const float* src, float g, int64_t n) {
    if (n > 0 && (!dst || !src)) return crlot::fail(CRLOT_EINVAL, "null buffer");
    return free_call(crlot::kCallAxpy, dst, nullptr, dst, src, nullptr, g, n);
}

int crlot_call_axpy_windowed(float* dst, const float* src, const float* win, float g, int64_t n) {
    if (n > 0 && (!dst || !src || !win)) return crlot::fail(CRLOT_EINVAL, "null buffer");
    return free_call(crlot::kCallAxpyWin, dst, nullptr, dst, src, win, g, n);
}

int crlot_call_normalize_and_clear(float* out, float* acc, const float* norm, float eps, int64_t n) {
    if (n > 0 && (!out || !acc || !norm)) return crlot::fail(CRLOT_EINVAL, "null buffer");
    return free_call(crlot::kCallNormalize, out, acc, acc, norm, nullptr, eps, n);
}

}  // extern "C"
