// objects.cpp -- the reference's two stateful host objects on the hot path, as C ABI:
//
//   crlot_framer_*  dsp::Framer (framer.h:26-127, framer.cc:15-181): interleaved
//                   PCM in, N*C-sample frames out every H samples; ZERO_PAD / DROP.
//                   Pure host bookkeeping + copies (the batched engine frames on
//                   the device instead: crlot_roundtrip's load stage).
//   crlot_ola_*     dsp::OLAAccumulator (OLAAccumulator.h:15-217, .cc:13-295)
//                   backed by device state: the per-channel rings and the COLA
//                   divisors live in HBM and every add/produce is a kernel
//                   (ola.hip); the host keeps the reference's counters
//                   (read_pos_, produced_, flushing_) so the call sequence
//                   behaves exactly as the reference's, quirks included.
//
// Errors follow the reference's exceptions: std::invalid_argument ->
// CRLOT_EINVAL with the reference's message (the C++ layer rethrows it).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <type_traits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>
#include <new>
#include <string>
#include <vector>

#include <mutex>

#include "batch.h"
#include "call.h"
#include "respool.h"
#include "crlot_dsp.h"
#include "kernels.h"

namespace crlot {
int set_error(int code, const std::string& msg);  // abi.cpp: crlot_last_error()'s slot
}

namespace {

int fail(int code, const std::string& msg) { return crlot::set_error(code, msg); }
int hip_fail(hipError_t e, const char* what) {
    return fail(CRLOT_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

struct DeviceGuard {
    int prev = -1;
    bool moved = false;  // (restore only what this guard changed: one runtime query per call)
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (dev >= 0 && dev != prev) moved = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (moved && prev >= 0) (void)hipSetDevice(prev);
    }
};

}  // namespace

// =================================================================== Framer
struct crlot_framer {
    int64_t n = 0, h = 0, c = 1;
    int32_t mode = CRLOT_ZERO_PAD;
    bool ready = false;           // set_params called (framer.cc:31)
    std::vector<float> buf;       // interleaved samples
    int64_t wr = 0, rd = 0;       // positions in samples (not frames)
    std::vector<float> last;      // the frame pop() returned last (batched speculation, batch.h)

    void clear() {                // Framer::reset (framer.cc:76-86)
        buf.clear();
        wr = rd = 0;
        if (ready) buf.assign(size_t(n * c * 2), 0.0f);
    }
    int64_t available() const {   // calculate_available_frames (framer.cc:88-117)
        if (!ready || wr <= rd) return 0;
        const int64_t per_ch = (wr - rd) / c;
        if (per_ch < n) return (mode == CRLOT_ZERO_PAD && per_ch > 0) ? 1 : 0;
        int64_t k = (per_ch - n) / h + 1;
        // DROP keeps only frames that fit whole (always true for k above)
        if (mode == CRLOT_DROP && (k - 1) * h + n > per_ch) k = k > 0 ? k - 1 : 0;
        return k;
    }
};

namespace {
// the Framer that popped last (batch.h framer_last_signal); cleared when it changes
// or dies.  framer_last_signal reads that Framer's buffers from whatever thread runs
// an FFT forward, so every Framer mutation (push, pop and its compaction,
// set_params, reset, destroy) holds g_pop_mu too: a reader never sees a buffer
// mid-reallocation.  The sections are short and uncontended unless
// several threads push or pop at once.
std::mutex g_pop_mu;
const crlot_framer* g_last_pop = nullptr;
void forget_framer_locked(const crlot_framer* f) {
    if (g_last_pop == f) g_last_pop = nullptr;
}
}  // namespace

namespace crlot {
bool framer_last_signal(int64_t n, int64_t max_frames, const std::function<bool(const float*, int64_t)>& accept,
                        std::vector<float>* sig, int64_t* hop, int64_t* frames, int64_t* total, uint64_t* source) {
    std::lock_guard<std::mutex> lk(g_pop_mu);
    const crlot_framer* f = g_last_pop;
    if (!f || f->c != 1 || f->n != n || int64_t(f->last.size()) != n) return false;
    // frame 0 = the frame popped last; frame j >= 1 starts (j - 1) H into the
    // unread buffer, which begins H samples into frame 0 (framer.cc:164-167)
    const int64_t h = f->h, rest = f->wr - f->rd;
    if (h > n) return false;
    // frame j exists while j H < L (ZERO_PAD, padded) or j H + N <= L (DROP)
    const int64_t L = h + rest;
    const int64_t all = f->mode == CRLOT_ZERO_PAD ? (L + h - 1) / h : (L >= n ? (L - n) / h + 1 : 1);
    // the cheap test first (frame 0 against the caller's input), then a copy of
    // the first max_frames frames only: an unpredicted forward costs O(n), not
    // O(remaining signal)
    if (!accept(f->last.data(), h)) return false;
    const int64_t F = std::min(all, std::max<int64_t>(1, max_frames));
    const int64_t len = std::min(L, (F - 1) * h + n);
    *hop = h;
    *frames = F;
    *total = all;
    *source = reinterpret_cast<uintptr_t>(f);
    sig->resize(size_t(len));
    std::memcpy(sig->data(), f->last.data(), sizeof(float) * size_t(std::min(h, len)));
    if (len > h) std::memcpy(sig->data() + h, f->buf.data() + f->rd, sizeof(float) * size_t(len - h));
    return true;
}
}  // namespace crlot

extern "C" {

int crlot_framer_create(crlot_framer** out) {
    if (!out) return fail(CRLOT_EINVAL, "null argument");
    *out = new crlot_framer();
    return CRLOT_OK;
}

void crlot_framer_destroy(crlot_framer* f) {
    {
        std::lock_guard<std::mutex> lk(g_pop_mu);
        forget_framer_locked(f);
    }
    delete f;
}

int crlot_framer_set_params(crlot_framer* f, int64_t frame_size, int64_t hop_size, int64_t channels,
                            int32_t boundary_mode) {
    if (!f) return fail(CRLOT_EINVAL, "null framer");
    if (frame_size <= 0) return fail(CRLOT_EINVAL, "Frame size must be greater than 0");
    if (hop_size <= 0) return fail(CRLOT_EINVAL, "Hop size must be greater than 0");
    if (channels <= 0) return fail(CRLOT_EINVAL, "Channels must be greater than 0");
    if (boundary_mode != CRLOT_ZERO_PAD && boundary_mode != CRLOT_DROP)
        return fail(CRLOT_EINVAL, "Unknown boundary mode");
    std::lock_guard<std::mutex> lk(g_pop_mu);
    forget_framer_locked(f);
    f->n = frame_size;
    f->h = hop_size;
    f->c = channels;
    f->mode = boundary_mode;
    f->ready = true;
    f->clear();
    return CRLOT_OK;
}

int crlot_framer_push(crlot_framer* f, const float* interleaved, int64_t frames) {
    if (!f) return fail(CRLOT_EINVAL, "null framer");
    if (!f->ready || frames < 0) return 0;
    if (!interleaved && frames > 0) return 0;
    const int64_t add = frames * f->c;
    if (add == 0) return 1;
    std::lock_guard<std::mutex> lk(g_pop_mu);
    forget_framer_locked(f);  // the frames after the last pop change
    const int64_t need = f->wr + add;
    if (int64_t(f->buf.size()) < need)  // doubling growth (framer.cc:120-126)
        f->buf.resize(size_t(std::max<int64_t>(need, 2 * int64_t(f->buf.size()))), 0.0f);
    std::memcpy(f->buf.data() + f->wr, interleaved, sizeof(float) * size_t(add));
    f->wr = need;
    return 1;
}

int crlot_framer_pop(crlot_framer* f, float* out) {
    if (!f) return fail(CRLOT_EINVAL, "null framer");
    if (!f->ready || !out) return 0;
    std::lock_guard<std::mutex> lk(g_pop_mu);
    if (f->available() == 0) return 0;
    const int64_t len = f->n * f->c;     // extract_frame (framer.cc:128-181)
    const int64_t have = f->wr - f->rd;
    if (have >= len) {
        std::memcpy(out, f->buf.data() + f->rd, sizeof(float) * size_t(len));
    } else {
        if (f->mode == CRLOT_DROP) return 0;
        std::memcpy(out, f->buf.data() + f->rd, sizeof(float) * size_t(have));
        std::fill(out + have, out + len, 0.0f);
    }
    if (f->c == 1) {  // kept for the batched speculation (batch.h)
        f->last.assign(out, out + len);
        g_last_pop = f;
    } else {
        forget_framer_locked(f);
    }
    f->rd = std::min(f->rd + f->h * f->c, f->wr);
    if (f->rd > int64_t(f->buf.size()) / 2) {  // compaction once half the buffer is consumed
        const int64_t rest = f->wr - f->rd;
        if (rest > 0) std::memmove(f->buf.data(), f->buf.data() + f->rd, sizeof(float) * size_t(rest));
        f->wr = rest > 0 ? rest : 0;
        f->rd = 0;
    }
    return 1;
}

int64_t crlot_framer_available(const crlot_framer* f) {
    if (!f) return fail(CRLOT_EINVAL, "null framer");
    return f->available();
}

int crlot_framer_reset(crlot_framer* f) {
    if (!f) return fail(CRLOT_EINVAL, "null framer");
    std::lock_guard<std::mutex> lk(g_pop_mu);
    forget_framer_locked(f);
    f->clear();
    return CRLOT_OK;
}

int crlot_framer_info(const crlot_framer* f, int64_t* frame_size, int64_t* hop_size,
                      int64_t* channels, int32_t* boundary_mode, int64_t* buffer_size) {
    if (!f) return fail(CRLOT_EINVAL, "null framer");
    if (frame_size) *frame_size = f->ready ? f->n : 0;
    if (hop_size) *hop_size = f->ready ? f->h : 0;
    if (channels) *channels = f->c;
    if (boundary_mode) *boundary_mode = f->mode;
    if (buffer_size) *buffer_size = int64_t(f->buf.size());
    return CRLOT_OK;
}

}  // extern "C"

// =================================================================== OLAAccumulator
namespace {
constexpr int kSlots = 4;  // pinned staging slots for host-pointer calls
}

struct crlot_ola {
    crlot_ola_config cfg{};
    int device = 0;
    int64_t R = 0;                    // ring_len (OLAAccumulator.cc:249-258)
    std::vector<float> window, norm;  // host copies; window empty = none set
    // reference counters
    int64_t read_pos = 0, produced = 0;
    bool flushing = false;
    float host_peak = 0.0f;           // peak of host-pointer produce() calls
    // device state
    float* d_ring = nullptr;          // [C][R]
    float* d_den = nullptr;           // [R]
    float* d_win = nullptr;           // [N]
    unsigned* d_peak = nullptr;       // running max |out| of device produce() calls (float bits)
    hipStream_t own = nullptr;        // stream of the host-pointer calls
    hipStream_t last = nullptr;       // stream of the previous call (cross-stream ordering)
    bool last_set = false;
    hipEvent_t order = nullptr;
    struct Slot {
        float* h = nullptr;
        size_t cap = 0;
        hipEvent_t ev = nullptr;
        bool pending = false;
    } slot[kSlots];
    int next_slot = 0;
    // host-pointer calls run on a resident call server (call_rt.hip); device-form
    // calls on streams.  Switching between the two drains the other side first.
    crlot::CallServer* srv = nullptr;
    crlot::SharedServer* shared = nullptr;  // powers of two 256..4096, and other even sizes the any-size server holds: the size's
                                      // server, shared with the FFT plans (chained speculation)
    int mode = 0;                     // 0 none yet, 1 streams, 2 call server
    int64_t last_start = -1;          // start_sample and gain of the last host push
    float last_gain = 1.0f;
    int64_t last_req_n = 0;           // n of the last produce(): the next one's prediction
    struct Spec {                     // produce block speculated after the last add
        bool valid = false;
        bool chain = false;           // computed by a chained forward (its chain_done)
        uint64_t index = 0;
        int64_t rp = 0, n = 0;
        crlot::CallSlot slot;
    } spec;

    // batched speculation (batch.h): no add since creation / reset, and the
    // batch this object is attached to while its ring is virtual (its pushes
    // and produces served from the batch: the device ring untouched since)
    bool pristine = true;
    crlot::BatchSpec* vb = nullptr;
    uint64_t vgen = 0;
    int64_t vread = 0;   // samples produced from the batch (absolute, from the attach)
    int64_t vlast = -1;  // last batch frame pushed
    uint64_t tgen = 0;   // bumped by every table upload (upload_norm; batch.h fresh_ola)
    bool valias = false; // a push wrapped onto unread slots (no produce yet): batch_alias serves the produces
    bool vya = false;    // batch_alias ran (its slots are the ring, minus the ones read since)

    int64_t N() const { return cfg.frame_size; }
    int64_t H() const { return cfg.hop_size; }
    int64_t C() const { return cfg.channels; }
};

namespace {

// Held around an object's requests on a shared server.
struct ServerLock {
    std::mutex* m = nullptr;
    explicit ServerLock(crlot_ola* o) : m(o->shared ? &o->shared->mu : nullptr) {
        if (m) m->lock();
    }
    ~ServerLock() {
        if (m) m->unlock();
    }
};

// max |x[i]| folded as update_peak_meter's std::max chain does (a NaN never
// wins a std::max(acc, NaN), so any grouping gives the same value): four lanes
float peak_of(const float* x, int64_t n) {
    float m[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    int64_t i = 0;
    for (; i + 4 <= n; i += 4)
        for (int q = 0; q < 4; ++q) m[q] = std::max(m[q], std::fabs(x[i + q]));
    for (; i < n; ++i) m[0] = std::max(m[0], std::fabs(x[i]));
    return std::max(std::max(m[0], m[1]), std::max(m[2], m[3]));
}

// the OLA object whose window was set last (batch.h fresh_ola)
std::mutex g_fresh_mu;
crlot_ola* g_fresh_ola = nullptr;

// the rings of the live objects (call.h ola_ring_live)
std::mutex g_rings_mu;
std::vector<const float*> g_rings;
void ring_register(const float* r) {
    std::lock_guard<std::mutex> lk(g_rings_mu);
    g_rings.push_back(r);
}
void ring_unregister(const float* r) {
    std::lock_guard<std::mutex> lk(g_rings_mu);
    g_rings.erase(std::remove(g_rings.begin(), g_rings.end(), r), g_rings.end());
}

void ola_free(crlot_ola* o) {
    if (!o) return;
    {
        std::lock_guard<std::mutex> lk(g_fresh_mu);
        if (g_fresh_ola == o) g_fresh_ola = nullptr;
    }
    DeviceGuard g(o->device);
    if (o->shared) {
        std::lock_guard<std::mutex> lk(o->shared->mu);
        if (o->vb && o->vb->ola == o) o->vb->ola = nullptr;  // nothing to rebuild: the object goes
        o->vb = nullptr;
        if (o->shared->target.owner == o) o->shared->target = crlot::ChainTarget{};
        if (o->mode == 2) (void)o->srv->drain();  // its requests touch this object's rings
    } else {
        delete o->srv;  // waits for its requests, stops the kernel
    }
    if (o->last_set && o->last) (void)hipStreamSynchronize(o->last);
    if (o->own) (void)hipStreamSynchronize(o->own);
    // resources back to the pools (respool.h): device blocks stream-ordered on
    // the object's own stream, which then serves the next object
    for (auto& s : o->slot) {
        crlot::pool_event_put(o->device, s.ev);
        crlot::pool_pinned_put(s.h, s.cap * sizeof(float));
    }
    if (o->d_ring) ring_unregister(o->d_ring);
    if (o->srv) o->srv->unpoison(o->d_ring);  // (the block may serve a later object)
    if (o->own) {
        crlot::pool_free(o->d_ring, o->own);  // the object's one device block (crlot_ola_create)
    }
    crlot::pool_event_put(o->device, o->order);
    crlot::pool_stream_put(o->device, o->own);
    delete o;
}

// Make `s` the object's stream, ordered after everything issued on the previous
// one and after every request of the call server.
hipError_t use_stream(crlot_ola* o, hipStream_t s) {
    if (o->mode == 2) {
        ServerLock lk(o);
        if (o->srv->drain() != CRLOT_OK) return hipErrorLaunchFailure;
        o->spec.valid = false;
    }
    o->mode = 1;
    if (o->last_set && o->last != s) {
        hipError_t e;
        if ((e = hipEventRecord(o->order, o->last)) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(s, o->order, 0)) != hipSuccess) return e;
    }
    o->last = s;
    o->last_set = true;
    return hipSuccess;
}

// A pinned staging slot of at least `floats`, free for the host to write.
hipError_t take_slot(crlot_ola* o, size_t floats, crlot_ola::Slot** out) {
    crlot_ola::Slot& s = o->slot[o->next_slot];
    o->next_slot = (o->next_slot + 1) % kSlots;
    hipError_t e;
    if (s.pending) {
        if ((e = hipEventSynchronize(s.ev)) != hipSuccess) return e;
        s.pending = false;
    }
    if (!s.ev && (e = crlot::pool_event(o->device, &s.ev)) != hipSuccess) return e;
    if (s.cap < floats) {
        crlot::pool_pinned_put(s.h, s.cap * sizeof(float));
        s.h = nullptr;
        s.cap = 0;
        void* hb = nullptr;
        size_t cap = 0;
        if ((e = crlot::pool_pinned(floats * sizeof(float), &hb, &cap)) != hipSuccess) return e;
        s.h = static_cast<float*>(hb);
        s.cap = cap / sizeof(float);
    }
    *out = &s;
    return hipSuccess;
}

// OLAAccumulator::initialize_normalization (OLAAccumulator.cc:260-288) -> den
// on the device, ordered on the object's current stream.
std::atomic<uint64_t> g_tgen{0};  // process-wide: a new object at a freed one's address never repeats a tgen

int upload_norm(crlot_ola* o, hipStream_t s) {
    o->tgen = g_tgen.fetch_add(1, std::memory_order_relaxed) + 1;
    const bool has_w = !o->window.empty();
    crlot_norm_table(has_w ? o->window.data() : nullptr, o->N(), o->H(), o->R,
                     o->cfg.apply_window_inside, o->cfg.eps, o->norm.data());
    const float eps = o->cfg.eps;
    hipError_t e;
    if (!has_w) {  // no window: all ones (crlot_norm_table), a fill, no staging
        const float one = 1.0f > eps ? 1.0f : eps;  // normalize_and_clear's guard (kernels.cc:32)
        unsigned bits = 0;
        std::memcpy(&bits, &one, sizeof(bits));
        if ((e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(o->d_den), int(bits), size_t(o->R), s)))
            return hip_fail(e, "table upload");
        return CRLOT_OK;
    }
    // den and window are adjacent on the device (crlot_ola_create): one copy
    // from a staging slot laid out the same way
    const size_t wo = size_t(o->d_win - o->d_den);
    crlot_ola::Slot* sl = nullptr;
    if ((e = take_slot(o, wo + size_t(o->N()), &sl)) != hipSuccess) return hip_fail(e, "staging");
    for (int64_t i = 0; i < o->R; ++i)  // normalize_and_clear's guard (kernels.cc:32)
        sl->h[i] = (o->norm[i] > eps) ? o->norm[i] : eps;
    if (has_w) std::memcpy(sl->h + wo, o->window.data(), sizeof(float) * size_t(o->N()));
    const size_t floats = has_w ? wo + size_t(o->N()) : size_t(o->R);
    if ((e = hipMemcpyAsync(o->d_den, sl->h, sizeof(float) * floats, hipMemcpyHostToDevice, s)) ||
        (e = hipEventRecord(sl->ev, s)))
        return hip_fail(e, "table upload");
    sl->pending = true;
    return CRLOT_OK;
}

// Clamp [start_off, start_off + size) to the frame (OLAAccumulator.cc:68-79);
// returns false when nothing is added.
bool clamp(const crlot_ola* o, int64_t start_off, int64_t size, int64_t* eff) {
    if (size == 0 || start_off >= o->N()) return false;
    *eff = (start_off + size > o->N()) ? o->N() - start_off : size;
    return true;
}

// the window an add uses (OLAAccumulator.cc:82-83): the object's own copy with
// apply_window_inside, else the caller's (nullable)
bool use_window(const crlot_ola* o, bool caller_win) {
    return o->cfg.apply_window_inside ? !o->window.empty() : caller_win;
}

int add_common(crlot_ola* o, const float* d_src, int64_t cs, int64_t js, const float* d_win,
               int64_t start_sample, int64_t eff, float gain, hipStream_t s, int64_t channels = -1) {
    const int64_t len = std::min(eff, o->R);  // RingBuffer::split clamps to capacity
    const int64_t nch = channels < 0 ? o->C() : channels;
    hipError_t e = crlot::launch_ola_add(o->d_ring, int(nch), o->R, d_src, cs, js, d_win,
                                         start_sample % o->R, len, gain, s);
    if (e != hipSuccess) return hip_fail(e, "OLA add kernel launch");
    o->pristine = false;
    if (nch < o->C()) return CRLOT_OK;  // caller reports the null channel
    o->produced = std::max(o->produced, start_sample + eff);  // :114
    return CRLOT_OK;
}

// Host-pointer calls run on the object's call server: first wait for the
// stream-ordered work issued since the last request (and make the next request
// re-read device memory).
int to_server(crlot_ola* o) {
    if (!o->srv) {
        const size_t C = size_t(o->C()), N = size_t(o->N()), R = size_t(o->R);
        const bool pow2 = N >= 256 && N <= 4096 && (N & (N - 1)) == 0;
        // other even sizes: the any-size server of the FFT plans of this frame size
        const bool any = !pow2 && N % 2 == 0 && crlot::any_supported(int(N / 2)) && crlot::call_any_waves(int(N / 2)) > 0;
        int rc = CRLOT_OK;
        if ((pow2 || any) &&
            (o->shared = crlot::shared_server(o->device, pow2 ? int(N / 128) : -int(N / 2), &rc)) != nullptr) {
            o->srv = o->shared->srv;
        } else {
            const size_t blk = std::min(R, std::max<size_t>(N, 1024));
            rc = crlot::CallServer::create(o->device, 0, 8, C * N + N, C * blk, C * blk, &o->srv);
            if (rc != CRLOT_OK) return rc;
        }
    }
    if (o->srv->poisoned(o->d_ring))
        return fail(CRLOT_EHIP, "OLA object: a timed-out call left its ring state unknown; reset() it");
    if (o->mode == 1) {
        hipError_t e = o->last_set ? hipStreamSynchronize(o->last) : hipSuccess;
        if (e != hipSuccess) return hip_fail(e, "stream order");
        o->srv->acquire_next();
    }
    o->mode = 2;
    return CRLOT_OK;
}

// ChainTarget::predict: the push and produce this object's next frame will make,
// if it keeps the drop-in loop's rhythm (mono, whole frames at start + H, the
// object's own window or none, produce(n) of the previous count)
bool ola_predict(const void* owner, crlot::ChainPred* out) {
    const crlot_ola* o = static_cast<const crlot_ola*>(owner);
    if (o->C() != 1 || o->mode != 2 || o->last_start < 0) return false;
    out->ring = o->d_ring;
    out->den = o->d_den;
    out->win = (o->cfg.apply_window_inside && !o->window.empty()) ? o->d_win : nullptr;
    out->R = o->R;
    out->N = o->N();
    out->start = o->last_start + o->H();
    out->rp = o->read_pos;
    const int64_t produced_after = std::max(o->produced, out->start + o->N());
    const int64_t avail = produced_after > o->read_pos ? produced_after - o->read_pos : 0;
    out->n = std::min({o->last_req_n > 0 ? o->last_req_n : o->H(), avail, o->R});
    out->gain = o->last_gain;
    return true;
}

// The frame being pushed is the inverse the shared server speculated after the
// last forward, pushed where the chain predicted: commit it without a payload;
// the produce block the chain computed becomes this object's speculation.
// Returns 1 when it committed, 0 when the push must take the ordinary path.
int try_chain_push(crlot_ola* o, const float* frame, bool uw, bool caller_win, int64_t start_sample,
                   int64_t start_off, int64_t eff, float gain) {
    crlot::SharedServer* sh = o->shared;
    if (!sh || o->C() != 1 || o->mode != 2) return 0;
    crlot::CallServer* sv = sh->srv;
    const int64_t N = o->N();
    // learn the association: this object pushes the frames the server speculates
    // (or the output of the last single-frame inverse request: a caller that edits
    // the spectrum pushes what the inverse call returned)
    if (sh->target.owner != o && start_off == 0 && eff == N &&
        ((sh->fft.index + 4 > sv->submitted() && sh->fft.slot.spec && sv->live(sh->fft.slot) &&
          std::memcmp(frame, sh->fft.slot.spec, sizeof(float) * size_t(N)) == 0) ||
         (sh->inv.valid && sh->inv.index + 4 > sv->submitted() && sv->live(sh->inv.slot) &&
          std::memcmp(frame, sh->inv.slot.out, sizeof(float) * size_t(N)) == 0))) {
        sh->target.owner = o;
        sh->target.predict = ola_predict;
        return 0;
    }
    const crlot::ChainPred& pd = sh->chain.pred;
    const float* want_win = (uw && !caller_win) ? o->d_win : nullptr;
    if (!(sh->chain.valid && sh->chain.index == sv->submitted() && sh->target.owner == o && start_off == 0 &&
          eff == N && start_sample == pd.start && gain == pd.gain && !caller_win && want_win == pd.win &&
          pd.rp == o->read_pos && sv->live(sh->chain.slot) && sh->chain.frame &&
          std::memcmp(frame, sh->chain.frame, sizeof(float) * size_t(N)) == 0))
        return 0;
    sh->chain.valid = false;
    // the push itself rides on the next request (the server keeps the frame in LDS)
    crlot::CallReq::Pend pe{};
    pe.flags = crlot::kPendCommit;
    pe.ring = o->d_ring;
    pe.win = pd.win;
    pe.R = o->R;
    pe.start = start_sample % o->R;
    pe.len = N;
    pe.gain = gain;
    pe.src_index = sh->chain.index;
    pe.src_off = sh->chain.frame_off;  // the frame pushed, in the output arena
    int rc = sv->defer(pe);
    if (rc != CRLOT_OK) return rc;
    o->spec.valid = true;
    o->spec.chain = true;
    o->spec.index = sh->chain.index;
    o->spec.rp = pd.rp;
    o->spec.n = pd.n;
    o->spec.slot = sh->chain.slot;
    o->spec.slot.spec += N;  // the chained produce block follows the speculated frame
    o->produced = std::max(o->produced, start_sample + eff);  // :114
    o->last_start = start_sample;
    o->last_gain = gain;
    return 1;
}

// add_frame_SoA (rows = ch channel pointers) / push_frame_AoS (rows[0] = the
// interleaved frame at start_off): eff samples per channel; caller_win: a window
// slice the host copies in; obj_win: the object's device window (or null)
int server_add(crlot_ola* o, const float* const* rows, int64_t ch, bool aos, const float* caller_win,
               const float* obj_win, int64_t start_sample, int64_t eff, float gain) {
    int rc = to_server(o);
    if (rc != CRLOT_OK) return rc;
    crlot::CallServer* sv = o->srv;
    const int64_t C = o->C();
    const int64_t len = std::min(eff, o->R);  // RingBuffer::split clamps to capacity
    // speculate the produce the host will ask for next: its last count (H before the first)
    const int64_t produced_after = ch == C ? std::max(o->produced, start_sample + eff) : o->produced;
    const int64_t avail = produced_after > o->read_pos ? produced_after - o->read_pos : 0;
    const int64_t pn = std::min({o->last_req_n > 0 ? o->last_req_n : o->H(), avail, o->R});
    if ((rc = sv->grow(size_t(C * eff + eff), size_t(C * std::max<int64_t>(pn, 1)),
                       size_t(C * std::max<int64_t>(pn, 1)))) != CRLOT_OK)
        return rc;
    crlot::CallSlot sl;
    if ((rc = sv->next_slot(&sl)) != CRLOT_OK) return rc;
    if (aos) {
        sv->put(sl.in, rows[0], size_t(eff * C));
    } else {
        for (int64_t c = 0; c < ch; ++c) sv->put(sl.in + c * eff, rows[c], size_t(eff));
    }
    crlot::CallReq r{};
    r.op = crlot::kCallOlaAdd;
    r.channels = int32_t(ch);
    r.win_off = -1;
    if (caller_win) {
        sv->put(sl.in + ch * eff, caller_win, size_t(eff));
        r.win_off = sl.in_off + ch * eff;
    }
    r.p0 = obj_win;
    r.p1 = o->d_den;
    r.p2 = o->d_ring;
    r.i[0] = o->R;
    r.i[1] = start_sample % o->R;
    r.i[2] = len;
    r.i[3] = aos ? 1 : 0;
    r.f0 = gain;
    const bool spec = ch == C && pn > 0;
    if (spec) {
        r.flags = crlot::kCallSpec;
        r.i[4] = o->read_pos % o->R;
        r.i[5] = pn;
    }
    if ((rc = sv->submit(r, sl)) != CRLOT_OK) return rc;
    o->pristine = false;
    o->spec.valid = spec;
    o->spec.chain = false;
    o->spec.index = sl.index;
    o->spec.rp = o->read_pos;
    o->spec.n = pn;
    o->spec.slot = sl;
    if (ch == C) o->produced = std::max(o->produced, start_sample + eff);  // :114
    o->last_start = start_sample;
    o->last_gain = gain;
    return CRLOT_OK;
}


// ---- batched speculation (batch.h), all under the shared server's lock

// A mono host push of the inverse frame the batch just served, at the loop's
// rhythm: recorded without touching the device (the first one attaches the
// object, whose ring must be untouched, and computes the produce blocks of
// every remaining frame with the object's window and divisors).  1: served.
int batch_push(crlot_ola* o, const float* frame, bool caller_win, int64_t start_sample, int64_t start_off,
               int64_t eff, float gain) {
    if (o->srv && o->srv->poisoned(o->d_ring)) return 0;  // (the ordinary path reports it)
    crlot::BatchSpec* b = o->shared ? o->shared->batch : nullptr;
    if (!b || crlot::spec_mode() < 2 || b->pushed < 0 || o->C() != 1 || b->n != o->N()) return 0;
    const int64_t j = b->pushed, N = o->N();
    if (start_off != 0 || eff != N || caller_win || !o->cfg.apply_window_inside || o->window.empty() ||
        o->flushing || std::memcmp(frame, b->h_r + b->row(j) * size_t(N), sizeof(float) * size_t(N)) != 0)
        return 0;
    if (o->vb) {
        if (o->vb != b || b->ola != o || o->vgen != b->gen || j != o->vlast + 1 ||
            start_sample != (j - b->j0) * b->h || !(gain == b->gain))
            return 0;
        // a push reaching R samples past the oldest unread one wraps onto unread
        // ring data (the harness's push-everything-first order): the
        // batch's overlap-add does not alias, the ring does.  Before any produce
        // the wrapped ring is still a function of the frames (batch_alias);
        // after one, leave it to the ring
        // (a batch of several windows holds only the current one's frames: the ring's path)
        if (start_sample + N > o->vread + o->R) {
            if (o->vread != 0 || !b->single()) return 0;
            o->valias = true;
        }
    } else {
        if (!o->pristine || start_sample != 0 || o->read_pos != 0 || o->produced != 0) return 0;
        if (b->ola) {  // another object rode this batch: rebuild its ring first
            const int rc = crlot::ola_materialize_locked(b->ola);
            if (rc != CRLOT_OK) return rc;
        }
        const int rc = crlot::batch_attach(o->shared, o, j, o->R, o->d_win, o->d_den, gain, o->own, o->tgen);
        if (rc != CRLOT_OK) return rc;
        o->vb = b;
        o->vgen = b->gen;
        o->vread = 0;
        o->valias = o->vya = false;
    }
    b->pushed = -1;
    crlot::spec_count(crlot::kStatPush);
    o->vlast = j;
    o->pristine = false;
    o->spec.valid = false;
    o->produced = std::max(o->produced, start_sample + eff);  // :114
    o->last_start = start_sample;
    o->last_gain = gain;
    return 1;
}

// A mono host produce of n (already clamped to the available count) inside the
// blocks the batch's pushes have finalised.  1: served into out.
int batch_produce(crlot_ola* o, float* out, int64_t n) {
    if (o->srv && o->srv->poisoned(o->d_ring)) return 0;
    crlot::BatchSpec* b = o->vb;
    if (!b || crlot::spec_mode() < 2 || b->ola != o || o->vgen != b->gen || o->flushing || o->C() != 1) return 0;
    if (o->read_pos != o->vread % o->R) return 0;
    if (o->valias) {
        // every frame pushed, none produced between: slot p holds the wrapped sum
        // until read at position p, zero after (normalize_and_clear), so the
        // reads give y[p] for p < R and 0 / den beyond (position t reads slot
        // t mod R, already read and cleared once t >= R).  A read longer than
        // the ring (e2e_benchmark.cc's produce(T)) is clamped to it by
        // RingBuffer::split: R outputs, out[R, n) untouched, every slot cleared
        if (o->vlast != b->M - 1 || !b->single()) return 0;
        if (!o->vya) {
            const int rc = crlot::batch_alias(b, o->R, o->d_win, o->d_den);
            if (rc != CRLOT_OK) return rc;
            o->vya = true;
        }
        const int64_t m = std::min(n, o->R);
        for (int64_t i = 0; i < m; ++i) {
            const int64_t t = o->vread + i;
            out[i] = t < o->R ? b->ya[t] : 0.0f;
        }
        o->vread += n;
        crlot::spec_count(crlot::kStatProduce);
        return 1;
    }
    // positions no later frame reaches: up to the last pushed frame's hop, or to
    // its end once the batch's last frame is pushed (no later frame exists)
    const int64_t final_end =
        (o->vlast - b->j0 + 1) * b->h + (o->vlast == b->M - 1 ? std::max<int64_t>(0, b->n - b->h) : 0);
    // (a read longer than the ring is clamped by RingBuffer::split: the ring's path)
    if (n > o->R || o->vread + n > final_end || o->vread < b->y_lo) return 0;
    const int rc = crlot::batch_wait_y(b);
    if (rc != CRLOT_OK) return rc;
    std::memcpy(out, b->h_y + (o->vread - b->y_base), sizeof(float) * size_t(n));
    o->vread += n;
    crlot::spec_count(crlot::kStatProduce);
    return 1;
}

// the object's ring when a live batch no longer serves it: zero ring + the
// batch frames it was served, from the read position on (the cleared part of
// each push is exactly what its produces removed), in push order
int ola_materialize(crlot_ola* o) {
    crlot::BatchSpec* b = o->vb;
    if (!b) return CRLOT_OK;
    o->vb = nullptr;
    if (b->ola == o) b->ola = nullptr;
    if (o->vgen != b->gen) return fail(CRLOT_ERUNTIME, "OLA object: batched speculation state lost");
    crlot::spec_count(crlot::kStatRebuild);
    crlot::CallServer* sv = o->srv;
    int rc = sv ? sv->drain() : CRLOT_OK;
    if (rc != CRLOT_OK) return rc;
    if (o->valias && o->vya) {  // the wrapped slots, the ones read since cleared
        const int64_t z = std::min(o->vread, o->R);
        hipError_t e = hipMemcpyAsync(o->d_ring, b->d_acc, sizeof(float) * size_t(o->R), hipMemcpyDeviceToDevice, o->own);
        if (e == hipSuccess && z > 0) e = hipMemsetAsync(o->d_ring, 0, sizeof(float) * size_t(z), o->own);
        if (e == hipSuccess) e = hipStreamSynchronize(o->own);
        if (e != hipSuccess) return hip_fail(e, "OLA rebuild");
        if (sv) sv->acquire_next();
        o->spec.valid = false;
        return CRLOT_OK;
    }
    const int64_t N = o->N(), h = b->h;
    for (int64_t k = b->j0; k <= o->vlast; ++k) {
        const int64_t rel = (k - b->j0) * h, off = std::max<int64_t>(0, o->vread - rel);
        if (off >= N) continue;
        if (k < b->cb)  // (a continuing object never needs a frame the window dropped: batch.cpp continue_window)
            return fail(CRLOT_ERUNTIME, "OLA object: batched speculation lost a frame it needs");
        const hipError_t e = crlot::launch_ola_add(o->d_ring, 1, o->R, b->d_r + b->row(k) * size_t(N) + off, N, 1,
                                                   o->d_win + off, (rel + off) % o->R, N - off, b->gain, o->own);
        if (e != hipSuccess) return hip_fail(e, "OLA rebuild");
    }
    const hipError_t e = hipStreamSynchronize(o->own);
    if (e != hipSuccess) return hip_fail(e, "OLA rebuild");
    if (sv) sv->acquire_next();
    o->spec.valid = false;
    return CRLOT_OK;
}

// entry points outside the speculated loop: rebuild a virtual ring first
int ensure_real(crlot_ola* o) {
    if (!o->vb) return CRLOT_OK;
    ServerLock lk(o);
    return ola_materialize(o);
}

}  // namespace

namespace crlot {
int ola_materialize_locked(crlot_ola* o) { return ola_materialize(o); }
bool ola_ring_live(const float* ring) {
    std::lock_guard<std::mutex> lk(g_rings_mu);
    return std::find(g_rings.begin(), g_rings.end(), ring) != g_rings.end();
}
// the object read up to the window end's position with every frame before it
// pushed, so only frames from we - (ceil(N / H) - 1) on reach its unread positions
bool ola_can_continue(const crlot_ola* o, const BatchSpec* b) {
    return o->vb == b && b->ola == o && o->vgen == b->gen && o->vlast == b->we - 1 && !o->valias && !o->flushing &&
           o->vread >= (b->we - b->j0) * b->h;
}
}  // namespace crlot

extern "C" {

int crlot_ola_create(const crlot_ola_config* cfg, crlot_ola** out) {
    if (!cfg || !out) return fail(CRLOT_EINVAL, "null argument");
    *out = nullptr;
    // OLAConfig::isValid (OLAAccumulator.h:25-28)
    if (!(cfg->sample_rate > 0 && cfg->frame_size > 0 && cfg->hop_size > 0 && cfg->channels > 0 &&
          cfg->eps > 0.0f))
        return fail(CRLOT_EINVAL, "Invalid OLA configuration");
    if (cfg->frame_size > (int64_t(1) << 26) || cfg->channels > 65535)
        return fail(CRLOT_EUNSUPPORTED, "OLA object: frame or channel count beyond the device path");
    crlot_ola* o = new crlot_ola();
    o->cfg = *cfg;
    if (cfg->device < 0) {
        if (hipGetDevice(&o->device) != hipSuccess) {
            delete o;
            return fail(CRLOT_EHIP, "no HIP device");
        }
    } else {
        o->device = cfg->device;
    }
    DeviceGuard g(o->device);
    o->R = crlot_ring_len(o->N(), o->H());
    o->norm.assign(size_t(o->R), 1.0f);
    const size_t C = size_t(o->C()), R = size_t(o->R), N = size_t(o->N());
    hipError_t e;
    // one device block: ring [C][R], peak, den [R], window [N] (256-byte
    // aligned parts; ring and peak adjacent, so one memset clears both)
    auto up = [](size_t bytes) { return (bytes + 255) & ~size_t(255); };
    const size_t b_ring = up(sizeof(float) * C * R), b_peak = 256, b_den = up(sizeof(float) * R);
    void* blk = nullptr;
    if ((e = crlot::pool_stream(o->device, &o->own)) || (e = crlot::pool_event(o->device, &o->order)) ||
        (e = crlot::pool_malloc(o->device, &blk, b_ring + b_peak + b_den + up(sizeof(float) * N), o->own))) {
        ola_free(o);
        return e == hipErrorOutOfMemory ? fail(CRLOT_ENOMEM, "OLA object allocation")
                                        : hip_fail(e, "OLA object allocation");
    }
    char* base = static_cast<char*>(blk);
    o->d_ring = reinterpret_cast<float*>(base);
    o->d_peak = reinterpret_cast<unsigned*>(base + b_ring);
    o->d_den = reinterpret_cast<float*>(base + b_ring + b_peak);
    o->d_win = reinterpret_cast<float*>(base + b_ring + b_peak + b_den);
    ring_register(o->d_ring);
    if ((e = hipMemsetAsync(o->d_ring, 0, b_ring + sizeof(unsigned), o->own))) {
        ola_free(o);
        return hip_fail(e, "OLA object init");
    }
    (void)use_stream(o, o->own);
    // no window yet: all ones.  Not waited for: every later use of the ring and
    // tables is ordered after it on the object's stream (use_stream), and a
    // device failure surfaces at the next synchronising call
    int rc = upload_norm(o, o->own);
    if (rc != CRLOT_OK) {
        ola_free(o);
        return rc;
    }
    *out = o;
    return CRLOT_OK;
}

void crlot_ola_destroy(crlot_ola* o) { ola_free(o); }

int crlot_ola_set_window(crlot_ola* o, const float* w, int32_t wlen) {
    if (!o) return fail(CRLOT_EINVAL, "null OLA object");
    if (!w) return fail(CRLOT_EINVAL, "Window pointer cannot be null");
    if (int64_t(wlen) != o->N()) return fail(CRLOT_EINVAL, "Window size must match frame size");
    DeviceGuard g(o->device);
    int rc = ensure_real(o);
    if (rc != CRLOT_OK) return rc;
    crlot::note_window(w, wlen);
    o->window.assign(w, w + wlen);
    hipError_t e = use_stream(o, o->own);
    if (e != hipSuccess) return hip_fail(e, "stream order");
    rc = upload_norm(o, o->own);
    if (rc == CRLOT_OK) {
        std::lock_guard<std::mutex> lk(g_fresh_mu);
        g_fresh_ola = o;
    }
    return rc;
}

int crlot_ola_add_frame_soa(crlot_ola* o, const float* const* ch_frames, const float* window,
                            int64_t start_sample, int64_t start_off, int64_t size, float gain) {
    if (!o) return fail(CRLOT_EINVAL, "null OLA object");
    if (!ch_frames) return fail(CRLOT_EINVAL, "Channel frames pointer cannot be null");
    if (start_sample < 0 || start_off < 0 || size < 0) return fail(CRLOT_EINVAL, "negative position");
    int64_t eff = 0;
    if (!clamp(o, start_off, size, &eff)) return CRLOT_OK;
    // the reference throws at the first null channel after adding the ones
    // before it (OLAAccumulator.cc:80-82), and then leaves produced_ as it was
    int64_t ok = 0;
    while (ok < o->C() && ch_frames[ok]) ++ok;
    DeviceGuard g(o->device);
    const bool uw = use_window(o, window != nullptr);
    const bool caller_win = uw && !o->cfg.apply_window_inside;
    const float* rows_small[8];  // (no allocation for up to 8 channels)
    std::vector<const float*> rows_big(ok > 8 ? size_t(ok) : 0);
    const float** rows = ok > 8 ? rows_big.data() : rows_small;
    for (int64_t c = 0; c < ok; ++c) rows[c] = ch_frames[c] + start_off;
    int rc = to_server(o);
    if (rc != CRLOT_OK) return rc;
    ServerLock lk(o);
    if (ok == o->C()) {  // a mono push the batch predicted (as push_frame_AoS below)
        rc = batch_push(o, rows[0], caller_win, start_sample, start_off, eff, gain);
        if (rc != 0) return rc < 0 ? rc : CRLOT_OK;
    }
    if (o->vb && (rc = ola_materialize(o)) != CRLOT_OK) return rc;
    rc = ok == o->C() ? try_chain_push(o, rows[0], uw, caller_win, start_sample, start_off, eff, gain) : 0;
    if (rc < 0) return rc;
    if (rc == 0)
        rc = server_add(o, rows, ok, false, caller_win ? window + start_off : nullptr,
                        (uw && !caller_win) ? o->d_win + start_off : nullptr, start_sample, eff, gain);
    if (rc < 0) return rc;
    return ok < o->C() ? fail(CRLOT_EINVAL, "Channel frame pointer cannot be null") : CRLOT_OK;
}

int crlot_ola_push_frame_aos(crlot_ola* o, const float* interleaved, const float* window,
                             int64_t start_sample, int64_t start_off, int64_t size, float gain) {
    if (!o) return fail(CRLOT_EINVAL, "null OLA object");
    if (!interleaved) return fail(CRLOT_EINVAL, "Interleaved input pointer cannot be null");
    if (start_sample < 0 || start_off < 0 || size < 0) return fail(CRLOT_EINVAL, "negative position");
    int64_t eff = 0;
    if (!clamp(o, start_off, size, &eff)) return CRLOT_OK;
    DeviceGuard g(o->device);
    // push_frame_AoS deinterleaves [start_off, start_off + eff) and calls
    // add_frame_SoA with start_off = 0, so the window is read from index 0
    // (OLAAccumulator.cc:146-159)
    const bool uw = use_window(o, window != nullptr);
    const bool caller_win = uw && !o->cfg.apply_window_inside;
    const float* src = interleaved + start_off * o->C();
    int rc = to_server(o);
    if (rc != CRLOT_OK) return rc;
    ServerLock lk(o);
    rc = batch_push(o, src, window != nullptr, start_sample, start_off, eff, gain);
    if (rc != 0) return rc < 0 ? rc : CRLOT_OK;
    if (o->vb && (rc = ola_materialize(o)) != CRLOT_OK) return rc;
    // (a mono AoS frame is the SoA one; the window is read from index 0 as for start_off 0)
    rc = try_chain_push(o, src, uw, caller_win, start_sample, start_off == 0 ? 0 : -1, eff, gain);
    if (rc < 0) return rc;
    if (rc == 1) return CRLOT_OK;
    return server_add(o, &src, o->C(), true, caller_win ? window : nullptr, (uw && !caller_win) ? o->d_win : nullptr,
                      start_sample, eff, gain);
}

int crlot_ola_add_frame_soa_device(crlot_ola* o, const float* d_frames, int64_t ld_frames,
                                   const float* d_window, int64_t start_sample, int64_t start_off,
                                   int64_t size, float gain, void* stream) {
    if (!o) return fail(CRLOT_EINVAL, "null OLA object");
    if (!d_frames) return fail(CRLOT_EINVAL, "Channel frames pointer cannot be null");
    if (start_sample < 0 || start_off < 0 || size < 0) return fail(CRLOT_EINVAL, "negative position");
    int64_t eff = 0;
    if (!clamp(o, start_off, size, &eff)) return CRLOT_OK;
    if (o->C() > 1 && ld_frames < o->N()) return fail(CRLOT_EINVAL, "leading dimension too small");
    DeviceGuard g(o->device);
    if (const int rc = ensure_real(o); rc != CRLOT_OK) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);  // NULL: the default stream (crlot_dsp.h)
    hipError_t e = use_stream(o, s);
    if (e != hipSuccess) return hip_fail(e, "stream order");
    const bool uw = use_window(o, d_window != nullptr);
    const float* dw = !uw ? nullptr : o->cfg.apply_window_inside ? o->d_win + start_off : d_window + start_off;
    return add_common(o, d_frames + start_off, ld_frames, 1, dw, start_sample, eff, gain, s);
}

int crlot_ola_push_frame_aos_device(crlot_ola* o, const float* d_interleaved, const float* d_window,
                                    int64_t start_sample, int64_t start_off, int64_t size, float gain,
                                    void* stream) {
    if (!o) return fail(CRLOT_EINVAL, "null OLA object");
    if (!d_interleaved) return fail(CRLOT_EINVAL, "Interleaved input pointer cannot be null");
    if (start_sample < 0 || start_off < 0 || size < 0) return fail(CRLOT_EINVAL, "negative position");
    int64_t eff = 0;
    if (!clamp(o, start_off, size, &eff)) return CRLOT_OK;
    DeviceGuard g(o->device);
    if (const int rc = ensure_real(o); rc != CRLOT_OK) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);  // NULL: the default stream (crlot_dsp.h)
    hipError_t e = use_stream(o, s);
    if (e != hipSuccess) return hip_fail(e, "stream order");
    const bool uw = use_window(o, d_window != nullptr);
    const float* dw = !uw ? nullptr : o->cfg.apply_window_inside ? o->d_win : d_window;  // from index 0
    return add_common(o, d_interleaved + start_off * o->C(), 1, o->C(), dw, start_sample, eff, gain, s);
}

// produce (OLAAccumulator.cc:162-221): *n_out = samples provided
int crlot_ola_produce(crlot_ola* o, float* const* ch_out, int64_t n, int64_t* n_out) {
    if (n_out) *n_out = 0;
    if (!o) return fail(CRLOT_EINVAL, "null OLA object");
    if (!ch_out) return fail(CRLOT_EINVAL, "Output channel buffer cannot be null");
    if (n < 0) return fail(CRLOT_EINVAL, "negative count");
    if (n == 0) return CRLOT_OK;
    for (int64_t c = 0; c < o->C(); ++c)
        if (!ch_out[c]) return fail(CRLOT_EINVAL, "Output channel buffer cannot be null");
    o->last_req_n = n;
    const int64_t avail = o->produced > o->read_pos ? o->produced - o->read_pos : 0;
    if (avail == 0) return CRLOT_OK;
    n = std::min(n, avail);
    const int64_t len = std::min(n, o->R);  // split() clamps to capacity
    DeviceGuard g(o->device);
    int rc = to_server(o);
    if (rc != CRLOT_OK) return rc;
    ServerLock lk(o);
    if (o->vb) {
        rc = batch_produce(o, ch_out[0], n);
        if (rc < 0) return rc;
        if (rc == 0 && (rc = ola_materialize(o)) != CRLOT_OK) return rc;
        if (rc == 1) {
            o->read_pos = (o->read_pos + n) % o->R;  // :213
            o->host_peak = std::max(o->host_peak, peak_of(ch_out[0], n));
            if (n_out) *n_out = n;
            return CRLOT_OK;
        }
    }
    crlot::CallServer* sv = o->srv;
    const int64_t C = o->C();
    const bool hit = o->spec.valid && o->spec.index == sv->submitted() && o->spec.rp == o->read_pos &&
                     o->spec.n == len && sv->live(o->spec.slot);
    o->spec.valid = false;
    if (!hit && (rc = sv->grow(size_t(C * o->N() + o->N()), size_t(C * len), size_t(C * len))) != CRLOT_OK)
        return rc;
    crlot::CallReq r{};
    r.op = crlot::kCallOlaProduce;
    r.win_off = -1;
    r.channels = int32_t(C);
    r.p1 = o->d_den;
    r.p2 = o->d_ring;
    r.i[0] = o->R;
    r.i[1] = o->read_pos % o->R;
    r.i[2] = len;
    if (hit) {
        // served from the block speculated after the last add (the same bits); the
        // ring is cleared by the next request (mono: deferred onto it)
        if ((rc = o->spec.chain ? sv->wait_chain(o->spec.index) : sv->wait_spec(o->spec.index)) != CRLOT_OK)
            return rc;
        for (int64_t c = 0; c < C; ++c)
            std::memcpy(ch_out[c], o->spec.slot.spec + c * len, sizeof(float) * size_t(len));
        if (C == 1) {
            crlot::CallReq::Pend pe{};
            pe.flags = crlot::kPendClear;
            pe.ring = o->d_ring;
            pe.R = o->R;
            pe.rp = o->read_pos % o->R;
            pe.n = len;
            if ((rc = sv->defer(pe)) != CRLOT_OK) return rc;
        } else {
            crlot::CallSlot sl;
            if ((rc = sv->next_slot(&sl)) != CRLOT_OK) return rc;
            r.flags = crlot::kCallClearOnly;
            if ((rc = sv->submit(r, sl)) != CRLOT_OK) return rc;
        }
    } else {
        crlot::CallSlot sl;
        if ((rc = sv->next_slot(&sl)) != CRLOT_OK) return rc;
        if ((rc = sv->submit(r, sl)) != CRLOT_OK) return rc;
        if ((rc = sv->wait(sl.index)) != CRLOT_OK) return rc;
        for (int64_t c = 0; c < C; ++c) std::memcpy(ch_out[c], sl.out + c * len, sizeof(float) * size_t(len));
    }
    o->read_pos = (o->read_pos + n) % o->R;  // :213
    o->host_peak = std::max(o->host_peak, peak_of(ch_out[0], n));  // update_peak_meter (:289-295), channel 0
    if (n_out) *n_out = n;
    return CRLOT_OK;
}

int crlot_ola_produce_device(crlot_ola* o, float* d_out, int64_t ld_out, int64_t n, int64_t* n_out,
                             void* stream) {
    if (n_out) *n_out = 0;
    if (!o) return fail(CRLOT_EINVAL, "null OLA object");
    if (!d_out) return fail(CRLOT_EINVAL, "Output channel buffer cannot be null");
    if (n < 0) return fail(CRLOT_EINVAL, "negative count");
    if (n == 0) return CRLOT_OK;
    const int64_t avail = o->produced > o->read_pos ? o->produced - o->read_pos : 0;
    if (avail == 0) return CRLOT_OK;
    n = std::min(n, avail);
    if (o->C() > 1 && ld_out < n) return fail(CRLOT_EINVAL, "leading dimension too small");
    const int64_t len = std::min(n, o->R);
    DeviceGuard g(o->device);
    if (const int rc = ensure_real(o); rc != CRLOT_OK) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);  // NULL: the default stream (crlot_dsp.h)
    hipError_t e = use_stream(o, s);
    if (e != hipSuccess) return hip_fail(e, "stream order");
    e = crlot::launch_ola_produce(o->d_ring, int(o->C()), o->R, o->d_den, d_out, ld_out, o->read_pos % o->R,
                                  len, n, o->d_peak, s);
    if (e != hipSuccess) return hip_fail(e, "OLA produce kernel launch");
    o->read_pos = (o->read_pos + n) % o->R;
    if (n_out) *n_out = n;
    return CRLOT_OK;
}

// flush (OLAAccumulator.cc:223-228): only the counters move
int crlot_ola_flush(crlot_ola* o) {
    if (!o) return fail(CRLOT_EINVAL, "null OLA object");
    o->flushing = true;
    o->produced = std::max(o->produced, o->read_pos + o->N());
    return CRLOT_OK;
}

// reset (OLAAccumulator.cc:230-247): zero rings and counters, drop the window
int crlot_ola_reset(crlot_ola* o) {
    if (!o) return fail(CRLOT_EINVAL, "null OLA object");
    DeviceGuard g(o->device);
    if (o->vb) {  // the ring is zeroed below: a virtual one needs no rebuild
        ServerLock lk(o);
        if (o->vb->ola == o) o->vb->ola = nullptr;
        o->vb = nullptr;
    }
    hipError_t e = use_stream(o, o->own);
    if (e != hipSuccess) return hip_fail(e, "stream order");
    if ((e = hipMemsetAsync(o->d_ring, 0, sizeof(float) * size_t(o->C() * o->R), o->own)) ||
        (e = hipMemsetAsync(o->d_peak, 0, sizeof(unsigned), o->own)))
        return hip_fail(e, "OLA reset");
    o->read_pos = o->produced = 0;
    o->host_peak = 0.0f;
    o->flushing = false;
    o->window.clear();
    o->last_start = -1;
    o->last_req_n = 0;
    o->spec.valid = false;
    o->pristine = true;
    if (o->srv) o->srv->unpoison(o->d_ring);  // (the zeroed ring is known again)
    return upload_norm(o, o->own);
}

int crlot_ola_info(const crlot_ola* o, int64_t* produced_samples, int64_t* read_pos, int64_t* ring_size,
                   int32_t* has_window) {
    if (!o) return fail(CRLOT_EINVAL, "null OLA object");
    if (produced_samples) *produced_samples = o->produced;
    if (read_pos) *read_pos = o->read_pos;
    if (ring_size) *ring_size = o->R;
    if (has_window) *has_window = o->window.empty() ? 0 : 1;
    return CRLOT_OK;
}

int crlot_ola_meter_peak(crlot_ola* o, float* peak) {
    if (!o || !peak) return fail(CRLOT_EINVAL, "null argument");
    DeviceGuard g(o->device);
    unsigned bits = 0;
    hipError_t e;
    if (o->last_set && (e = hipStreamSynchronize(o->last)) != hipSuccess) return hip_fail(e, "sync");
    if ((e = hipMemcpy(&bits, o->d_peak, sizeof(bits), hipMemcpyDeviceToHost)) != hipSuccess)
        return hip_fail(e, "peak readback");
    float dp;
    std::memcpy(&dp, &bits, sizeof(dp));
    *peak = std::max(o->host_peak, dp);
    return CRLOT_OK;
}

int crlot_ola_norm_table(const crlot_ola* o, float* out) {
    if (!o || !out) return fail(CRLOT_EINVAL, "null argument");
    std::memcpy(out, o->norm.data(), sizeof(float) * size_t(o->R));
    return CRLOT_OK;
}

int crlot_ola_synchronize(crlot_ola* o) {
    if (!o) return fail(CRLOT_EINVAL, "null OLA object");
    DeviceGuard g(o->device);
    if (const int rc = ensure_real(o); rc != CRLOT_OK) return rc;
    if (o->mode == 2) {
        ServerLock lk(o);
        return o->srv->drain();
    }
    hipError_t e = o->last_set ? hipStreamSynchronize(o->last) : hipSuccess;
    return e == hipSuccess ? CRLOT_OK : hip_fail(e, "sync");
}

}  // extern "C"

// =================================================================== OLA kernels (free functions)
// dsp::axpy / axpy_windowed / normalize_and_clear (kernels.h:28-53): batched
// device forms over rows of n elements (ola.hip).  The reference's host-pointer
// signatures are served by the resident call path (call_rt.hip).
extern "C" {

int crlot_axpy(float* d_dst, const float* d_src, float g, int64_t n, int64_t batch, int64_t ld_dst,
               int64_t ld_src, void* stream) {
    if (n < 0 || batch < 0) return fail(CRLOT_EINVAL, "negative size");
    if (n == 0 || batch == 0) return CRLOT_OK;
    if (!d_dst || !d_src) return fail(CRLOT_EINVAL, "null buffer");
    if (batch > 1 && (ld_dst < n || ld_src < n)) return fail(CRLOT_EINVAL, "leading dimension too small");
    if (batch > 65535) return fail(CRLOT_EUNSUPPORTED, "batch above 65535 rows");
    hipError_t e = crlot::launch_axpy(d_dst, ld_dst, d_src, ld_src, nullptr, g, n, batch,
                                      static_cast<hipStream_t>(stream));
    return e == hipSuccess ? CRLOT_OK : hip_fail(e, "axpy kernel launch");
}

int crlot_axpy_windowed(float* d_dst, const float* d_src, const float* d_win, float g, int64_t n, int64_t batch,
                        int64_t ld_dst, int64_t ld_src, void* stream) {
    if (n < 0 || batch < 0) return fail(CRLOT_EINVAL, "negative size");
    if (n == 0 || batch == 0) return CRLOT_OK;
    if (!d_dst || !d_src || !d_win) return fail(CRLOT_EINVAL, "null buffer");
    if (batch > 1 && (ld_dst < n || ld_src < n)) return fail(CRLOT_EINVAL, "leading dimension too small");
    if (batch > 65535) return fail(CRLOT_EUNSUPPORTED, "batch above 65535 rows");
    hipError_t e = crlot::launch_axpy(d_dst, ld_dst, d_src, ld_src, d_win, g, n, batch,
                                      static_cast<hipStream_t>(stream));
    return e == hipSuccess ? CRLOT_OK : hip_fail(e, "axpy_windowed kernel launch");
}

int crlot_normalize_and_clear(float* d_out, float* d_acc, const float* d_norm, float eps, int64_t n, int64_t batch,
                              int64_t ld_out, int64_t ld_acc, void* stream) {
    if (n < 0 || batch < 0) return fail(CRLOT_EINVAL, "negative size");
    if (n == 0 || batch == 0) return CRLOT_OK;
    if (!d_out || !d_acc || !d_norm) return fail(CRLOT_EINVAL, "null buffer");
    if (batch > 1 && (ld_out < n || ld_acc < n)) return fail(CRLOT_EINVAL, "leading dimension too small");
    if (batch > 65535) return fail(CRLOT_EUNSUPPORTED, "batch above 65535 rows");
    hipError_t e = crlot::launch_normalize_and_clear(d_out, ld_out, d_acc, ld_acc, d_norm, eps, n, batch,
                                                     static_cast<hipStream_t>(stream));
    return e == hipSuccess ? CRLOT_OK : hip_fail(e, "normalize_and_clear kernel launch");
}

}  // extern "C"

// =================================================================== FrameQueue
// dsp::FrameQueue (FrameQueue.h:35-59, FrameQueue.cc:9-115): every frame of a
// whole signal materialised at construction, AoS [frame][N].  Frames are built
// on the device (k_fq_frames, ola.hip) and kept there (device_frames: the
// GPU-native input of batched transforms); the reference's host-pointer
// accessors read a host copy taken at construction.
constexpr size_t kFqPinnedMax = size_t(16) << 20;

struct crlot_framequeue {
    int device = 0;
    int64_t n = 0, h = 0, f = 0;
    // [frame][n] (getFrame / getAllFrames): a pooled pinned block up to
    // kFqPinnedMax bytes (no page faults on a fresh queue, a direct DMA for the
    // device copy), plain heap memory beyond
    float* frames = nullptr;
    size_t count = 0, cap = 0;
    bool pinned = false;
    // the same frames in HBM, uploaded at the first device_frames() (the GPU-native
    // input of batched transforms; the host-pointer accessors never need it)
    mutable std::mutex dmu;
    mutable float* d_frames = nullptr;
};

namespace {
// the FrameQueue frame read last through the host accessors (batch.h
// framequeue_last_rows); cleared when that queue dies
const crlot_framequeue* g_last_fq = nullptr;
int64_t g_last_fq_idx = -1;
void note_fq_read(const crlot_framequeue* q, int64_t idx) {
    std::lock_guard<std::mutex> lk(g_pop_mu);
    g_last_fq = q;
    g_last_fq_idx = idx;
}
}  // namespace

namespace crlot {
bool fresh_ola(int64_t n, int64_t h, int device, hipStream_t s, FreshOla* out) {
    std::lock_guard<std::mutex> lk(g_fresh_mu);
    crlot_ola* o = g_fresh_ola;
    if (!o || !o->pristine || o->vb || o->mode == 2 || o->flushing || o->C() != 1 || o->N() != n || o->H() != h ||
        o->device != device || !o->cfg.apply_window_inside || o->window.empty() || o->R < o->N())
        return false;
    // s after the tables' upload (the object's current stream; use_stream's pattern)
    if (hipEventRecord(o->order, o->last_set ? o->last : o->own) != hipSuccess ||
        hipStreamWaitEvent(s, o->order, 0) != hipSuccess)
        return false;
    out->o = o;
    out->d_win = o->d_win;
    out->d_den = o->d_den;
    out->R = o->R;
    out->tgen = o->tgen;
    return true;
}

bool framequeue_last_rows(int64_t n, int64_t max_frames, const std::function<bool(const float*)>& accept,
                          int64_t* hop, int64_t* frames, int64_t* total, int* device, uint64_t* source,
                          int64_t* first, const std::function<float*(size_t)>& dst) {
    std::lock_guard<std::mutex> lk(g_pop_mu);
    const crlot_framequeue* q = g_last_fq;
    if (!q || q->n != n || g_last_fq_idx < 0 || g_last_fq_idx >= q->f) return false;
    const int64_t i = g_last_fq_idx;
    if (!accept(q->frames + size_t(i) * size_t(n))) return false;  // (row 0 first: no copy for a miss)
    const int64_t F = std::min(q->f - i, std::max<int64_t>(1, max_frames));
    const size_t floats = size_t(F) * size_t(n);
    float* d = dst(floats);
    if (!d) return false;
    std::memcpy(d, q->frames + size_t(i) * size_t(n), sizeof(float) * floats);
    *hop = q->h;
    *frames = F;
    *total = q->f - i;
    *device = q->device;
    *source = reinterpret_cast<uintptr_t>(q);
    *first = i;
    return true;
}
}  // namespace crlot

namespace {
// FrameQueue::calculateNumFrames on the padded length (FrameQueue.cc:98-115)
int64_t fq_count(int64_t T, int64_t n, int64_t h, bool center) {
    const int64_t padded = T + (center ? 2 * (n / 2) : 0);
    if (padded < n) return 0;
    const int64_t tail = n > h ? n - h : 0;
    return (padded - tail) / h;
}
}  // namespace

extern "C" {

int64_t crlot_framequeue_count(int64_t T, int64_t frame_size, int64_t hop_size, int32_t center) {
    if (T < 0 || frame_size <= 0 || hop_size <= 0) return fail(CRLOT_EINVAL, "bad argument");
    return fq_count(T, frame_size, hop_size, center != 0);
}

int crlot_framequeue_frames(const float* d_x, int32_t n_streams, int64_t T, int64_t ld_x, int64_t frame_size,
                            int64_t hop_size, int32_t center, int32_t pad_mode, float* d_frames, void* stream) {
    if (frame_size <= 0) return fail(CRLOT_EINVAL, "Frame size must be greater than 0");
    if (hop_size <= 0) return fail(CRLOT_EINVAL, "Hop size must be greater than 0");
    if (n_streams < 0 || T < 0 || (n_streams > 1 && ld_x < T)) return fail(CRLOT_EINVAL, "bad size");
    if (pad_mode < CRLOT_PAD_CONSTANT || pad_mode > CRLOT_PAD_EDGE) return fail(CRLOT_EINVAL, "Unknown pad mode");
    if (!d_x && T > 0) return fail(CRLOT_EINVAL, "Input pointer cannot be null when length > 0");
    const int64_t F = fq_count(T, frame_size, hop_size, center != 0);
    if (F == 0 || n_streams == 0) return CRLOT_OK;
    if (!d_frames) return fail(CRLOT_EINVAL, "null buffer");
    hipError_t e = crlot::launch_fq_frames(d_x, T, ld_x, n_streams, d_frames, F, frame_size, hop_size,
                                           center ? frame_size / 2 : 0, pad_mode, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? CRLOT_OK : hip_fail(e, "FrameQueue kernel launch");
}

int crlot_framequeue_create(const float* in, int64_t len, int64_t frame_size, int64_t hop_size, int32_t center,
                            int32_t pad_mode, int32_t device, crlot_framequeue** out) {
    if (!out) return fail(CRLOT_EINVAL, "null argument");
    *out = nullptr;
    // FrameQueue.cc:13-22
    if (frame_size <= 0) return fail(CRLOT_EINVAL, "Frame size must be greater than 0");
    if (hop_size <= 0) return fail(CRLOT_EINVAL, "Hop size must be greater than 0");
    if (!in && len > 0) return fail(CRLOT_EINVAL, "Input pointer cannot be null when length > 0");
    if (len < 0) return fail(CRLOT_EINVAL, "negative length");
    if (pad_mode < CRLOT_PAD_CONSTANT || pad_mode > CRLOT_PAD_EDGE) return fail(CRLOT_EINVAL, "Unknown pad mode");
    crlot_framequeue* q = new crlot_framequeue();
    if (device < 0) {
        if (hipGetDevice(&q->device) != hipSuccess) {
            delete q;
            return fail(CRLOT_EHIP, "no HIP device");
        }
    } else {
        q->device = device;
    }
    q->n = frame_size;
    q->h = hop_size;
    q->f = fq_count(len, frame_size, hop_size, center != 0);
    // The frames on the host, as FrameQueue.cc:69-96 builds them (the same
    // indexing as the device form k_fq_frames, ola.hip: copies, so the same bits):
    // a host-pointer class serves host memory, and framing a whole signal is one
    // pass of copies, cheaper here than a device round trip.
    const size_t nf = size_t(q->f) * size_t(q->n);
    q->count = nf;
    if (nf > 0) {
        void* hb = nullptr;
        if (sizeof(float) * nf <= kFqPinnedMax && crlot::pool_pinned(sizeof(float) * nf, &hb, &q->cap) == hipSuccess) {
            q->frames = static_cast<float*>(hb);
            q->pinned = true;
        } else {
            q->frames = new (std::nothrow) float[nf];
            if (!q->frames) {
                delete q;
                return fail(CRLOT_ENOMEM, "FrameQueue allocation");
            }
        }
    }
    const int64_t pad = center ? frame_size / 2 : 0;
    for (int64_t k = 0; k < q->f; ++k) {
        float* dst = q->frames + size_t(k) * size_t(q->n);
        const int64_t o = k * hop_size - pad;
        const int64_t j0 = std::max<int64_t>(0, -o), j1 = std::min<int64_t>(frame_size, len - o);
        if (j1 > j0) std::memcpy(dst + j0, in + o + j0, sizeof(float) * size_t(j1 - j0));
        for (int64_t j = 0; j < frame_size; ++j) {
            if (j >= j0 && j < j1) continue;
            const int64_t idx = o + j;
            float v = 0.0f;
            if (len > 0 && pad_mode == CRLOT_PAD_REFLECT) {
                int64_t i = idx;  // reflect101 (Indexing.h:18-33)
                if (len > 1)
                    while (i < 0 || i >= len) i = i < 0 ? -i - 1 : 2 * len - 2 - i;
                else
                    i = 0;
                v = in[i];
            } else if (len > 0 && pad_mode == CRLOT_PAD_EDGE) {
                v = in[idx < 0 ? 0 : len - 1];
            }
            dst[j] = v;
        }
    }
    *out = q;
    return CRLOT_OK;
}

void crlot_framequeue_destroy(crlot_framequeue* q) {
    if (!q) return;
    {
        std::lock_guard<std::mutex> lk(g_pop_mu);
        if (g_last_fq == q) g_last_fq = nullptr;
    }
    if (q->d_frames) {  // (the caller finished its device-side reads of the frames)
        DeviceGuard g(q->device);
        (void)hipFree(q->d_frames);
    }
    if (q->pinned)
        crlot::pool_pinned_put(q->frames, q->cap);
    else
        delete[] q->frames;
    delete q;
}

int crlot_framequeue_info(const crlot_framequeue* q, int64_t* num_frames, int64_t* frame_size, int64_t* hop_size) {
    if (!q) return fail(CRLOT_EINVAL, "null FrameQueue");
    if (num_frames) *num_frames = q->f;
    if (frame_size) *frame_size = q->n;
    if (hop_size) *hop_size = q->h;
    return CRLOT_OK;
}

const float* crlot_framequeue_frame(const crlot_framequeue* q, int64_t frame_idx) {
    if (!q) {
        fail(CRLOT_EINVAL, "null FrameQueue");
        return nullptr;
    }
    if (frame_idx < 0 || frame_idx >= q->f) {  // FrameQueue.cc:49-54
        fail(CRLOT_ERANGE, "Frame index out of range");
        return nullptr;
    }
    note_fq_read(q, frame_idx);
    return q->frames + size_t(frame_idx) * size_t(q->n);
}

int crlot_framequeue_copy_frame(const crlot_framequeue* q, int64_t frame_idx, float* out) {
    if (!q) return fail(CRLOT_EINVAL, "null FrameQueue");
    if (frame_idx < 0 || frame_idx >= q->f) return fail(CRLOT_ERANGE, "Frame index out of range");
    if (!out) return fail(CRLOT_EINVAL, "Output buffer cannot be null");  // FrameQueue.cc:56-67
    note_fq_read(q, frame_idx);
    std::memcpy(out, q->frames + size_t(frame_idx) * size_t(q->n), sizeof(float) * size_t(q->n));
    return CRLOT_OK;
}

const float* crlot_framequeue_all_frames(const crlot_framequeue* q) { return q ? q->frames : nullptr; }

const float* crlot_framequeue_device_frames(const crlot_framequeue* q) {
    if (!q) return nullptr;
    std::lock_guard<std::mutex> lk(q->dmu);
    if (!q->d_frames && q->count > 0) {  // uploaded on first use, then kept
        DeviceGuard g(q->device);
        const size_t bytes = sizeof(float) * q->count;
        void* d = nullptr;
        hipError_t e = hipMalloc(&d, bytes);
        if (e == hipSuccess) e = hipMemcpy(d, q->frames, bytes, hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            if (d) (void)hipFree(d);
            hip_fail(e, "FrameQueue device frames");
            return nullptr;
        }
        q->d_frames = static_cast<float*>(d);
    }
    return q->d_frames;
}

}  // extern "C"
