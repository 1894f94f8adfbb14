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
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

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
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (dev >= 0 && dev != prev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
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

extern "C" {

int crlot_framer_create(crlot_framer** out) {
    if (!out) return fail(CRLOT_EINVAL, "null argument");
    *out = new crlot_framer();
    return CRLOT_OK;
}

void crlot_framer_destroy(crlot_framer* f) { delete f; }

int crlot_framer_set_params(crlot_framer* f, int64_t frame_size, int64_t hop_size, int64_t channels,
                            int32_t boundary_mode) {
    if (!f) return fail(CRLOT_EINVAL, "null framer");
    if (frame_size <= 0) return fail(CRLOT_EINVAL, "Frame size must be greater than 0");
    if (hop_size <= 0) return fail(CRLOT_EINVAL, "Hop size must be greater than 0");
    if (channels <= 0) return fail(CRLOT_EINVAL, "Channels must be greater than 0");
    if (boundary_mode != CRLOT_ZERO_PAD && boundary_mode != CRLOT_DROP)
        return fail(CRLOT_EINVAL, "Unknown boundary mode");
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
    const int64_t need = f->wr + add;
    if (int64_t(f->buf.size()) < need)  // doubling growth (framer.cc:120-126)
        f->buf.resize(size_t(std::max<int64_t>(need, 2 * int64_t(f->buf.size()))), 0.0f);
    std::memcpy(f->buf.data() + f->wr, interleaved, sizeof(float) * size_t(add));
    f->wr = need;
    return 1;
}

int crlot_framer_pop(crlot_framer* f, float* out) {
    if (!f) return fail(CRLOT_EINVAL, "null framer");
    if (!f->ready || !out || f->available() == 0) return 0;
    const int64_t len = f->n * f->c;     // extract_frame (framer.cc:128-181)
    const int64_t have = f->wr - f->rd;
    if (have >= len) {
        std::memcpy(out, f->buf.data() + f->rd, sizeof(float) * size_t(len));
    } else {
        if (f->mode == CRLOT_DROP) return 0;
        std::memcpy(out, f->buf.data() + f->rd, sizeof(float) * size_t(have));
        std::fill(out + have, out + len, 0.0f);
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
    float* d_in = nullptr;            // staged frame: C*N samples + N window values
    float* d_out = nullptr;           // produce staging [C][R]
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
    float* h_out = nullptr;           // pinned produce landing [C][R]

    int64_t N() const { return cfg.frame_size; }
    int64_t H() const { return cfg.hop_size; }
    int64_t C() const { return cfg.channels; }
};

namespace {

void ola_free(crlot_ola* o) {
    if (!o) return;
    DeviceGuard g(o->device);
    if (o->own) (void)hipStreamSynchronize(o->own);
    if (o->last_set && o->last) (void)hipStreamSynchronize(o->last);
    for (auto& s : o->slot) {
        if (s.ev) (void)hipEventDestroy(s.ev);
        if (s.h) (void)hipHostFree(s.h);
    }
    for (float* p : {o->d_ring, o->d_den, o->d_win, o->d_in, o->d_out})
        if (p) (void)hipFree(p);
    if (o->d_peak) (void)hipFree(o->d_peak);
    if (o->h_out) (void)hipHostFree(o->h_out);
    if (o->order) (void)hipEventDestroy(o->order);
    if (o->own) (void)hipStreamDestroy(o->own);
    delete o;
}

// Make `s` the object's stream, ordered after everything issued on the previous one.
hipError_t use_stream(crlot_ola* o, hipStream_t s) {
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
    if (!s.ev && (e = hipEventCreateWithFlags(&s.ev, hipEventDisableTiming)) != hipSuccess) return e;
    if (s.cap < floats) {
        if (s.h) (void)hipHostFree(s.h);
        s.h = nullptr;
        s.cap = 0;
        if ((e = hipHostMalloc(reinterpret_cast<void**>(&s.h), floats * sizeof(float))) != hipSuccess) return e;
        s.cap = floats;
    }
    *out = &s;
    return hipSuccess;
}

// OLAAccumulator::initialize_normalization (OLAAccumulator.cc:260-288) -> den
// on the device, ordered on the object's current stream.
int upload_norm(crlot_ola* o, hipStream_t s) {
    const bool has_w = !o->window.empty();
    crlot_norm_table(has_w ? o->window.data() : nullptr, o->N(), o->H(), o->R,
                     o->cfg.apply_window_inside, o->cfg.eps, o->norm.data());
    crlot_ola::Slot* sl = nullptr;
    hipError_t e = take_slot(o, size_t(o->R + o->N()), &sl);
    if (e != hipSuccess) return hip_fail(e, "staging");
    const float eps = o->cfg.eps;
    for (int64_t i = 0; i < o->R; ++i)  // normalize_and_clear's guard (kernels.cc:32)
        sl->h[i] = (o->norm[i] > eps) ? o->norm[i] : eps;
    if (has_w) std::memcpy(sl->h + o->R, o->window.data(), sizeof(float) * size_t(o->N()));
    if ((e = hipMemcpyAsync(o->d_den, sl->h, sizeof(float) * size_t(o->R), hipMemcpyHostToDevice, s)) ||
        (has_w && (e = hipMemcpyAsync(o->d_win, sl->h + o->R, sizeof(float) * size_t(o->N()),
                                      hipMemcpyHostToDevice, s))) ||
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
    if (nch < o->C()) return CRLOT_OK;  // caller reports the null channel
    o->produced = std::max(o->produced, start_sample + eff);  // :114
    return CRLOT_OK;
}

// stage `floats` host values (frames, then optionally a window slice) and copy
// them to d_in on the object's own stream
int stage_in(crlot_ola* o, const std::vector<std::pair<const float*, int64_t>>& parts) {
    size_t total = 0;
    for (auto& p : parts) total += size_t(p.second);
    crlot_ola::Slot* sl = nullptr;
    hipError_t e = take_slot(o, total, &sl);
    if (e != hipSuccess) return hip_fail(e, "staging");
    size_t at = 0;
    for (auto& p : parts) {
        std::memcpy(sl->h + at, p.first, sizeof(float) * size_t(p.second));
        at += size_t(p.second);
    }
    if ((e = hipMemcpyAsync(o->d_in, sl->h, sizeof(float) * total, hipMemcpyHostToDevice, o->own)) ||
        (e = hipEventRecord(sl->ev, o->own)))
        return hip_fail(e, "frame upload");
    sl->pending = true;
    return CRLOT_OK;
}

}  // namespace

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
    if ((e = hipStreamCreateWithFlags(&o->own, hipStreamNonBlocking)) ||
        (e = hipEventCreateWithFlags(&o->order, hipEventDisableTiming)) ||
        (e = hipMalloc(&o->d_ring, sizeof(float) * C * R)) || (e = hipMalloc(&o->d_den, sizeof(float) * R)) ||
        (e = hipMalloc(&o->d_win, sizeof(float) * N)) || (e = hipMalloc(&o->d_in, sizeof(float) * (C + 1) * N)) ||
        (e = hipMalloc(&o->d_out, sizeof(float) * C * R)) || (e = hipMalloc(&o->d_peak, sizeof(unsigned))) ||
        (e = hipHostMalloc(reinterpret_cast<void**>(&o->h_out), sizeof(float) * C * R))) {
        ola_free(o);
        return e == hipErrorOutOfMemory ? fail(CRLOT_ENOMEM, "OLA object allocation")
                                        : hip_fail(e, "OLA object allocation");
    }
    if ((e = hipMemsetAsync(o->d_ring, 0, sizeof(float) * C * R, o->own)) ||
        (e = hipMemsetAsync(o->d_peak, 0, sizeof(unsigned), o->own))) {
        ola_free(o);
        return hip_fail(e, "OLA object init");
    }
    (void)use_stream(o, o->own);
    int rc = upload_norm(o, o->own);  // no window yet: all ones
    if (rc == CRLOT_OK && (e = hipStreamSynchronize(o->own)) != hipSuccess) rc = hip_fail(e, "OLA init");
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
    o->window.assign(w, w + wlen);
    hipError_t e = use_stream(o, o->own);
    if (e != hipSuccess) return hip_fail(e, "stream order");
    return upload_norm(o, o->own);
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
    hipError_t e = use_stream(o, o->own);
    if (e != hipSuccess) return hip_fail(e, "stream order");
    const bool uw = use_window(o, window != nullptr);
    const bool caller_win = uw && !o->cfg.apply_window_inside;
    std::vector<std::pair<const float*, int64_t>> parts;
    for (int64_t c = 0; c < ok; ++c) parts.push_back({ch_frames[c] + start_off, eff});
    if (caller_win) parts.push_back({window + start_off, eff});
    int rc = stage_in(o, parts);
    if (rc != CRLOT_OK) return rc;
    const float* dw = !uw ? nullptr : caller_win ? o->d_in + ok * eff : o->d_win + start_off;
    rc = add_common(o, o->d_in, eff, 1, dw, start_sample, eff, gain, o->own, ok);
    if (rc != CRLOT_OK) return rc;
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
    hipError_t e = use_stream(o, o->own);
    if (e != hipSuccess) return hip_fail(e, "stream order");
    // push_frame_AoS deinterleaves [start_off, start_off + eff) and calls
    // add_frame_SoA with start_off = 0, so the window is read from index 0
    // (OLAAccumulator.cc:146-159)
    const bool uw = use_window(o, window != nullptr);
    const bool caller_win = uw && !o->cfg.apply_window_inside;
    std::vector<std::pair<const float*, int64_t>> parts{{interleaved + start_off * o->C(), eff * o->C()}};
    if (caller_win) parts.push_back({window, eff});
    int rc = stage_in(o, parts);
    if (rc != CRLOT_OK) return rc;
    const float* dw = !uw ? nullptr : caller_win ? o->d_in + o->C() * eff : o->d_win;
    return add_common(o, o->d_in, 1, o->C(), dw, start_sample, eff, gain, o->own);
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
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : o->own;
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
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : o->own;
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
    const int64_t avail = o->produced > o->read_pos ? o->produced - o->read_pos : 0;
    if (avail == 0) return CRLOT_OK;
    n = std::min(n, avail);
    const int64_t len = std::min(n, o->R);  // split() clamps to capacity
    DeviceGuard g(o->device);
    hipError_t e = use_stream(o, o->own);
    if (e != hipSuccess) return hip_fail(e, "stream order");
    if ((e = crlot::launch_ola_produce(o->d_ring, int(o->C()), o->R, o->d_den, o->d_out, len,
                                       o->read_pos % o->R, len, len, nullptr, o->own)) ||
        (e = hipMemcpyAsync(o->h_out, o->d_out, sizeof(float) * size_t(len * o->C()), hipMemcpyDeviceToHost,
                            o->own)) ||
        (e = hipStreamSynchronize(o->own)))
        return hip_fail(e, "OLA produce");
    for (int64_t c = 0; c < o->C(); ++c)
        std::memcpy(ch_out[c], o->h_out + c * len, sizeof(float) * size_t(len));
    o->read_pos = (o->read_pos + n) % o->R;  // :213
    for (int64_t i = 0; i < n; ++i) {        // update_peak_meter (:289-295), channel 0
        const float a = std::fabs(ch_out[0][i]);
        o->host_peak = std::max(o->host_peak, a);
    }
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
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : o->own;
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
    hipError_t e = use_stream(o, o->own);
    if (e != hipSuccess) return hip_fail(e, "stream order");
    if ((e = hipMemsetAsync(o->d_ring, 0, sizeof(float) * size_t(o->C() * o->R), o->own)) ||
        (e = hipMemsetAsync(o->d_peak, 0, sizeof(unsigned), o->own)))
        return hip_fail(e, "OLA reset");
    o->read_pos = o->produced = 0;
    o->host_peak = 0.0f;
    o->flushing = false;
    o->window.clear();
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
    hipError_t e = o->last_set ? hipStreamSynchronize(o->last) : hipSuccess;
    return e == hipSuccess ? CRLOT_OK : hip_fail(e, "sync");
}

}  // extern "C"
