// crlot_dsp.hpp -- C++ host surface over the C ABI (header-only).
//
// Mirrors the reference's C++ API for the hot path so C++ callers drop in:
//   crlot::dsp::Framer             <- dsp::Framer           (framer.h:26-127)
//   crlot::dsp::FrameQueue         <- dsp::FrameQueue       (FrameQueue.h:35-59), device-built frames
//   crlot::dsp::axpy / axpy_windowed / normalize_and_clear
//                                  <- dsp/ola/kernels.h:28-53 (+ batched _device forms)
//   crlot::dsp::OLAConfig          <- dsp::OLAConfig        (OLAAccumulator.h:15-29)
//   crlot::dsp::OLAAccumulator     <- dsp::OLAAccumulator   (OLAAccumulator.h:63-217), device rings
//   crlot::dsp::WindowLUT          <- dsp::WindowLUT        (WindowLUT.h:80-287), incl. the
//                                     GetWindowSafe / GetWindow / getInstance cache
//   crlot::dsp::fft::FftPlanDesc   <- dsp::fft::FftPlanDesc (fft_api.h:16-23)
//   crlot::dsp::fft::IFftPlan      <- dsp::fft::IFftPlan    (fft_api.h:26-48)
//   crlot::dsp::fft::HipFftPlan    <- KissFftPlan (kissfft_adapter.cc:11-264), Real + Complex
//   crlot::dsp::fft::MakeFftPlan   <- dsp::fft::MakeFftPlan (fft_api.h:51), HIP-backed
//   crlot::io::WavReader/WavWriter <- WavReader / WavWriter  (io/wav.h:11-72)
//   crlot::StftEngine              <- the Framer -> window -> FFT -> iFFT -> OLA loop
//                                     of bench/e2e_benchmark.cc:138-186, batched
// Error codes become the reference's exception types: CRLOT_EINVAL ->
// std::invalid_argument, CRLOT_ENOMEM -> std::bad_alloc, everything else ->
// std::runtime_error.  Host-pointer calls stage through device buffers owned by
// the object; device-pointer calls (suffix _device) take HBM-resident data.
#pragma once

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <exception>
#include <complex>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <utility>
#include <vector>

#include "crlot_dsp.h"

namespace crlot {

inline void check(int rc, const char* what) {
    if (rc >= 0) return;
    std::string msg = std::string(what) + ": " + crlot_last_error();
    if (rc == CRLOT_EINVAL) throw std::invalid_argument(msg);
    if (rc == CRLOT_ENOMEM) throw std::bad_alloc();
    if (rc == CRLOT_ERANGE) throw std::out_of_range(msg);
    throw std::runtime_error(msg);
}

inline void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// Device buffer (RAII).
template <typename T>
class DeviceBuffer {
   public:
    DeviceBuffer() = default;
    explicit DeviceBuffer(size_t n) { resize(n); }
    ~DeviceBuffer() {
        if (p_) (void)hipFree(p_);
    }
    DeviceBuffer(const DeviceBuffer&) = delete;
    DeviceBuffer& operator=(const DeviceBuffer&) = delete;
    void resize(size_t n) {
        if (n <= n_) return;
        if (p_) (void)hipFree(p_);
        p_ = nullptr;
        n_ = 0;
        if (hipMalloc(&p_, n * sizeof(T)) != hipSuccess) throw std::bad_alloc();
        n_ = n;
    }
    T* get() const { return p_; }
    size_t size() const { return n_; }

   private:
    T* p_ = nullptr;
    size_t n_ = 0;
};

// Owning plan handle.
class Plan {
   public:
    explicit Plan(const crlot_plan_desc& d) { check(crlot_plan_create(&d, &p_), "crlot_plan_create"); }
    ~Plan() { crlot_plan_destroy(p_); }
    Plan(const Plan&) = delete;
    Plan& operator=(const Plan&) = delete;
    crlot_plan* get() const { return p_; }
    int frame_size() const {
        int32_t n = 0;
        check(crlot_plan_info(p_, &n, nullptr, nullptr), "crlot_plan_info");
        return n;
    }
    int hop_size() const {
        int32_t h = 0;
        check(crlot_plan_info(p_, nullptr, &h, nullptr), "crlot_plan_info");
        return h;
    }

   private:
    crlot_plan* p_ = nullptr;
};

// Batched round trip: n_streams mono streams, each T samples.
class StftEngine {
   public:
    struct Config {
        int frame_size = 1024, hop_size = 256;
        int window_type = CRLOT_WIN_HANN;
        bool periodic = false;
        int boundary_mode = CRLOT_ZERO_PAD;
        bool analysis_window = true, apply_window_inside = true;
        float eps = 1e-8f, gain = 1.0f;
        int device = -1;
        bool center = true;                  // boundary_mode == CRLOT_FRAMEQUEUE
        int pad_mode = CRLOT_PAD_CONSTANT;   // (dsp::FrameQueue defaults)
    };
    explicit StftEngine(const Config& c) : plan_(desc(c)), n_(c.frame_size) {}
    int64_t frame_count(int64_t T) const { return crlot_frame_count(plan_.get(), T); }
    int64_t output_length(int64_t T) const { return crlot_output_length(plan_.get(), T); }
    // d_x [n_streams][ld_x], d_y [n_streams][ld_y] device pointers
    void roundtrip_device(const float* d_x, float* d_y, int n_streams, int64_t T, int64_t ld_x,
                          int64_t ld_y, hipStream_t s = nullptr) {
        check(crlot_roundtrip(plan_.get(), d_x, d_y, n_streams, T, ld_x, ld_y, s), "crlot_roundtrip");
    }
    // host convenience: x [n_streams][T] -> y [n_streams][output_length(T)]
    std::vector<float> roundtrip(const std::vector<float>& x, int n_streams, int64_t T) {
        const int64_t L = output_length(T);
        dx_.resize(size_t(n_streams) * T);
        dy_.resize(size_t(n_streams) * L);
        hip_check(hipMemcpy(dx_.get(), x.data(), sizeof(float) * n_streams * T, hipMemcpyHostToDevice),
                  "hipMemcpy");
        roundtrip_device(dx_.get(), dy_.get(), n_streams, T, T, L);
        std::vector<float> y(size_t(n_streams) * L);
        hip_check(hipMemcpy(y.data(), dy_.get(), sizeof(float) * y.size(), hipMemcpyDeviceToHost),
                  "hipMemcpy");
        return y;
    }
    // groups of `channels` interleaved channels (Framer(N, H, C) PCM): d_x group g
    // at +g*ld_x (T rows of C), d_y group g at +g*ld_y (output_length(T) rows of C)
    void roundtrip_interleaved_device(const float* d_x, float* d_y, int n_groups, int channels, int64_t T,
                                      int64_t ld_x, int64_t ld_y, hipStream_t s = nullptr) {
        check(crlot_roundtrip_interleaved(plan_.get(), d_x, d_y, n_groups, channels, T, ld_x, ld_y, s),
              "crlot_roundtrip_interleaved");
    }
    void set_spectral_gain(const float* gain_or_null) {
        check(crlot_plan_set_spectral_gain(plan_.get(), gain_or_null), "set_spectral_gain");
    }
    // crlot_plan_set_frame_pairing: two frames per complex transform (default) or per frame
    void set_frame_pairing(bool enable) {
        check(crlot_plan_set_frame_pairing(plan_.get(), enable ? 1 : 0), "set_frame_pairing");
    }
    // The round trip split at its spectral step (e2e_benchmark.cc:160-162).
    // Spectra: complex64 rows of frame_size/2 + 1 bins, frame k of stream s at
    // d_spec + s*ld_spec + k*ld_frame floats (ld_frame >= frame_size + 2, even).
    int64_t bins() const { return n_ / 2 + 1; }
    void stft_device(const float* d_x, float* d_spec, int n_streams, int64_t T, int64_t ld_x, int64_t ld_spec,
                     int64_t ld_frame, hipStream_t s = nullptr) {
        check(crlot_stft(plan_.get(), d_x, d_spec, n_streams, T, ld_x, ld_spec, ld_frame, s), "crlot_stft");
    }
    // spectra (F frames per stream) -> gain / mask step -> irfft -> OLA -> y [F * hop]
    void istft_ola_device(const float* d_spec, float* d_y, int n_streams, int64_t F, int64_t ld_spec,
                          int64_t ld_frame, int64_t ld_y, hipStream_t s = nullptr) {
        check(crlot_istft_ola(plan_.get(), d_spec, d_y, n_streams, F, ld_spec, ld_frame, ld_y, s),
              "crlot_istft_ola");
    }
    // per-frame real mask rows of bins(): frame k of stream s at d_mask + s*ld_stream + k*ld_frame
    // (ld_stream 0: one mask shared by the streams); nullptr clears it
    void set_spectral_mask(const float* d_mask_or_null, int64_t ld_frame = 0, int64_t ld_stream = 0) {
        check(crlot_plan_set_spectral_mask(plan_.get(), d_mask_or_null, ld_frame ? ld_frame : bins(), ld_stream),
              "set_spectral_mask");
    }
    crlot_plan* plan() const { return plan_.get(); }

   private:
    static crlot_plan_desc desc(const Config& c) {
        crlot_plan_desc d{};
        d.frame_size = c.frame_size;
        d.hop_size = c.hop_size;
        d.window_type = c.window_type;
        d.periodic = c.periodic;
        d.boundary_mode = c.boundary_mode;
        d.analysis_window = c.analysis_window;
        d.apply_window_inside = c.apply_window_inside;
        d.eps = c.eps;
        d.ola_gain = c.gain;
        d.device = c.device;
        d.center = c.center;
        d.pad_mode = c.pad_mode;
        return d;
    }
    Plan plan_;
    int n_;
    DeviceBuffer<float> dx_, dy_;
};

// Real-time per-hop streaming with hops in host memory (BASELINE config 4):
// the resident kernel behind crlot_stream_rt_*.  push_hop copies one hop of
// channels x H samples in ([H][C] interleaved PCM or [C][H]), returns the H
// output samples per channel in the same layout once the frame completes
// (DROP Framer + push_frame_AoS + produce(H); 0 before N samples arrived).
class RealtimeStream {
   public:
    RealtimeStream(const StftEngine& eng, int channels, bool interleaved, int depth = 4) {
        check(crlot_stream_rt_create(eng.plan(), channels, interleaved ? 1 : 0, depth, &st_),
              "crlot_stream_rt_create");
    }
    ~RealtimeStream() { crlot_stream_rt_destroy(st_); }
    RealtimeStream(const RealtimeStream&) = delete;
    RealtimeStream& operator=(const RealtimeStream&) = delete;
    size_t push_hop(const float* hop_in, float* hop_out) {
        int32_t em = 0;
        check(crlot_stream_rt_push_hop(st_, hop_in, hop_out, &em), "crlot_stream_rt_push_hop");
        return size_t(em);
    }
    void reset() { check(crlot_stream_rt_reset(st_), "crlot_stream_rt_reset"); }
    double last_device_ns() const {
        double ns = 0;
        check(crlot_stream_rt_info(st_, nullptr, &ns, nullptr), "crlot_stream_rt_info");
        return ns;
    }
    crlot_stream_rt* handle() const { return st_; }

   private:
    crlot_stream_rt* st_ = nullptr;
};

// io/wav.h WavReader / WavWriter (same methods; open() returns false on a
// file the reference would reject, crlot_last_error() says why).
namespace io {

class WavReader {
   public:
    WavReader() = default;
    ~WavReader() { close(); }
    WavReader(const WavReader&) = delete;
    WavReader& operator=(const WavReader&) = delete;
    bool open(const std::string& filename) {
        close();
        if (crlot_wav_reader_open(filename.c_str(), &r_) != CRLOT_OK) return false;
        crlot_wav_reader_info(r_, &ch_, &rate_, &frames_, &bits_, nullptr);
        return true;
    }
    void close() {
        if (r_) crlot_wav_reader_close(r_);
        r_ = nullptr;
    }
    bool read(float* buffer, size_t frames_to_read, size_t* frames_read = nullptr) {
        if (!r_) return false;
        uint64_t got = 0;
        if (crlot_wav_reader_read(r_, buffer, frames_to_read, &got) != CRLOT_OK) return false;
        if (frames_read) *frames_read = size_t(got);
        return got > 0 || frames_to_read == 0;
    }
    std::vector<float> read_all() {
        if (!r_) return {};
        std::vector<float> v(size_t(frames_) * ch_);
        uint64_t got = 0;
        if (!v.empty()) crlot_wav_reader_read(r_, v.data(), frames_, &got);
        v.resize(size_t(got) * ch_);
        return v;
    }
    uint32_t get_channels() const { return r_ ? ch_ : 0; }
    uint32_t get_sample_rate() const { return r_ ? rate_ : 0; }
    uint64_t get_total_frames() const { return r_ ? frames_ : 0; }
    uint32_t get_bits_per_sample() const { return r_ ? bits_ : 0; }
    bool is_open() const { return r_ != nullptr; }

   private:
    crlot_wav_reader* r_ = nullptr;
    uint32_t ch_ = 0, rate_ = 0, bits_ = 0;
    uint64_t frames_ = 0;
};

class WavWriter {
   public:
    WavWriter() = default;
    ~WavWriter() { close(); }
    WavWriter(const WavWriter&) = delete;
    WavWriter& operator=(const WavWriter&) = delete;
    bool open(const std::string& filename, uint32_t channels, uint32_t sample_rate,
              uint32_t bits_per_sample = 16, bool float_format = false) {
        close();
        return crlot_wav_writer_open(filename.c_str(), channels, sample_rate, bits_per_sample,
                                     float_format, &w_) == CRLOT_OK;
    }
    void close() {
        if (w_) crlot_wav_writer_close(w_);
        w_ = nullptr;
    }
    bool write(const float* buffer, size_t frames_to_write, size_t* frames_written = nullptr) {
        if (!w_) return false;
        uint64_t put = 0;
        const int rc = crlot_wav_writer_write(w_, buffer, frames_to_write, &put);
        if (frames_written) *frames_written = size_t(put);
        return rc == CRLOT_OK && put == frames_to_write;
    }
    bool is_open() const { return w_ != nullptr; }

   private:
    crlot_wav_writer* w_ = nullptr;
};

}  // namespace io

namespace dsp {

// dsp::base (base/span.h, base/aligned_alloc.h) and dsp::ring::RingBuffer
// (ring/ring_buffer.h:17-117): the host containers the reference's OLA object is
// built on.  The drop-in OLAAccumulator keeps its rings in HBM; these exist so
// code written against the reference's headers (its RingBuffer tests, harness
// helpers) builds and behaves the same.  Semantics per ring_buffer.cc: split()
// clamps the length to the capacity and wraps once; a shadow ring allocates
// twice the capacity and mirrors the head after a wrapping write.
namespace base {
template <typename T>
class Span {
public:
    Span() = default;
    Span(T* p, size_t n) : p_(p), n_(n) {}
    T* data() const { return p_; }
    size_t size() const { return n_; }
    bool empty() const { return n_ == 0; }
    T& operator[](size_t i) const { return p_[i]; }
    T* begin() const { return p_; }
    T* end() const { return p_ + n_; }

private:
    T* p_ = nullptr;
    size_t n_ = 0;
};
// 64-byte aligned storage (aligned_alloc.h:18-45); nullptr for n == 0, bad_alloc on failure
template <typename T>
T* AllocateAligned(size_t n) {
    if (n == 0) return nullptr;
    if (n > SIZE_MAX / sizeof(T)) throw std::bad_alloc();
    void* p = nullptr;
    if (posix_memalign(&p, 64, n * sizeof(T)) != 0) throw std::bad_alloc();
    return static_cast<T*>(p);
}
inline void DeallocateAligned(void* p) { std::free(p); }
// std::allocator with 64-byte alignment (the window tables the reference hands
// out are 32-byte aligned for its SIMD loads: window_lut_test.cc:285-330)
template <typename T>
struct AlignedAllocator {
    using value_type = T;
    AlignedAllocator() = default;
    template <typename U>
    AlignedAllocator(const AlignedAllocator<U>&) {}
    T* allocate(size_t n) { return n ? AllocateAligned<T>(n) : nullptr; }
    void deallocate(T* p, size_t) { DeallocateAligned(p); }
    template <typename U>
    bool operator==(const AlignedAllocator<U>&) const { return true; }
    template <typename U>
    bool operator!=(const AlignedAllocator<U>&) const { return false; }
};
}  // namespace base

namespace ring {
template <typename T>
class RingBuffer {
    static_assert(std::is_trivially_copyable<T>::value, "RingBuffer elements are copied bytewise");

public:
    explicit RingBuffer(size_t capacity, bool shadow = false) : cap_(capacity), shadow_(shadow) {
        if (capacity == 0) throw std::invalid_argument("RingBuffer capacity must be > 0");
        const size_t phys = physical_capacity();
        buf_ = base::AllocateAligned<T>(phys);
        std::fill(buf_, buf_ + phys, T{});
    }
    ~RingBuffer() { base::DeallocateAligned(buf_); }
    RingBuffer(const RingBuffer&) = delete;
    RingBuffer& operator=(const RingBuffer&) = delete;

    size_t capacity() const noexcept { return cap_; }
    size_t physical_capacity() const noexcept { return shadow_ ? 2 * cap_ : cap_; }
    bool has_shadow() const noexcept { return shadow_; }
    size_t write_pos() const noexcept { return wpos_; }
    T* data() noexcept { return buf_; }
    const T* data() const noexcept { return buf_; }

    std::pair<base::Span<T>, base::Span<T>> split(size_t start, size_t len) noexcept {
        const auto r = spans(start, len);
        return {base::Span<T>(r.a, r.na), base::Span<T>(r.b, r.nb)};
    }
    std::pair<base::Span<const T>, base::Span<const T>> split(size_t start, size_t len) const noexcept {
        const auto r = spans(start, len);
        return {base::Span<const T>(r.a, r.na), base::Span<const T>(r.b, r.nb)};
    }
    // mirror elements [0, n) of the ring past its end (shadow rings only)
    void shadow_sync(size_t n) {
        if (shadow_ && n > 0) std::memcpy(buf_ + cap_, buf_, std::min(n, cap_) * sizeof(T));
    }
    T* contiguous_read_ptr(size_t pos) noexcept { return buf_ + (shadow_ ? pos : pos % cap_); }
    const T* contiguous_read_ptr(size_t pos) const noexcept { return buf_ + (shadow_ ? pos : pos % cap_); }
    // n elements at the write position, wrapping once to the head
    size_t write(const T* src, size_t n) {
        if (!src || n == 0) return 0;
        const size_t room = cap_ - wpos_;
        if (n <= room) {
            std::memcpy(buf_ + wpos_, src, n * sizeof(T));
            wpos_ = (wpos_ + n == cap_) ? 0 : wpos_ + n;
            return n;
        }
        std::memcpy(buf_ + wpos_, src, room * sizeof(T));
        const size_t head = std::min(n - room, cap_);
        std::memcpy(buf_, src + room, head * sizeof(T));
        wpos_ = head;
        shadow_sync(head);
        return room + head;
    }

private:
    struct Spans {
        T* a;
        size_t na;
        T* b;
        size_t nb;
    };
    Spans spans(size_t start, size_t len) const noexcept {
        if (len == 0) return {nullptr, 0, nullptr, 0};
        len = std::min(std::min(len, SIZE_MAX - start), cap_);
        start %= cap_;
        if (start + len <= cap_) return {buf_ + start, len, nullptr, 0};
        return {buf_ + start, cap_ - start, buf_, len - (cap_ - start)};
    }
    T* buf_ = nullptr;
    size_t cap_ = 0, wpos_ = 0;
    bool shadow_ = false;
};
}  // namespace ring

enum class WindowType { HANN, HAMMING, BLACKMAN, RECT, BLACKMAN_HARRIS };
enum class NormalizationType { NONE, SUM_TO_ONE, L2_NORM, OLA_UNITY_GAIN, OLA_SUM_WSQ };

// dsp::WindowLUT (WindowLUT.h:80-287): an instance owns one table
// (WindowLUT(nfft, type, periodic, norm).data()), and the process-wide cache
// hands out tables by (type, N, periodic, norm) -- GetWindowSafe as an aliasing
// shared_ptr that outlives clearCache(), the deprecated GetWindow as a raw
// pointer valid until clearCache().  Tables are the reference's, bit-exact
// (crlot_window_table, host code).
struct WindowData {
    std::vector<float, base::AlignedAllocator<float>> values;  // 64-byte aligned
    size_t size = 0;
    WindowType type = WindowType::HANN;
    bool periodic = false;
    NormalizationType norm = NormalizationType::NONE;
};

class WindowLUT {
   public:
    WindowLUT(size_t nfft, WindowType type, bool periodic = false,
              NormalizationType norm = NormalizationType::NONE) {
        if (nfft == 0) throw std::invalid_argument("Window size must be greater than 0");
        data_ = create(type, nfft, periodic, norm);
    }
    WindowLUT() = default;  // cache-only instance (getInstance)
    WindowLUT(const WindowLUT&) = delete;
    WindowLUT& operator=(const WindowLUT&) = delete;

    const float* data() const {
        if (!data_) throw std::runtime_error("Window data not initialized");
        return data_->values.data();
    }
    size_t size() const { return data_ ? data_->size : 0; }
    WindowType type() const { return data_ ? data_->type : WindowType::HANN; }
    bool periodic() const { return data_ ? data_->periodic : false; }
    NormalizationType normalization() const { return data_ ? data_->norm : NormalizationType::NONE; }

    // WindowLUT.cc:75-105: a hit must be of the current generation
    std::shared_ptr<const float> GetWindowSafe(WindowType type, size_t N, bool periodic = false,
                                               NormalizationType norm = NormalizationType::NONE) {
        if (N == 0) throw std::invalid_argument("Window size must be greater than 0");
        const uint64_t key = cache_key(type, N, periodic, norm);
        const uint64_t gen = generation().load();
        std::lock_guard<std::mutex> lock(mutex());
        auto it = safe_cache().find(key);
        if (it != safe_cache().end() && it->second.generation == gen)
            return std::shared_ptr<const float>(it->second.data, it->second.data->values.data());
        std::shared_ptr<WindowData> d(create(type, N, periodic, norm).release());
        safe_cache()[key] = Entry{d, gen};
        return std::shared_ptr<const float>(d, d->values.data());
    }

    // WindowLUT.cc:107-131 (deprecated in the reference: valid until clearCache)
    [[deprecated("Use GetWindowSafe() for thread safety")]]
    const float* GetWindow(WindowType type, size_t N, bool periodic = false,
                           NormalizationType norm = NormalizationType::NONE) {
        if (N == 0) throw std::invalid_argument("Window size must be greater than 0");
        const uint64_t key = cache_key(type, N, periodic, norm);
        std::lock_guard<std::mutex> lock(mutex());
        auto it = legacy_cache().find(key);
        if (it != legacy_cache().end()) return it->second->values.data();
        auto d = create(type, N, periodic, norm);
        const float* p = d->values.data();
        legacy_cache()[key] = std::move(d);
        return p;
    }

    static WindowLUT& getInstance() {
        static WindowLUT instance;
        return instance;
    }
    size_t getCacheSize() const {
        std::lock_guard<std::mutex> lock(mutex());
        return safe_cache().size() + legacy_cache().size();
    }
    // WindowLUT.cc:138-162: bump the generation (older handles stay valid),
    // drop entries two generations old; force_immediate empties both caches
    void clearCache(bool force_immediate = false) {
        std::lock_guard<std::mutex> lock(mutex());
        if (force_immediate) {
            safe_cache().clear();
            legacy_cache().clear();
            return;
        }
        generation().fetch_add(1);
        const uint64_t cur = generation().load();
        for (auto it = safe_cache().begin(); it != safe_cache().end();)
            it = (it->second.generation < cur - 1) ? safe_cache().erase(it) : std::next(it);
        legacy_cache().clear();
    }
    uint64_t getCurrentGeneration() const { return generation().load(); }

    static double calculateSum(const float* w, size_t N) {
        double s = 0.0;
        for (size_t i = 0; w && i < N; ++i) s += double(w[i]);
        return s;
    }
    static double calculateSumOfSquares(const float* w, size_t N) {
        double s = 0.0;
        for (size_t i = 0; w && i < N; ++i) s += double(w[i]) * double(w[i]);
        return s;
    }
    static double calculateRMSError(const float* a, const float* b, size_t N) {
        if (!a || !b || N == 0) return 0.0;
        double s = 0.0;
        for (size_t i = 0; i < N; ++i) {
            const double d = double(a[i]) - double(b[i]);
            s += d * d;
        }
        return std::sqrt(s / double(N));
    }

   private:
    struct Entry {
        std::shared_ptr<WindowData> data;
        uint64_t generation = 0;
    };
    // [type:8][periodic:1][norm:3][size:52] (WindowLUT.cc:448-457)
    static uint64_t cache_key(WindowType t, size_t N, bool periodic, NormalizationType norm) {
        return (uint64_t(t) << 56) | (uint64_t(periodic ? 1 : 0) << 55) | (uint64_t(norm) << 52) |
               (uint64_t(N) & 0xFFFFFFFFFFFFFULL);
    }
    static std::unique_ptr<WindowData> create(WindowType type, size_t N, bool periodic,
                                              NormalizationType norm) {
        if (type == WindowType::BLACKMAN_HARRIS)
            throw std::invalid_argument("Blackman-Harris window not yet implemented");
        auto d = std::make_unique<WindowData>();
        d->values.resize(N);
        d->size = N;
        d->type = type;
        d->periodic = periodic;
        d->norm = norm;
        check(crlot_window_table(int32_t(type), int64_t(N), periodic, int32_t(norm), d->values.data()),
              "crlot_window_table");
        return d;
    }
    static std::mutex& mutex() {
        static std::mutex m;
        return m;
    }
    static std::unordered_map<uint64_t, Entry>& safe_cache() {
        static std::unordered_map<uint64_t, Entry> c;
        return c;
    }
    static std::unordered_map<uint64_t, std::unique_ptr<WindowData>>& legacy_cache() {
        static std::unordered_map<uint64_t, std::unique_ptr<WindowData>> c;
        return c;
    }
    static std::atomic<uint64_t>& generation() {
        static std::atomic<uint64_t> g{1};
        return g;
    }
    std::unique_ptr<WindowData> data_;
};

// dsp::BoundaryMode (framer.h:11-14)
enum class BoundaryMode { ZERO_PAD, DROP };

// dsp::Framer (framer.h:26-127), host object over crlot_framer_*.
class Framer {
   public:
    Framer() { check(crlot_framer_create(&f_), "crlot_framer_create"); }
    ~Framer() { crlot_framer_destroy(f_); }
    Framer(const Framer&) = delete;
    Framer& operator=(const Framer&) = delete;
    void set_params(size_t frame_size, size_t hop_size, size_t channels = 1,
                    BoundaryMode boundary_mode = BoundaryMode::ZERO_PAD) {
        check(crlot_framer_set_params(f_, int64_t(frame_size), int64_t(hop_size), int64_t(channels),
                                      boundary_mode == BoundaryMode::DROP ? CRLOT_DROP : CRLOT_ZERO_PAD),
              "Framer::set_params");
    }
    bool push(const float* interleaved, size_t frames) {
        return check_bool(crlot_framer_push(f_, interleaved, int64_t(frames)));
    }
    bool pop(float* out_frame) { return check_bool(crlot_framer_pop(f_, out_frame)); }
    size_t available_frames() const { return size_t(crlot_framer_available(f_)); }
    void reset() { check(crlot_framer_reset(f_), "Framer::reset"); }
    size_t frame_size() const { return size_t(info().n); }
    size_t hop_size() const { return size_t(info().h); }
    size_t channels() const { return size_t(info().c); }
    BoundaryMode boundary_mode() const {
        return info().mode == CRLOT_DROP ? BoundaryMode::DROP : BoundaryMode::ZERO_PAD;
    }
    size_t buffer_size() const { return size_t(info().buf); }

   private:
    struct Info {
        int64_t n = 0, h = 0, c = 0, buf = 0;
        int32_t mode = 0;
    };
    Info info() const {
        Info i;
        check(crlot_framer_info(f_, &i.n, &i.h, &i.c, &i.mode, &i.buf), "Framer");
        return i;
    }
    static bool check_bool(int rc) {
        check(rc, "Framer");
        return rc == 1;
    }
    crlot_framer* f_ = nullptr;
};

// dsp::OLAConfig (OLAAccumulator.h:15-29); `device` selects the HIP device (-1: current).
struct OLAConfig {
    int sample_rate = 0;
    size_t frame_size = 0;
    size_t hop_size = 0;
    size_t channels = 0;
    float eps = 1e-8f;
    bool apply_window_inside = false;
    bool shadow_ring = false;
    int device = -1;
    bool isValid() const {
        return sample_rate > 0 && frame_size > 0 && hop_size > 0 && channels > 0 && eps > 0.0f;
    }
};

// dsp::OLAAccumulator (OLAAccumulator.h:63-217): the rings live on the device
// (crlot_ola_*); the reference's signatures take host pointers, the *_device
// forms take HBM pointers and a stream.  Non-copyable, non-movable, like the
// reference.
class OLAAccumulator {
   public:
    explicit OLAAccumulator(const OLAConfig& cfg) : cfg_(cfg) {
        if (!cfg.isValid()) throw std::invalid_argument("Invalid OLA configuration");
        crlot_ola_config c{};
        c.sample_rate = cfg.sample_rate;
        c.frame_size = int64_t(cfg.frame_size);
        c.hop_size = int64_t(cfg.hop_size);
        c.channels = int64_t(cfg.channels);
        c.eps = cfg.eps;
        c.apply_window_inside = cfg.apply_window_inside;
        c.shadow_ring = cfg.shadow_ring;
        c.device = cfg.device;
        check(crlot_ola_create(&c, &o_), "OLAAccumulator");
    }
    ~OLAAccumulator() { crlot_ola_destroy(o_); }
    OLAAccumulator(const OLAAccumulator&) = delete;
    OLAAccumulator& operator=(const OLAAccumulator&) = delete;
    OLAAccumulator(OLAAccumulator&&) = delete;
    OLAAccumulator& operator=(OLAAccumulator&&) = delete;

    void set_window(const float* w, int wlen) { check(crlot_ola_set_window(o_, w, wlen), "set_window"); }
    void add_frame_SoA(const float* const* ch_frames, const float* window, size_t start_sample,
                       size_t start_off, size_t size, float gain) {
        check(crlot_ola_add_frame_soa(o_, ch_frames, window, int64_t(start_sample), int64_t(start_off),
                                      int64_t(size), gain),
              "add_frame_SoA");
    }
    void push_frame_AoS(const float* interleaved, const float* window, size_t start_sample,
                        size_t start_off, size_t size, float gain) {
        check(crlot_ola_push_frame_aos(o_, interleaved, window, int64_t(start_sample), int64_t(start_off),
                                       int64_t(size), gain),
              "push_frame_AoS");
    }
    size_t produce(float* const* ch_out, size_t n) {
        int64_t got = 0;
        check(crlot_ola_produce(o_, ch_out, int64_t(n), &got), "produce");
        return size_t(got);
    }
    // device forms: frames / outputs in HBM, channel c at +c*ld
    void add_frame_SoA_device(const float* d_frames, size_t ld_frames, const float* d_window,
                              size_t start_sample, size_t start_off, size_t size, float gain,
                              hipStream_t s = nullptr) {
        check(crlot_ola_add_frame_soa_device(o_, d_frames, int64_t(ld_frames), d_window, int64_t(start_sample),
                                             int64_t(start_off), int64_t(size), gain, s),
              "add_frame_SoA_device");
    }
    void push_frame_AoS_device(const float* d_interleaved, const float* d_window, size_t start_sample,
                               size_t start_off, size_t size, float gain, hipStream_t s = nullptr) {
        check(crlot_ola_push_frame_aos_device(o_, d_interleaved, d_window, int64_t(start_sample),
                                              int64_t(start_off), int64_t(size), gain, s),
              "push_frame_AoS_device");
    }
    size_t produce_device(float* d_out, size_t ld_out, size_t n, hipStream_t s = nullptr) {
        int64_t got = 0;
        check(crlot_ola_produce_device(o_, d_out, int64_t(ld_out), int64_t(n), &got, s), "produce_device");
        return size_t(got);
    }
    void flush() { check(crlot_ola_flush(o_), "flush"); }
    void reset() { check(crlot_ola_reset(o_), "reset"); }
    void synchronize() { check(crlot_ola_synchronize(o_), "synchronize"); }
    size_t produced_samples() const { return size_t(state().produced); }
    size_t read_pos() const { return size_t(state().read_pos); }
    float meter_peak() const {
        float p = 0.0f;
        check(crlot_ola_meter_peak(o_, &p), "meter_peak");
        return p;
    }
    const OLAConfig& config() const { return cfg_; }
    bool has_window() const { return state().has_window != 0; }
    size_t ring_size() const { return size_t(state().ring); }

   private:
    struct State {
        int64_t produced = 0, read_pos = 0, ring = 0;
        int32_t has_window = 0;
    };
    State state() const {
        State s;
        check(crlot_ola_info(o_, &s.produced, &s.read_pos, &s.ring, &s.has_window), "OLAAccumulator");
        return s;
    }
    OLAConfig cfg_;
    crlot_ola* o_ = nullptr;
};

// dsp::PadMode (FrameQueue.h:8-12)
enum class PadMode { CONSTANT, REFLECT, EDGE };

// dsp::FrameQueue (FrameQueue.h:35-59): every frame of a whole signal, built on
// the device at construction (crlot_framequeue_*).  getFrame / copyFrame /
// getAllFrames read the reference's AoS host copy; device_frames() is the same
// [num_frames][frame_size] block in HBM.  Throws as the reference:
// std::invalid_argument on zero sizes or a null input with len > 0,
// std::out_of_range on a frame index past the end.
class FrameQueue {
   public:
    FrameQueue(const float* in, size_t len, size_t frame_size, size_t hop_size, bool center = true,
               PadMode pad_mode = PadMode::CONSTANT, int device = -1) {
        const int rc = crlot_framequeue_create(in, int64_t(len), int64_t(frame_size), int64_t(hop_size),
                                               center ? 1 : 0, int32_t(pad_mode), device, &q_);
        if (rc != CRLOT_OK) check(rc, "FrameQueue");
        check(crlot_framequeue_info(q_, &f_, &n_, &h_), "FrameQueue");
    }
    ~FrameQueue() { crlot_framequeue_destroy(q_); }
    FrameQueue(const FrameQueue&) = delete;
    FrameQueue& operator=(const FrameQueue&) = delete;
    size_t getNumFrames() const { return size_t(f_); }
    size_t getFrameSize() const { return size_t(n_); }
    size_t getHopSize() const { return size_t(h_); }
    // (through the library, which notes the frame read last: the batched
    // speculation of a per-frame loop over the queue starts from it)
    const float* getFrame(size_t frame_idx) const {
        if (frame_idx >= size_t(f_)) throw std::out_of_range("Frame index out of range");
        return crlot_framequeue_frame(q_, int64_t(frame_idx));
    }
    void copyFrame(size_t frame_idx, float* output) const {
        if (frame_idx >= size_t(f_)) throw std::out_of_range("Frame index out of range");
        if (output == nullptr) throw std::invalid_argument("Output buffer cannot be null");
        check(crlot_framequeue_copy_frame(q_, int64_t(frame_idx), output), "FrameQueue::copyFrame");
    }
    // (a copy made at the first call: most callers read frames one at a time)
    const std::vector<float>& getAllFrames() const {
        std::call_once(all_once_, [this] {
            const float* a = crlot_framequeue_all_frames(q_);
            if (a) frames_.assign(a, a + size_t(f_ * n_));
        });
        return frames_;
    }
    const float* device_frames() const { return crlot_framequeue_device_frames(q_); }

   private:
    crlot_framequeue* q_ = nullptr;
    int64_t f_ = 0, n_ = 0, h_ = 0;
    mutable std::once_flag all_once_;
    mutable std::vector<float> frames_;
};

// dsp::axpy / axpy_windowed / normalize_and_clear (kernels.h:28-53): the
// reference's noexcept host-pointer signatures, run on the device (a resident
// call kernel, crlot_call_*).  A device failure cannot be reported through a
// noexcept signature: it terminates, as an exception escaping one would.
namespace detail {
[[noreturn]] inline void kernel_failed(const char* what) noexcept {
    std::fprintf(stderr, "crlot::dsp::%s failed: %s\n", what, crlot_last_error());
    std::terminate();
}
}  // namespace detail
inline void axpy(float* dst, const float* src, float g, size_t n) noexcept {
    if (crlot_call_axpy(dst, src, g, int64_t(n)) != CRLOT_OK) detail::kernel_failed("axpy");
}
inline void axpy_windowed(float* dst, const float* src, const float* win, float g, size_t n) noexcept {
    if (crlot_call_axpy_windowed(dst, src, win, g, int64_t(n)) != CRLOT_OK) detail::kernel_failed("axpy_windowed");
}
inline void normalize_and_clear(float* out, float* acc, const float* norm, float eps, size_t n) noexcept {
    if (crlot_call_normalize_and_clear(out, acc, norm, eps, int64_t(n)) != CRLOT_OK)
        detail::kernel_failed("normalize_and_clear");
}
// batched device forms: `batch` rows of n at + b*ld, the window / norm row shared
inline void axpy_device(float* d_dst, const float* d_src, float g, size_t n, size_t batch = 1, size_t ld_dst = 0,
                        size_t ld_src = 0, hipStream_t s = nullptr) {
    check(crlot_axpy(d_dst, d_src, g, int64_t(n), int64_t(batch), int64_t(ld_dst ? ld_dst : n),
                     int64_t(ld_src ? ld_src : n), s),
          "axpy_device");
}
inline void axpy_windowed_device(float* d_dst, const float* d_src, const float* d_win, float g, size_t n,
                                 size_t batch = 1, size_t ld_dst = 0, size_t ld_src = 0, hipStream_t s = nullptr) {
    check(crlot_axpy_windowed(d_dst, d_src, d_win, g, int64_t(n), int64_t(batch), int64_t(ld_dst ? ld_dst : n),
                              int64_t(ld_src ? ld_src : n), s),
          "axpy_windowed_device");
}
inline void normalize_and_clear_device(float* d_out, float* d_acc, const float* d_norm, float eps, size_t n,
                                       size_t batch = 1, size_t ld_out = 0, size_t ld_acc = 0,
                                       hipStream_t s = nullptr) {
    check(crlot_normalize_and_clear(d_out, d_acc, d_norm, eps, int64_t(n), int64_t(batch),
                                    int64_t(ld_out ? ld_out : n), int64_t(ld_acc ? ld_acc : n), s),
          "normalize_and_clear_device");
}

namespace fft {

enum class FftDomain { Real, Complex };

struct FftPlanDesc {
    FftDomain domain;
    int nfft;
    bool in_place;
    int batch;
    int stride_in;
    int stride_out;
};

// dsp::fft::IFftPlan (fft_api.h:26-48), same virtuals and defaults.
class IFftPlan {
   public:
    virtual ~IFftPlan() = default;
    virtual void forward(const float* in, std::complex<float>* out, int batch = 1) = 0;
    virtual void inverse(const std::complex<float>* in, float* out, int batch = 1) = 0;
    virtual void forward_complex(const std::complex<float>* in, std::complex<float>* out,
                                 int batch = 1) = 0;
    virtual void inverse_complex(const std::complex<float>* in, std::complex<float>* out,
                                 int batch = 1) = 0;
    virtual FftDomain domain() const = 0;
    virtual int size() const = 0;
    virtual bool supports_batch() const { return true; }
    virtual int max_batch_size() const { return 16; }
};

// HIP-backed plan with KissFftPlan's semantics in both domains
// (kissfft_adapter.cc:83-246): real forward sanitizes its input; real and
// complex inverse scale by 1/nfft and sanitize; complex forward is the raw DFT.
// Batch b starts at b*stride*len, element i sits at i*stride (len = nfft, or
// nfft/2+1 for the real spectrum).  Validation mirrors KissFftPlan
// (kissfft_adapter.cc:13-63) except the batch ceiling, which the device path
// does not need (MakeFftPlan below applies it).  Host pointers go to the plan's
// resident call kernel (crlot_fft_*_host: no launch or copy-engine transfer per
// call); calls on one plan are serialised, as the reference's plan owns scratch.
// forward_device / inverse_device take HBM pointers and a stream.
class HipFftPlan final : public IFftPlan {
   public:
    explicit HipFftPlan(const FftPlanDesc& d) : d_(validate(d)) {
        crlot_fft_desc fd{d.domain == FftDomain::Real ? CRLOT_FFT_REAL : CRLOT_FFT_COMPLEX, d.nfft, -1};
        check(crlot_fft_plan_create(&fd, &p_), "crlot_fft_plan_create");
    }
    ~HipFftPlan() override { crlot_fft_plan_destroy(p_); }
    HipFftPlan(const HipFftPlan&) = delete;
    HipFftPlan& operator=(const HipFftPlan&) = delete;

    void forward(const float* in, std::complex<float>* out, int batch = 1) override {
        if (d_.domain != FftDomain::Real)
            throw std::runtime_error("Real FFT not supported for Complex domain plan");
        check_batch(batch);
        const int64_t n = d_.nfft, bins = n / 2 + 1;
        run(in, 1, span(batch, d_.stride_in, n), reinterpret_cast<float*>(out), 2, span(batch, d_.stride_out, bins),
            [&](const float* i, float* o) {
                return crlot_fft_forward_host(p_, i, o, batch, d_.stride_in * n, d_.stride_in,
                                              2 * d_.stride_out * bins, d_.stride_out);
            });
    }
    void inverse(const std::complex<float>* in, float* out, int batch = 1) override {
        if (d_.domain != FftDomain::Real)
            throw std::runtime_error("Real FFT not supported for Complex domain plan");
        check_batch(batch);
        const int64_t n = d_.nfft, bins = n / 2 + 1;
        run(reinterpret_cast<const float*>(in), 2, span(batch, d_.stride_in, bins), out, 1,
            span(batch, d_.stride_out, n), [&](const float* i, float* o) {
                return crlot_fft_inverse_host(p_, i, o, batch, 2 * d_.stride_in * bins, d_.stride_in,
                                              d_.stride_out * n, d_.stride_out);
            });
    }
    void forward_complex(const std::complex<float>* in, std::complex<float>* out, int batch = 1) override {
        complex_call(in, out, batch, false);
    }
    void inverse_complex(const std::complex<float>* in, std::complex<float>* out, int batch = 1) override {
        complex_call(in, out, batch, true);
    }
    FftDomain domain() const override { return d_.domain; }
    int size() const override { return d_.nfft; }
    crlot_fft_plan* handle() const { return p_; }
    // device forms: any batch, dense rows (ld = nfft floats in, nfft/2+1 pairs out)
    void forward_device(const float* d_in, std::complex<float>* d_out, int batch, hipStream_t s = nullptr) {
        const int64_t n = d_.nfft, bins = n / 2 + 1;
        check(crlot_fft_forward(p_, d_in, reinterpret_cast<float*>(d_out), batch, n, 1, 2 * bins, 1, s),
              "forward_device");
    }
    void inverse_device(const std::complex<float>* d_in, float* d_out, int batch, hipStream_t s = nullptr) {
        const int64_t n = d_.nfft, bins = n / 2 + 1;
        check(crlot_fft_inverse(p_, reinterpret_cast<const float*>(d_in), d_out, batch, 2 * bins, 1, n, 1, s),
              "inverse_device");
    }

   private:
    static FftPlanDesc validate(const FftPlanDesc& d) {
        if (d.domain != FftDomain::Real && d.domain != FftDomain::Complex)
            throw std::runtime_error("Unsupported FFT domain");
        if (d.batch < 1) throw std::runtime_error("Batch size must be at least 1");
        if (d.stride_in < 1 || d.stride_out < 1) throw std::runtime_error("Stride must be at least 1");
        if (d.in_place) throw std::runtime_error("In-place FFT is not yet supported");
        if (d.domain == FftDomain::Real && d.nfft % 2 != 0)
            throw std::runtime_error("FFT size must be even for real FFT");
        return d;
    }
    // elements a strided batch addresses: the last batch's last element + 1
    // (the reference touches only i*stride, i < len: kissfft_adapter.cc:97-98, 139-140)
    static int64_t span(int batch, int stride, int64_t len) {
        return (int64_t(batch) - 1) * stride * len + (len - 1) * stride + 1;
    }
    void check_batch(int batch) const {
        if (batch < 1 || batch > d_.batch) throw std::runtime_error("Invalid batch size");
    }
    void complex_call(const std::complex<float>* in, std::complex<float>* out, int batch, bool inv) {
        if (d_.domain != FftDomain::Complex)
            throw std::runtime_error("Complex FFT not supported for Real domain plan");
        check_batch(batch);
        const int64_t n = d_.nfft;
        run(reinterpret_cast<const float*>(in), 2, span(batch, d_.stride_in, n),
            reinterpret_cast<float*>(out), 2, span(batch, d_.stride_out, n), [&](const float* i, float* o) {
                return (inv ? crlot_fft_inverse_complex_host : crlot_fft_forward_complex_host)(
                    p_, i, o, batch, 2 * d_.stride_in * n, d_.stride_in, 2 * d_.stride_out * n,
                    d_.stride_out);
            });
    }
    // host pointers straight to the plan's host-call path (crlot_fft_*_host:
    // the resident call kernel; the reference writes only the strided output
    // elements, and so do these)
    template <typename F>
    void run(const float* in, int, int64_t, float* out, int, int64_t, F launch) {
        check(launch(in, out), "fft");
    }
    FftPlanDesc d_;
    crlot_fft_plan* p_ = nullptr;
};
using HipRealFftPlan = HipFftPlan;  // earlier name

// dsp::fft::MakeFftPlan (fft_api.h:51) with KissFftPlan's checks, including its
// batch ceiling of 16 (kissfft_adapter.cc:21-23).
inline std::unique_ptr<IFftPlan> MakeFftPlan(const FftPlanDesc& d) {
    if (d.domain != FftDomain::Real && d.domain != FftDomain::Complex)
        throw std::runtime_error("Unsupported FFT domain");
    if (d.batch < 1 || d.batch > 16) throw std::runtime_error("Batch size must be between 1 and 16");
    return std::make_unique<HipFftPlan>(d);
}

}  // namespace fft
}  // namespace dsp
}  // namespace crlot
