// crlot_dsp.hpp -- C++ host surface over the C ABI (header-only).
//
// Mirrors the reference's C++ API for the hot path so C++ callers drop in:
//   crlot::dsp::WindowLUT          <- dsp::WindowLUT        (WindowLUT.h:80-199)
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

#include <complex>
#include <cstdint>
#include <memory>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "crlot_dsp.h"

namespace crlot {

inline void check(int rc, const char* what) {
    if (rc >= 0) return;
    std::string msg = std::string(what) + ": " + crlot_last_error();
    if (rc == CRLOT_EINVAL) throw std::invalid_argument(msg);
    if (rc == CRLOT_ENOMEM) throw std::bad_alloc();
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
    explicit StftEngine(const Config& c) : plan_(desc(c)) {}
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
    void set_spectral_gain(const float* gain_or_null) {
        check(crlot_plan_set_spectral_gain(plan_.get(), gain_or_null), "set_spectral_gain");
    }
    // crlot_plan_set_frame_pairing: two frames per complex transform (default) or per frame
    void set_frame_pairing(bool enable) {
        check(crlot_plan_set_frame_pairing(plan_.get(), enable ? 1 : 0), "set_frame_pairing");
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
    DeviceBuffer<float> dx_, dy_;
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

enum class WindowType { HANN, HAMMING, BLACKMAN, RECT, BLACKMAN_HARRIS };
enum class NormalizationType { NONE, SUM_TO_ONE, L2_NORM, OLA_UNITY_GAIN, OLA_SUM_WSQ };

// WindowLUT(nfft, type, periodic, norm).data(): the reference's tables, bit-exact.
class WindowLUT {
   public:
    WindowLUT(size_t nfft, WindowType type, bool periodic = false,
              NormalizationType norm = NormalizationType::NONE)
        : data_(nfft) {
        if (nfft == 0) throw std::invalid_argument("Window size must be greater than 0");
        if (type == WindowType::BLACKMAN_HARRIS)
            throw std::invalid_argument("Blackman-Harris window not yet implemented");
        check(crlot_window_table(int32_t(type), int64_t(nfft), periodic, int32_t(norm), data_.data()),
              "crlot_window_table");
    }
    const float* data() const { return data_.data(); }
    size_t size() const { return data_.size(); }

   private:
    std::vector<float> data_;
};

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
// does not need (MakeFftPlan below applies it).  Host pointers are staged
// through device buffers owned by the plan, so calls are not reentrant (as in
// the reference, whose plan owns scratch).
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
        run(in, 1, batch * d_.stride_in * n, reinterpret_cast<float*>(out), 2, batch * d_.stride_out * bins,
            [&](const float* i, float* o) {
                return crlot_fft_forward(p_, i, o, batch, d_.stride_in * n, d_.stride_in,
                                         2 * d_.stride_out * bins, d_.stride_out, nullptr);
            });
    }
    void inverse(const std::complex<float>* in, float* out, int batch = 1) override {
        if (d_.domain != FftDomain::Real)
            throw std::runtime_error("Real FFT not supported for Complex domain plan");
        check_batch(batch);
        const int64_t n = d_.nfft, bins = n / 2 + 1;
        run(reinterpret_cast<const float*>(in), 2, batch * d_.stride_in * bins, out, 1,
            batch * d_.stride_out * n, [&](const float* i, float* o) {
                return crlot_fft_inverse(p_, i, o, batch, 2 * d_.stride_in * bins, d_.stride_in,
                                         d_.stride_out * n, d_.stride_out, nullptr);
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
    void check_batch(int batch) const {
        if (batch < 1 || batch > d_.batch) throw std::runtime_error("Invalid batch size");
    }
    void complex_call(const std::complex<float>* in, std::complex<float>* out, int batch, bool inv) {
        if (d_.domain != FftDomain::Complex)
            throw std::runtime_error("Complex FFT not supported for Real domain plan");
        check_batch(batch);
        const int64_t n = d_.nfft;
        run(reinterpret_cast<const float*>(in), 2, batch * d_.stride_in * n,
            reinterpret_cast<float*>(out), 2, batch * d_.stride_out * n, [&](const float* i, float* o) {
                return (inv ? crlot_fft_inverse_complex : crlot_fft_forward_complex)(
                    p_, i, o, batch, 2 * d_.stride_in * n, d_.stride_in, 2 * d_.stride_out * n,
                    d_.stride_out, nullptr);
            });
    }
    // stage host -> device, launch, device -> host.  The reference writes only
    // the strided output elements, so the device output starts as a copy of the
    // caller's buffer.
    template <typename F>
    void run(const float* in, int in_w, int64_t in_elems, float* out, int out_w, int64_t out_elems, F launch) {
        const size_t in_f = size_t(in_w) * in_elems, out_f = size_t(out_w) * out_elems;
        din_.resize(in_f);
        dout_.resize(out_f);
        hip_check(hipMemcpy(din_.get(), in, sizeof(float) * in_f, hipMemcpyHostToDevice), "hipMemcpy");
        hip_check(hipMemcpy(dout_.get(), out, sizeof(float) * out_f, hipMemcpyHostToDevice), "hipMemcpy");
        check(launch(din_.get(), dout_.get()), "fft");
        hip_check(hipMemcpy(out, dout_.get(), sizeof(float) * out_f, hipMemcpyDeviceToHost), "hipMemcpy");
    }
    FftPlanDesc d_;
    crlot_fft_plan* p_ = nullptr;
    DeviceBuffer<float> din_, dout_;
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
