// integration/hip_adapter.cc -- the IFftPlan backend a maintainer adds to the
// reference tree.  Kept here so tests can compile it
// against the reference's own dsp/fft/api/fft_api.h (tests/test_integration.py).
// dsp/fft/backends/hip_adapter.cc  (reference tree; selected by --define FFT_BACKEND=hip)
#include "dsp/fft/api/fft_api.h"
#include <stdexcept>
#include <crlot_dsp.hpp>           // crlot::dsp::fft::HipRealFftPlan does the work

namespace dsp::fft {
class HipFftPlan : public IFftPlan {
 public:
  explicit HipFftPlan(const FftPlanDesc& d)
      : impl_({crlot::dsp::fft::FftDomain::Real, d.nfft, d.in_place, d.batch,
               d.stride_in, d.stride_out}), nfft_(d.nfft) {
    if (d.domain != FftDomain::Real) throw std::runtime_error("Unsupported FFT domain");
    if (d.batch < 1 || d.batch > 16) throw std::runtime_error("Batch size must be between 1 and 16");
  }
  void forward(const float* in, std::complex<float>* out, int batch) override { impl_.forward(in, out, batch); }
  void inverse(const std::complex<float>* in, float* out, int batch) override { impl_.inverse(in, out, batch); }
  void forward_complex(const std::complex<float>*, std::complex<float>*, int) override {
    throw std::runtime_error("complex domain: use the kissfft backend");
  }
  void inverse_complex(const std::complex<float>*, std::complex<float>*, int) override {
    throw std::runtime_error("complex domain: use the kissfft backend");
  }
  FftDomain domain() const override { return FftDomain::Real; }
  int size() const override { return nfft_; }
 private:
  crlot::dsp::fft::HipRealFftPlan impl_;
  int nfft_;
};
std::unique_ptr<IFftPlan> MakeFftPlan(const FftPlanDesc& d) { return std::make_unique<HipFftPlan>(d); }
}  // namespace dsp::fft
