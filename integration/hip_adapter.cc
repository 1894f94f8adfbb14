// integration/hip_adapter.cc -- the IFftPlan backend a maintainer adds to the
// reference tree.  Kept here so tests can compile it
// against the reference's own dsp/fft/api/fft_api.h (tests/test_integration.py).
// dsp/fft/backends/hip_adapter.cc  (reference tree; selected by --define FFT_BACKEND=hip)
#include "dsp/fft/api/fft_api.h"
#include <stdexcept>
#include <crlot_dsp.hpp>           // crlot::dsp::fft::HipFftPlan does the work

namespace dsp::fft {
namespace {
crlot::dsp::fft::FftPlanDesc to_crlot(const FftPlanDesc& d) {
  return {d.domain == FftDomain::Real ? crlot::dsp::fft::FftDomain::Real
                                      : crlot::dsp::fft::FftDomain::Complex,
          d.nfft, d.in_place, d.batch, d.stride_in, d.stride_out};
}
}  // namespace

class HipFftPlan : public IFftPlan {
 public:
  explicit HipFftPlan(const FftPlanDesc& d) : impl_(to_crlot(d)), domain_(d.domain) {}
  void forward(const float* in, std::complex<float>* out, int batch) override { impl_.forward(in, out, batch); }
  void inverse(const std::complex<float>* in, float* out, int batch) override { impl_.inverse(in, out, batch); }
  void forward_complex(const std::complex<float>* in, std::complex<float>* out, int batch) override {
    impl_.forward_complex(in, out, batch);
  }
  void inverse_complex(const std::complex<float>* in, std::complex<float>* out, int batch) override {
    impl_.inverse_complex(in, out, batch);
  }
  FftDomain domain() const override { return domain_; }
  int size() const override { return impl_.size(); }
 private:
  crlot::dsp::fft::HipFftPlan impl_;
  FftDomain domain_;
};

// KissFftPlan's checks (kissfft_adapter.cc:13-63), batch ceiling included.
std::unique_ptr<IFftPlan> MakeFftPlan(const FftPlanDesc& d) {
  if (d.domain != FftDomain::Real && d.domain != FftDomain::Complex)
    throw std::runtime_error("Unsupported FFT domain");
  if (d.batch < 1 || d.batch > 16) throw std::runtime_error("Batch size must be between 1 and 16");
  return std::make_unique<HipFftPlan>(d);
}
}  // namespace dsp::fft
