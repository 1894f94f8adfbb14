// Drop-in for the reference's dsp/fft/api/fft_api.h (fft_api.h:7-51):
// MakeFftPlan returns the HIP-backed plan (include/crlot_dsp.hpp HipFftPlan),
// with kissfft_adapter.cc's semantics (sanitize, 1/N, stride).
#pragma once

#include "../../../../crlot_dsp.hpp"

namespace dsp {
namespace fft {
using crlot::dsp::fft::FftDomain;    // fft_api.h:10-13
using crlot::dsp::fft::FftPlanDesc;  // fft_api.h:16-23
using crlot::dsp::fft::IFftPlan;     // fft_api.h:26-48
using crlot::dsp::fft::MakeFftPlan;  // fft_api.h:51
}  // namespace fft
}  // namespace dsp
