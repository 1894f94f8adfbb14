// Drop-in for the reference's dsp/base/span.h (span.h:8-33): the same include
// path and name (include/crlot_dsp.hpp, crlot::dsp::base).
#pragma once

#include "../../../crlot_dsp.hpp"

namespace dsp {
namespace base {
using crlot::dsp::base::Span;
}  // namespace base
}  // namespace dsp
