// Drop-in for the reference's dsp/window/WindowLUT.h (WindowLUT.h:9-287): the
// same tables bit for bit and the GetWindowSafe / GetWindow / getInstance cache
// (include/crlot_dsp.hpp).
#pragma once

#include "../../../crlot_dsp.hpp"

namespace dsp {
using crlot::dsp::NormalizationType;  // WindowLUT.h:25-31
using crlot::dsp::WindowData;         // WindowLUT.h:37-76
using crlot::dsp::WindowLUT;          // WindowLUT.h:80-287
using crlot::dsp::WindowType;         // WindowLUT.h:14-20
}  // namespace dsp
