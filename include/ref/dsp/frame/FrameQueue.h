// Drop-in for the reference's dsp/frame/FrameQueue.h (FrameQueue.h:6-59):
// frames built on the device, bit-exact with FrameQueue.cc (include/crlot_dsp.hpp).
#pragma once

#include "../../../crlot_dsp.hpp"

namespace dsp {
using crlot::dsp::FrameQueue;  // FrameQueue.h:23-59
using crlot::dsp::PadMode;     // FrameQueue.h:8-12
}  // namespace dsp
