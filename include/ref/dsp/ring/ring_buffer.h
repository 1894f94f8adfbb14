// Drop-in for the reference's dsp/ring/ring_buffer.h (ring_buffer.h:8-117): the
// host ring the reference's OLA object is built on (include/crlot_dsp.hpp,
// crlot::dsp::ring; the drop-in OLAAccumulator's own rings live in HBM).
#pragma once

#include "../base/span.h"

namespace dsp {
namespace ring {
using crlot::dsp::ring::RingBuffer;
}  // namespace ring
}  // namespace dsp
