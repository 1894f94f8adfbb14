// Drop-in for the reference's dsp/ola/OLAAccumulator.h (OLAAccumulator.h:10-217):
// the rings live in HBM, every add / produce runs on the device
// (include/crlot_dsp.hpp).
#pragma once

#include "../../../crlot_dsp.hpp"
#include "../ring/ring_buffer.h"  // (the reference header includes it: OLAAccumulator.h:7)

namespace dsp {
using crlot::dsp::OLAAccumulator;  // OLAAccumulator.h:55-217
using crlot::dsp::OLAConfig;       // OLAAccumulator.h:15-29
}  // namespace dsp
