// Drop-in for the reference's dsp/frame/framer.h (framer.h:6-127): the same
// include path and names, served by the MI355X library (include/crlot_dsp.hpp).
// Build a reference harness against it with -I<repo>/include/ref ahead of the
// reference's own include path; link -lcrlot_dsp.
#pragma once

#include "../../../crlot_dsp.hpp"

namespace dsp {
using crlot::dsp::BoundaryMode;  // framer.h:11-14
using crlot::dsp::Framer;        // framer.h:26-127
}  // namespace dsp
