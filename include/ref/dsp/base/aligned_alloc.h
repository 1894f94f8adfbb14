// Drop-in for the reference's dsp/base/aligned_alloc.h (aligned_alloc.h:13-47):
// 64-byte aligned host storage (include/crlot_dsp.hpp, crlot::dsp::base).
#pragma once

#include "../../../crlot_dsp.hpp"

namespace dsp {
namespace base {
using crlot::dsp::base::AllocateAligned;
using crlot::dsp::base::DeallocateAligned;
}  // namespace base
}  // namespace dsp
