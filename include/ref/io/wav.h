// Drop-in for the reference's io/wav.h (wav.h:11-72; global namespace there):
// RIFF PCM / float WAV reader and writer (include/crlot_dsp.hpp crlot::io).
#pragma once

#include "../../crlot_dsp.hpp"

using crlot::io::WavReader;  // wav.h:11-40
using crlot::io::WavWriter;  // wav.h:42-72
