// build_info.cpp -- what this library was built from (crlot_build_info).
// CRLOT_SRC_HASH is tools/src_hash.py's lib_hash() of the sources at build time,
// passed in by the Makefile; bench.py and smoke() compare it with the tree's.
#include "crlot_dsp.h"

#ifndef CRLOT_SRC_HASH
#define CRLOT_SRC_HASH "unknown"
#endif

extern "C" const char* crlot_build_info(void) { return "src:" CRLOT_SRC_HASH " arch:gfx950"; }
