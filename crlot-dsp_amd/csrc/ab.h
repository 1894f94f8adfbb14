// ab.h -- A/B switches (internal).  Environment variables that pick between
// bit-identical launch shapes for measurements are read only in builds with
// -DCRLOT_AB_SWITCHES (`make variant`); the release library reads no
// environment and always takes the defaults.
#pragma once

#include <cstdlib>

namespace crlot {
inline const char* ab_env(const char* name) {
#ifdef CRLOT_AB_SWITCHES
    return std::getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}
}  // namespace crlot
