// respool.cpp -- see respool.h.
#include "respool.h"
#include "ab.h"

#include <cstdint>
#include <cstdlib>
#include <map>
#include <mutex>
#include <vector>

namespace crlot {
namespace {

std::mutex g_mu;
std::map<int, std::vector<hipStream_t>> g_streams;          // free streams per device
std::map<size_t, std::vector<void*>> g_pinned;              // free pinned blocks per size class
bool g_pool_set[64] = {};

size_t size_class(size_t bytes) {
    size_t c = 256;
    while (c < bytes) c <<= 1;
    return c;
}

constexpr size_t kMaxFree = 64;  // per stream list / size class

}  // namespace

hipError_t pool_stream(int device, hipStream_t* out) {
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto& v = g_streams[device];
        if (!v.empty()) {
            *out = v.back();
            v.pop_back();
            return hipSuccess;
        }
    }
    return hipStreamCreateWithFlags(out, hipStreamNonBlocking);
}

void pool_stream_put(int device, hipStream_t s) {
    if (!s) return;
    std::lock_guard<std::mutex> lk(g_mu);
    auto& v = g_streams[device];
    if (v.size() < kMaxFree)
        v.push_back(s);
    else
        (void)hipStreamDestroy(s);
}

hipError_t pool_pinned(size_t bytes, void** out, size_t* cap) {
    const size_t c = size_class(bytes);
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto& v = g_pinned[c];
        if (!v.empty()) {
            *out = v.back();
            v.pop_back();
            *cap = c;
            return hipSuccess;
        }
    }
    *cap = c;
    return hipHostMalloc(out, c);
}

void pool_pinned_put(void* p, size_t cap) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(g_mu);
    auto& v = g_pinned[cap];
    if (v.size() < kMaxFree)
        v.push_back(p);
    else
        (void)hipHostFree(p);
}

bool no_pool() {
    static const bool v = [] {
        const char* e = crlot::ab_env("CRLOT_NO_POOL");  // diagnostic: plain hipMalloc / hipFree
        return e && e[0] == '1';
    }();
    return v;
}

hipError_t pool_malloc(int device, void** out, size_t bytes, hipStream_t s) {
    if (no_pool()) return hipMalloc(out, bytes);
    if (device >= 0 && device < 64) {
        std::lock_guard<std::mutex> lk(g_mu);
        if (!g_pool_set[device]) {
            hipMemPool_t mp = nullptr;
            if (hipDeviceGetDefaultMemPool(&mp, device) == hipSuccess && mp) {
                uint64_t keep = UINT64_MAX;
                (void)hipMemPoolSetAttribute(mp, hipMemPoolAttrReleaseThreshold, &keep);
            }
            g_pool_set[device] = true;
        }
    }
    return hipMallocAsync(out, bytes, s);
}

void pool_free(void* p, hipStream_t s) {
    if (!p) return;
    if (no_pool())
        (void)hipFree(p);
    else
        (void)hipFreeAsync(p, s);
}

}  // namespace crlot
