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
std::map<int, std::vector<hipEvent_t>> g_events;           // free events per device
std::map<size_t, std::vector<void*>> g_pinned;              // free pinned blocks per size class
bool g_pool_set[64] = {};
hipMemPool_t g_pool[64] = {};

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

hipError_t pool_event(int device, hipEvent_t* out) {
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto& v = g_events[device];
        if (!v.empty()) {
            *out = v.back();
            v.pop_back();
            return hipSuccess;
        }
    }
    return hipEventCreateWithFlags(out, hipEventDisableTiming);
}

void pool_event_put(int device, hipEvent_t ev) {
    if (!ev) return;
    std::lock_guard<std::mutex> lk(g_mu);
    auto& v = g_events[device];
    if (v.size() < 4 * kMaxFree)
        v.push_back(ev);
    else
        (void)hipEventDestroy(ev);
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

// Stream-ordered device memory from a pool private to this library (one per
// device), so frees stay cached for the next object's allocation without
// changing the process-wide default pool's release policy.  The pool keeps up
// to kKeepBytes of freed memory; beyond that it returns memory to the device at
// the next synchronisation.  Devices where the pool cannot be created fall back
// to the default pool, untouched.
constexpr uint64_t kKeepBytes = uint64_t(256) << 20;

hipError_t pool_malloc(int device, void** out, size_t bytes, hipStream_t s) {
    if (no_pool()) return hipMalloc(out, bytes);
    hipMemPool_t mp = nullptr;
    if (device >= 0 && device < 64) {
        std::lock_guard<std::mutex> lk(g_mu);
        if (!g_pool_set[device]) {
            hipMemPoolProps props{};
            props.allocType = hipMemAllocationTypePinned;
            props.handleTypes = hipMemHandleTypeNone;
            props.location.type = hipMemLocationTypeDevice;
            props.location.id = device;
            if (hipMemPoolCreate(&g_pool[device], &props) == hipSuccess && g_pool[device]) {
                uint64_t keep = kKeepBytes;
                (void)hipMemPoolSetAttribute(g_pool[device], hipMemPoolAttrReleaseThreshold, &keep);
            } else {
                g_pool[device] = nullptr;
            }
            g_pool_set[device] = true;
        }
        mp = g_pool[device];
    }
    return mp ? hipMallocFromPoolAsync(out, bytes, mp, s) : hipMallocAsync(out, bytes, s);
}

void pool_free(void* p, hipStream_t s) {
    if (!p) return;
    if (no_pool())
        (void)hipFree(p);
    else
        (void)hipFreeAsync(p, s);
}

}  // namespace crlot
