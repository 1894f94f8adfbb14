// call.h -- host side of the resident call server (call.cpp, call_rt.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>
#include <vector>

#include "crlot_dsp.h"
#include "kernels.h"

namespace crlot {

// The arena slots of one request: host views (in: write-combined device
// memory or pinned host memory; out / spec: pinned host memory) and offsets.
struct CallSlot {
    uint64_t index = 0;  // 1-based request number: done >= index once it completed
    uint64_t gen = 0;    // arena generation the views point into (CallServer::live)
    float* in = nullptr;
    float* out = nullptr;
    float* spec = nullptr;
    int64_t in_off = 0, out_off = 0, spec_off = 0;
};

// One resident K_call<e> kernel and its request ring.  Single-owner: callers
// serialise access (the objects are single-threaded like the reference's).
class CallServer {
   public:
    static int create(int device, int e, int depth, size_t in_cap, size_t out_cap, size_t spec_cap,
                      CallServer** out);
    ~CallServer();
    CallServer(const CallServer&) = delete;
    CallServer& operator=(const CallServer&) = delete;

    // make every slot hold at least these many floats (drains and reallocates)
    int grow(size_t in_cap, size_t out_cap, size_t spec_cap);
    // the slots of the next request (waits until their previous user finished)
    int next_slot(CallSlot* sl);
    // copy n input floats into an input slot (write-combined when in device memory)
    void put(float* dst, const float* src, size_t n);
    // fill the slot offsets of r, post it, ring the doorbell, (re)launch if needed
    int submit(CallReq& r, const CallSlot& sl);
    int wait(uint64_t index);       // request `index` completed (its out slot is readable)
    int wait_spec(uint64_t index);  // ... and its speculation slot
    int wait_chain(uint64_t index); // ... and its chained produce block (kCallChain)
    // Ring work deferred onto the next request (CallReq::Pend): a commit and
    // then a clear of one ring; anything that cannot merge flushes first.
    int defer(const CallReq::Pend& p);
    int flush();                    // post the deferred work now (an op-0 request)
    int drain();                    // every submitted request (and speculation) completed
    int stop();                     // kernel gone (requests already completed stay so)
    // the next request runs an agent-scope acquire first (the object's device
    // state was written by kernels on other streams since the last request)
    void acquire_next() { acquire_next_ = true; }
    uint64_t submitted() const { return q_; }
    const CallReq::Pend& pending() const { return pend_; }  // the ring work the next request carries
    // the slot's views still point into the current arenas (grow() reallocates
    // them: a speculation recorded before a grow is gone)
    bool live(const CallSlot& s) const { return s.gen == gen_ && gen_ != 0; }
    uint64_t done() const { return __atomic_load_n(&hctl_->done, __ATOMIC_ACQUIRE); }
    int device() const { return device_; }
    const CallHostCtl* host_ctl() const { return hctl_; }  // diagnostics (phase stamps)

    // An OLA ring a request that timed out still changes (or changed) on the device
    // while the host gave up on it: its object's bookkeeping no longer matches the
    // ring, so its calls fail until reset() (which zeroes the ring and unpoisons it).
    bool poisoned(const float* ring) const;
    void unpoison(const float* ring);

   private:
    CallServer() = default;
    int alloc(size_t in_cap, size_t out_cap, size_t spec_cap);
    void release();
    int launch();
    bool running();
    int wait_counter(const uint64_t* ctr, uint64_t target);
    void store_ctl(uint64_t* p, uint64_t v);

    int device_ = 0, e_ = 0, depth_ = 4;
    hipStream_t s_ = nullptr;
    hipEvent_t ev_ = nullptr;  // recorded after each launch: complete = kernel gone
    bool launched_ = false;
    bool wc_inputs_ = false;   // input block in fine-grained device memory (BAR writes)
    bool acquire_next_ = false;
    char* dblk_ = nullptr;     // fine-grained device block (host-mapped)
    char* dhost_ = nullptr;    // ... or pinned host block (fallback)
    char* ddev_ = nullptr;     // device view of the input block
    char* hblk_ = nullptr;     // pinned host block
    char* hctl_dev_ = nullptr; // device view of hblk_
    CallCtl* ctl_ = nullptr;
    CallReq* reqs_ = nullptr;
    float* in_ = nullptr;
    CallHostCtl* hctl_ = nullptr;
    float* out_ = nullptr;
    size_t in_cap_ = 0, out_cap_ = 0, spec_cap_ = 0;
    uint64_t q_ = 0;                   // requests submitted
    uint64_t gen_ = 0;                 // arena generation (bumped by every allocation)
    bool broken_ = false;              // a request timed out: the server refuses new work ...
    uint64_t broken_at_ = 0;           // ... until done() reaches the requests submitted by then
    // per slot: the OLA rings the request there changes (its add / produce / chained
    // produce ring, and the ring of the deferred work it carries)
    std::vector<const float*> slot_rings_;
    // rings a timed-out request changes behind the host's bookkeeping (poisoned())
    std::vector<const float*> poisoned_;
    void timed_out(uint64_t done_seen);  // the timeout paths of wait_counter (done_seen: < the target)
    std::vector<uint64_t> spec_req_;   // per slot: request with a pending speculation (0: none)
    uint64_t last_chain_ = 0;          // the last request with a chained produce
    CallReq::Pend pend_{};             // deferred ring work (flags 0: none)
    uint64_t last_late_ = 0;           // the last request that ran its ring work late (kCallPendLate)
    uint64_t idle_ticks_ = 0;
    double tick_ns_ = 10.0;
};

// atexit: stop the per-device free-function servers (their kernels would
// otherwise idle out after the process began tearing the runtime down)
void stop_free_function_servers();

// The produce block an OLA object expects after its next push, as the forward
// FFT of the frame it will push is being submitted (the chain of the drop-in
// per-frame loop: forward -> inverse -> push_frame_AoS(inverse output) ->
// produce).  Filled by the object (objects.cpp) through ChainTarget::predict.
struct ChainPred {
    float* ring = nullptr;
    const float* den = nullptr;
    const float* win = nullptr;  // the object's window (apply_window_inside) or null
    int64_t R = 0, N = 0;
    int64_t start = 0;           // predicted push start (absolute sample)
    int64_t rp = 0, n = 0;       // predicted produce: read position (absolute) and count
    float gain = 1.0f;
};
struct ChainTarget {
    const void* owner = nullptr;             // the OLA object
    bool (*predict)(const void* owner, ChainPred* out) = nullptr;
};

// One resident K_call<E> per (device, E), shared by every FFT plan of size
// N = 128 E on the device and by the OLA objects of frame size N there, so a
// frame's calls sit in ONE queue and the forward can speculate on the push and
// produce that follow it.  Callers hold `mu` around their requests.
struct SharedServer {
    std::mutex mu;
    CallServer* srv = nullptr;
    int e = 0;
    float* d_tw = nullptr;  // the size's pass twiddles and super twiddles (device, owned)
    float* d_st = nullptr;
    void* d_plan = nullptr; // e < 0 (any size): the Stockham pass plan (device, owned)
    int any_waves = 0;      // ... and how many transforms one request runs at once
    bool any_two = false;   // ... and whether its LDS keeps two chained frames (late commits)
    struct FftSpec {        // the inverse speculated after the last forward
        bool valid = false;
        uint64_t index = 0;
        int batch = 0;
        CallSlot slot;      // slot.out: the spectrum returned; slot.spec: its inverse
    } fft;
    struct Chain {          // the produce speculated after that inverse, for `target`
        bool valid = false;
        uint64_t index = 0;
        ChainPred pred;
        CallSlot slot;      // chained produce block at slot.spec + N
        // the frame the push must equal (host) and its arena offset (the deferred
        // commit's source after a relaunch): a chained forward's speculated inverse
        // (slot.spec), or a chained inverse request's own output (slot.out)
        const float* frame = nullptr;
        int64_t frame_off = 0;
    } chain;
    struct LastInverse {    // the last single-frame inverse request (the OLA association)
        bool valid = false;
        uint64_t index = 0;
        CallSlot slot;      // slot.out: the frame it returned
    } inv;
    ChainTarget target;     // the OLA object that pushed the last speculated inverse
    struct BatchSpec* batch = nullptr;  // batched speculation of the whole loop (batch.h)
};
// test-only (crlot_test_inject CRLOT_INJECT_CALL_TIMEOUT): the next k waits time out
bool test_timeout_now();
void test_inject_timeouts(int count);
// the shared server of (device, e) (created on first use; never destroyed);
// e < 0: the FFT-only server of complex size P = -e (any size, call_any_waves)
SharedServer* shared_server(int device, int e, int* rc);

// The rings of the live OLA objects (objects.cpp): a timed-out request poisons
// only those (a ring whose object is gone has no bookkeeping left to protect).
bool ola_ring_live(const float* ring);

}  // namespace crlot
