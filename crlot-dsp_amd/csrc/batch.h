// batch.h -- batched speculation of the reference's per-frame drop-in loop
// (internal; batch.cpp, hooks in abi.cpp fft_host and objects.cpp).
//
// bench/e2e_benchmark.cc:138-186 runs, per frame k of a signal pushed whole
// into a Framer:  pop -> p = frame * w -> IFftPlan::forward(p) -> inverse ->
// OLAAccumulator::push_frame_AoS(inverse, k H) -> produce(H).  Every call of
// that loop is a function of the signal, the window and the OLA object's
// tables, all known once the first forward arrives.  So at the first forward
// whose input is (bit for bit) the last popped Framer frame times a window
// table the library built, the library runs the WHOLE remaining chain as one
// batch on the device (analysis products, forward and inverse transforms of
// every frame; after the first push, the overlap-add of every frame with the
// object's window and divisors), copies the results to pinned host memory, and
// serves each later call from there -- but only after checking that the call's
// input bits and arguments are exactly the ones predicted, and with the very
// kernels (K_rfft / K_irfft / the gather's fma chain) whose bits equal the call
// kernel's.  The first call that differs ends the batch; the OLA object's
// device ring is then rebuilt from the frames it was served (materialize), so
// the next call sees exactly the state the individual calls would have left.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <vector>

#include "crlot_dsp.h"

struct crlot_ola;
struct crlot_plan;

namespace crlot {

struct SharedServer;

// Batches are bounded: at most kBatchWindow frames are transformed per chain, in
// windows.  When the callers reach a window's end the next forward starts the
// next window from the same source (its frames continue the logical signal),
// carrying the last frames' inverse outputs over on the device so that an
// attached OLA object's overlap-add continues across the seam; device and pinned
// buffers therefore hold at most kBatchWindow + kBatchWarm frames.
constexpr int64_t kBatchWindow = 512;
constexpr int64_t kGainMinRun = 4;  // inverses a learned gain must serve to count as fixed
constexpr int64_t kBatchWarm = 63;  // warm-up frames kept: ceil(N / H) - 1 for H >= N / 64

// The most recently popped mono Framer: accept(frame 0, hop) decides on the frame
// popped last (nothing is copied before), then the signal of its first
// max_frames frames is copied: frame j (j = 0: the frame just popped) =
// sig[j H : j H + N], zeros past the end.  *frames = frames covered, *total =
// frames the Framer still holds (from the popped one on), *source identifies the
// Framer.  False when there is none or accept refuses (objects.cpp).
bool framer_last_signal(int64_t n, int64_t max_frames, const std::function<bool(const float*, int64_t)>& accept,
                        std::vector<float>* sig, int64_t* hop, int64_t* frames, int64_t* total, uint64_t* source);
// The second source: the frames of the FrameQueue read last (getFrame /
// copyFrame), from the frame just read on (bench/performance_benchmark.cc:174-246
// feeds each FrameQueue frame, unwindowed, to the forward): accept(row 0) first,
// then at most max_frames rows copied [frames][n] into the buffer dst(floats)
// returns.  *first = the row's index in its queue.  False when there is none,
// accept refuses or dst returns null (objects.cpp).
bool framequeue_last_rows(int64_t n, int64_t max_frames, const std::function<bool(const float*)>& accept,
                          int64_t* hop, int64_t* frames, int64_t* total, int* device, uint64_t* source,
                          int64_t* first, const std::function<float*(size_t)>& dst);
// The OLA object whose window was set last, when it is a mono, untouched,
// apply_window_inside object of frame n, hop h on `device` (the harness builds it
// before the loop, performance_benchmark.cc:195-197): its device window and
// divisors, with `s` ordered after their upload, so a new batch can compute that
// object's overlap-add speculatively (its first push is then served without a
// device round trip).  tgen: its tables' generation (OLA upload_norm).
struct FreshOla {
    crlot_ola* o = nullptr;
    const float* d_win = nullptr;
    const float* d_den = nullptr;
    int64_t R = 0;
    uint64_t tgen = 0;
};
bool fresh_ola(int64_t n, int64_t h, int device, hipStream_t s, FreshOla* out);
// Window tables the library built (crlot_window_table) or was handed
// (OLAAccumulator::set_window), newest first, for the speculation's search.
void note_window(const float* w, int64_t n);
std::vector<std::vector<float>> windows_of_size(int64_t n);

// 1: the per-call speculation of the call server only; 2 (default): batched
// speculation of the whole loop too (crlot_set_call_speculation)
int spec_mode();
enum { kStatStart = 0, kStatForward, kStatInverse, kStatPush, kStatProduce, kStatRebuild, kStatFrames, kStatWindows,
       kStatDeclined, kStatGains, kStatGainBackoffs, kStatCount };
void spec_count(int what);

struct BatchSpec {
    bool active = false;     // frames of the current window are being served
    uint64_t gen = 0;        // bumped by every start (not by a window continuation)
    int64_t n = 0, h = 0;
    int64_t M = 0;           // frames of the whole batch (the source's frames at the start)
    // the window: frames [wb, we) are served; the buffers hold frames [cb, we)
    // (cb < wb: inverse outputs carried over from the previous window, for the
    // attached object's overlap-add); buffer row of frame j = j - cb
    int64_t cb = 0, wb = 0, we = 0;
    uint64_t source = 0;     // the Framer / FrameQueue the frames come from
    int64_t src_first = 0;   // FrameQueue: queue index of frame 0 of the batch
    std::vector<float> sig;  // host copy of the window's signal from frame wb on (verifies forward inputs)
    std::vector<float> win;  // the analysis window found
    bool rows_src = false;   // the FrameQueue source: forward inputs are the rows themselves
    int64_t next_fwd = 0;    // frame whose forward comes next
    int64_t inv_ready = -1;  // frame whose forward was served and whose inverse may be asked
    int64_t pushed = -1;     // last frame whose inverse was served (push candidate)
    // device / pinned buffers (grow-only, at most kBatchWindow + kBatchWarm
    // frames).  The chain's results share one block each side (one copy back):
    // spectra [rows][N + 2] (interleaved complex), inverse frames [rows][N] (=
    // push inputs), produce blocks [rows H + N - H] (after attach), and the fresh
    // object's wrapped produce [R] (spec_ola)
    hipStream_t s = nullptr;
    hipEvent_t ev = nullptr;
    float* d_sig = nullptr;
    float* d_p = nullptr;    // [rows][N] analysis products
    float* d_blk = nullptr;
    float* h_blk = nullptr;
    float* m_blk = nullptr;    // h_blk / h_stage as the device addresses them (mapped pinned memory)
    float* m_stage = nullptr;
    float* d_spec = nullptr; // views into d_blk / h_blk
    float* d_r = nullptr;
    float* d_y = nullptr;
    float* h_spec = nullptr;
    float* h_r = nullptr;
    float* h_y = nullptr;
    float* d_acc = nullptr;  // [R] ring slots of a push-everything-first object (batch_alias)
    float* d_ya = nullptr;   // [R] their produce (batch_alias without spec_ola)
    float* h_ya = nullptr;
    const float* ya = nullptr;  // the wrapped produce in use (h_ya or in h_blk)
    float* h_stage = nullptr;  // the FrameQueue source: its rows of the window (verifies forward inputs)
    float* d_den_rot = nullptr;  // [R] the attached object's divisors from the window's origin on
    size_t c_sig = 0, c_p = 0, c_blk = 0, c_hblk = 0, c_hs = 0, c_acc = 0, c_ya = 0, c_hya = 0, c_den_rot = 0;
    size_t rows_cap = 0;     // frames the result block was laid out for
    // the OLA object the batch's inverses are pushed to (objects.cpp)
    crlot_ola* ola = nullptr;
    int64_t j0 = 0;          // first frame pushed to it
    float gain = 1.0f;
    const float* ola_ws = nullptr;  // its device window and divisors, ring length (batch_attach)
    const float* ola_den = nullptr;
    int64_t ola_R = 0;
    bool y_ready = false;    // h_y holds the object's produce blocks (event ev)
    bool y_waited = false;
    int64_t y_base = 0;      // position (from j0 H) of h_y[0]
    int64_t y_lo = 0;        // first position h_y holds completely (the window's carried frames reach it)
    // the overlap-add computed with the chain for a fresh OLA object (fresh_ola),
    // gain 1 and j0 = 0: h_y and the wrapped d_acc / h_ya, used if it attaches so
    FreshOla spec_ola;
    bool spec_y = false;     // computed with this batch
    bool spec_used = false;  // the attached object is the one it was computed for
    // the caller's spectral step, when it is a fixed real gain per bin (learned
    // from an inverse input the batch did not predict, batch_inverse): the
    // inverses of frames from sgain_from on are those of fl(gain * spectrum), and
    // an inverse is served only if its input is those products bit for bit
    std::vector<float> sgain;  // [N/2 + 1]; empty: the identity step
    int64_t sgain_from = 0;
    int64_t learn_after = -1;  // no new learning attempt before this frame (after a failed one)
    int64_t gain_served = 0;   // inverses served with the gain learned last
    int64_t learn_backoff = 16;  // frames without learning after a gain that did not last
    float* d_sgain = nullptr;
    float* d_specg = nullptr;  // [rows][N + 2] gained spectra (the inverse's input)
    size_t c_sgain = 0, c_specg = 0;
    bool single() const { return cb == 0 && we == M; }  // one window holds every frame
    size_t row(int64_t j) const { return size_t(j - cb); }
};

// objects.cpp: the attached object's state allows its overlap-add to continue
// into the next window (every frame before `we` pushed and read up to `we`'s
// position, no wrap); *first = the first frame whose unread contributions remain
bool ola_can_continue(const crlot_ola* o, const BatchSpec* b);

// abi.cpp fft_host, under sh->mu: a contiguous batch-1 real forward / inverse.
// 1: served into `out`; 0: not (take the ordinary path); < 0: error.
int batch_forward(SharedServer* sh, crlot_plan* inner, int64_t n, const float* in, float* out);
// inner: the FFT plan (null: serve only, never learn a spectral gain -- the
// early path before the device guard)
int batch_inverse(SharedServer* sh, crlot_plan* inner, int64_t n, const float* in, float* out);
// ends the batch (a call it does not predict); an attached OLA object is
// materialized first (objects.cpp ola_materialize_locked)
int batch_abort(SharedServer* sh);
// objects.cpp, under sh->mu
int ola_materialize_locked(crlot_ola* o);
// the batch's gather for an OLA object attaching at frame j0 (objects.cpp passes
// its tables): produce blocks of frames j0 .. M-1, and the N - H samples after
// them that only those frames reach, into h_y
int batch_attach(SharedServer* sh, crlot_ola* o, int64_t j0, int64_t R, const float* d_ws, const float* d_den,
                 float gain, hipStream_t tables_stream, uint64_t tgen);
int batch_wait_y(BatchSpec* b);
// abi.cpp: the plan's K_rfft + K_irfft in one launch (CRLOT_EUNSUPPORTED: none)
int plan_rfft_irfft(crlot_plan* p, const float* in, float* spec, float* r, float* r_host, int32_t batch,
                    void* stream);
// the attached object's ring once every batch frame j0 .. M-1 was pushed with no
// produce between, the later pushes wrapping onto unread slots (the reference
// harness's order, bench/performance_benchmark.cc:212-231): slots into d_acc,
// their produce into h_ya (waited for)
int batch_alias(BatchSpec* b, int64_t R, const float* d_ws, const float* d_den);

}  // namespace crlot
