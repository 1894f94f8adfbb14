// batch.cpp -- batched speculation of the per-frame drop-in loop (batch.h).
#include "batch.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "ab.h"
#include "call.h"
#include "kernels.h"

namespace crlot {
int set_error(int code, const std::string& msg);  // abi.cpp
}

namespace crlot {
namespace {

int hip_fail(hipError_t e, const char* what) {
    return set_error(CRLOT_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

std::atomic<int> g_mode{2};
constexpr float kOne = 1.0f;
// crlot_call_speculation_stats: batches started, forwards / inverses / pushes /
// produces served from a batch, OLA rings rebuilt
std::atomic<int64_t> g_stats[kStatCount];

std::mutex g_win_mu;
std::vector<std::vector<float>> g_windows;  // newest first
constexpr size_t kMaxWindows = 16;

// crlot_test_inject(CRLOT_INJECT_BATCH_ALLOC, k): the next k batch buffer
// allocations fail (tests of the fail-soft path)
std::atomic<int> g_fail_alloc{0};
bool injected_failure() {
    int v = g_fail_alloc.load(std::memory_order_relaxed);
    while (v > 0)
        if (g_fail_alloc.compare_exchange_weak(v, v - 1, std::memory_order_relaxed)) return true;
    return false;
}

// bytes the batches hold (crlot_call_batch_capacity): device, pinned, pinned peak
std::atomic<int64_t> g_dev_bytes{0}, g_pin_bytes{0}, g_pin_peak{0};

// grow-only device and pinned buffers
hipError_t dgrow(float** p, size_t* cap, size_t need) {
    if (*cap >= need) return hipSuccess;
    if (injected_failure()) return hipErrorOutOfMemory;
    if (*p) (void)hipFree(*p);
    g_dev_bytes.fetch_sub(int64_t(*cap * sizeof(float)));
    *p = nullptr;
    *cap = 0;
    hipError_t e = hipMalloc(p, sizeof(float) * need);
    if (e == hipSuccess) {
        *cap = need;
        g_dev_bytes.fetch_add(int64_t(need * sizeof(float)));
    }
    return e;
}
hipError_t hgrow(float** p, size_t* cap, size_t need) {
    if (*cap >= need) return hipSuccess;
    if (injected_failure()) return hipErrorOutOfMemory;
    if (*p) (void)hipHostFree(*p);
    g_pin_bytes.fetch_sub(int64_t(*cap * sizeof(float)));
    *p = nullptr;
    *cap = 0;
    hipError_t e = hipHostMalloc(p, sizeof(float) * need, hipHostMallocDefault);
    if (e == hipSuccess) {
        *cap = need;
        const int64_t now = g_pin_bytes.fetch_add(int64_t(need * sizeof(float))) + int64_t(need * sizeof(float));
        int64_t pk = g_pin_peak.load();
        while (now > pk && !g_pin_peak.compare_exchange_weak(pk, now)) {
        }
    }
    return e;
}

// A/B (CRLOT_BATCH_ZC, default 3): bit 0, the first forward of a FrameQueue
// batch reads the pinned rows over the host link instead of after a copy engine
// upload
int zc_mode() {
    static const int v = [] {
        const char* e = ab_env("CRLOT_BATCH_ZC");
        return e ? std::atoi(e) : 3;
    }();
    return v;
}
bool zero_copy_in() { return (zc_mode() & 1) != 0; }
// (CRLOT_BATCH_ZC bit 1: the chain's kernels write the host copies of their
// results themselves)
bool zero_copy_out() { return (zc_mode() & 2) != 0; }
// A/B (CRLOT_BATCH_FUSE=0): forward and inverse as two launches
bool fuse_fft() {
    static const bool v = [] {
        const char* e = ab_env("CRLOT_BATCH_FUSE");
        return !(e && e[0] == '0');
    }();
    return v;
}

// A/B builds (CRLOT_BATCH_TRACE=1): the phases of batch starts, summed, printed
// at exit: source search + rows copy, enqueue, wait
#ifdef CRLOT_AB_SWITCHES
// phases of each start: 0 source search + rows copy, 1 stream/tables/buffers,
// 2 upload, 3 forward launch, 4 inverse launch, 5 overlap-add launches, 6 copy
// back + record, 7 wait; medians printed at exit
struct BatchTrace {
    std::vector<double> us[8];
    ~BatchTrace() {
        if (us[0].empty()) return;
        std::fprintf(stderr, "batch_trace starts=%zu median_us:", us[0].size());
        for (auto& v : us) {
            std::sort(v.begin(), v.end());
            std::fprintf(stderr, " %.2f", v.empty() ? 0.0 : v[v.size() / 2]);
        }
        std::fprintf(stderr, "\n");
    }
};
BatchTrace g_trace;
bool trace_on() {
    static const bool v = [] {
        const char* e = ab_env("CRLOT_BATCH_TRACE");
        return e && e[0] == '1';
    }();
    return v;
}
using tclk = std::chrono::steady_clock;
struct PhaseClock {
    tclk::time_point t = tclk::now();
    void lap(int i) {
        if (!trace_on()) return;
        const auto n = tclk::now();
        g_trace.us[i].push_back(std::chrono::duration<double, std::micro>(n - t).count());
        t = n;
    }
};
thread_local PhaseClock g_pc;
#define CRLOT_LAP(i) g_pc.lap(i)
#define CRLOT_LAP_START() (g_pc.t = tclk::now())
#else
#define CRLOT_LAP(i) ((void)0)
#define CRLOT_LAP_START() ((void)0)
#endif

// the forward input of frame j, as the loop forms it on the host (frame * w)
bool input_matches(const BatchSpec& b, int64_t j, const float* in) {
    if (b.rows_src)
        return std::memcmp(in, b.h_stage + size_t(j - b.wb) * size_t(b.n), sizeof(float) * size_t(b.n)) == 0;
    // the products into a scratch row, then one compare (a loop the compiler
    // vectorises; the same IEEE products); sig starts at frame wb
    const int64_t L = int64_t(b.sig.size()), base = (j - b.wb) * b.h, n = b.n;
    const int64_t lim = std::max<int64_t>(0, std::min<int64_t>(n, L - base));
    thread_local std::vector<float> row;
    if (int64_t(row.size()) < n) row.resize(size_t(n));
    float* r = row.data();
    const float* sg = b.sig.data() + (lim > 0 ? base : 0);
    const float* w = b.win.data();
    for (int64_t i = 0; i < lim; ++i) r[i] = sg[i] * w[i];
    for (int64_t i = lim; i < n; ++i) r[i] = 0.0f * w[i];
    return std::memcmp(r, in, sizeof(float) * size_t(n)) == 0;
}

// The result block laid out for `rows` frames (spectra [rows][N + 2], inverse
// frames [rows][N], produce blocks [rows H + N - H], a fresh object's wrapped
// produce [R]) and its views.
size_t y_floats(const BatchSpec* b, size_t rows) {
    return rows * size_t(b->h) + size_t(std::max<int64_t>(0, b->n - b->h));
}
void set_views(BatchSpec* b) {
    const size_t N = size_t(b->n), rows = b->rows_cap, row = N + 2;
    b->d_spec = b->d_blk;
    b->d_r = b->d_spec + rows * row;
    b->d_y = b->d_r + rows * N;
    b->h_spec = b->h_blk;
    b->h_r = b->h_spec + rows * row;
    b->h_y = b->h_r + rows * N;
}
// buffers for `rows` frames (whatever they held is dropped when they grow)
hipError_t ensure_rows(BatchSpec* b, size_t rows) {
    const size_t N = size_t(b->n), R = size_t(crlot_ring_len(b->n, b->h));
    const size_t blk = rows * (N + 2) + rows * N + y_floats(b, rows) + R;
    const size_t had = b->c_hblk;
    hipError_t e;
    if ((e = dgrow(&b->d_p, &b->c_p, rows * N)) || (e = dgrow(&b->d_blk, &b->c_blk, blk)) ||
        (e = hgrow(&b->h_blk, &b->c_hblk, blk)))
        return e;
    if (b->c_hblk != had || !b->m_blk) {
        void* m = nullptr;
        b->m_blk = hipHostGetDevicePointer(&m, b->h_blk, 0) == hipSuccess ? static_cast<float*>(m) : nullptr;
    }
    b->rows_cap = rows;
    set_views(b);
    return hipSuccess;
}

// the overlap-add of a fresh OLA object (fresh_ola) after the first window's
// inverse frames, both ways its produces may come (after each push; after every
// push, the ring wrapped -- meaningful for a one-window batch only): into the
// result block (zero-copy: its host side)
hipError_t launch_spec_ola(BatchSpec* b, int dev, bool zc_out) {
    b->spec_y = b->spec_used = false;
    if (b->cb != 0 || !fresh_ola(b->n, b->h, dev, b->s, &b->spec_ola)) return hipSuccess;
    const size_t N = size_t(b->n), rows = b->rows_cap, row = N + 2, R = size_t(b->spec_ola.R);
    const size_t F = size_t(b->we), ylen = y_floats(b, F);
    if (rows * row + rows * N + y_floats(b, rows) + R > std::min(b->c_blk, b->c_hblk)) return hipSuccess;
    hipError_t e;
    if ((e = dgrow(&b->d_acc, &b->c_acc, R))) return e;
    Geometry g;
    g.n = int(b->n);
    g.h = int(b->h);
    g.ring_len = int(R);
    g.gain = 1.0f;
    DevTables t;
    t.ws = b->spec_ola.d_win;
    t.den = b->spec_ola.d_den;
    float* yout = zc_out ? b->m_blk + (rows * row + rows * N) : b->d_y;
    if ((e = launch_ola_gather_wrap(g, t, b->d_r, b->n, int64_t(F), int64_t(ylen), b->d_acc, yout + ylen, b->s,
                                    yout)) ||
        (!zc_out && (e = hipMemcpyAsync(b->h_y, b->d_y, sizeof(float) * (ylen + R), hipMemcpyDeviceToHost, b->s))))
        return e;
    b->spec_y = true;
    return hipSuccess;
}

// the attached object's produce blocks over the buffer's frames [cb, we): the
// window's positions from wb on are complete (the carried frames reach the
// first ones)
hipError_t launch_ola_window(BatchSpec* b, bool zc_out) {
    const size_t N = size_t(b->n), rows = b->rows_cap, row = N + 2;
    const int64_t first = std::max(b->cb, b->j0);  // the object's frames in the buffers
    const int64_t F = b->we - first;
    const size_t ylen = y_floats(b, size_t(F));
    // the gather divides position p by den[p mod R] from its own origin, frame
    // first's start, which sits (first - j0) H into the object's ring: a rotated
    // copy of the divisors puts that origin at index 0
    const size_t R = size_t(b->ola_R), off = size_t((first - b->j0) * b->h) % R;
    hipError_t e;
    if ((e = dgrow(&b->d_den_rot, &b->c_den_rot, R)) ||
        (e = hipMemcpyAsync(b->d_den_rot, b->ola_den + off, sizeof(float) * (R - off), hipMemcpyDeviceToDevice, b->s)) ||
        (off > 0 && (e = hipMemcpyAsync(b->d_den_rot + (R - off), b->ola_den, sizeof(float) * off,
                                        hipMemcpyDeviceToDevice, b->s))))
        return e;
    Geometry g;
    g.n = int(b->n);
    g.h = int(b->h);
    g.ring_len = int(R);
    g.gain = b->gain;
    DevTables t;
    t.ws = b->ola_ws;
    t.den = b->d_den_rot;
    float* yout = zc_out ? b->m_blk + (rows * row + rows * N) : b->d_y;
    if ((e = launch_ola_gather(g, t, b->d_r + b->row(first) * N, b->n, yout, 1, F, int64_t(ylen), int64_t(ylen),
                               b->s)) ||
        (!zc_out && (e = hipMemcpyAsync(b->h_y, b->d_y, sizeof(float) * ylen, hipMemcpyDeviceToHost, b->s))))
        return e;
    b->y_base = (first - b->j0) * b->h;
    b->y_lo = (std::max(b->wb, first) - b->j0) * b->h;
    b->y_ready = true;
    b->y_waited = false;
    return hipSuccess;
}

// the window's new frames [wb, we) (carry frames before them already in rows
// [0, carry) of d_r): products, forward, inverse, and the overlap-add of the
// attached object (continuing) or of a fresh one (first window); results to
// pinned memory; enqueued on b->s up to the event b->ev (run_chain waits for it)
int launch_chain(BatchSpec* b, crlot_plan* inner, int64_t carry) {
    const size_t N = size_t(b->n), F = size_t(b->we - b->wb), rows = b->rows_cap, row = N + 2;
    const size_t L = b->sig.size();
    hipError_t e;
    if (!b->s && (e = hipStreamCreateWithFlags(&b->s, hipStreamNonBlocking)) != hipSuccess)
        return hip_fail(e, "batch stream");
    if (!b->ev && (e = hipEventCreateWithFlags(&b->ev, hipEventDisableTiming)) != hipSuccess)
        return hip_fail(e, "batch event");
    b->spec_y = b->spec_used = false;
    int dev = -1;
    if ((e = hipGetDevice(&dev))) return hip_fail(e, "batch device");
    if (size_t(carry) + F > rows) return set_error(CRLOT_ERUNTIME, "batch window exceeds its buffers");
    // zero-copy (default): the kernels read the pinned rows and write the host
    // copies of their results themselves -- no copy engine, one dependent launch
    // fewer per copy
    const bool zc_out = zero_copy_out() && b->m_blk;
    CRLOT_LAP(1);
    const float* d_in = b->d_p;
    if (b->rows_src) {  // the FrameQueue's rows (already in h_stage) are the forward inputs
        if (zero_copy_in() && b->m_stage)
            d_in = b->m_stage;
        else if ((e = hipMemcpyAsync(b->d_p, b->h_stage, sizeof(float) * F * N, hipMemcpyHostToDevice, b->s)))
            return hip_fail(e, "batch frames");
    } else {
        b->m_stage = nullptr;  // (h_stage may move; the rows source maps it again)
        if ((e = dgrow(&b->d_sig, &b->c_sig, L + N)) || (e = hgrow(&b->h_stage, &b->c_hs, L + N)))
            return hip_fail(e, "batch buffers");
        std::memcpy(b->h_stage, b->sig.data(), sizeof(float) * L);
        std::memcpy(b->h_stage + L, b->win.data(), sizeof(float) * N);
        if ((e = hipMemcpyAsync(b->d_sig, b->h_stage, sizeof(float) * (L + N), hipMemcpyHostToDevice, b->s)) ||
            (e = launch_windowed_frames(b->d_sig, int64_t(L), b->d_sig + L, b->d_p, int64_t(F), b->n, b->h, b->s)))
            return hip_fail(e, "batch frames");
    }
    CRLOT_LAP(2);
    // forward + inverse: one launch where the plan has the fused kernel; with a
    // learned spectral gain, forward, the gain and inverse as three
    const size_t c = size_t(carry);
    float* spec_dev = b->d_spec + c * row;
    float* r_dev = b->d_r + c * N;
    const bool gained = !b->sgain.empty();
    bool spec_r_host = false;
    int rc = fuse_fft() && !gained
                 ? plan_rfft_irfft(inner, d_in, zc_out ? b->m_blk + c * row : spec_dev, r_dev,
                                   zc_out ? b->m_blk + rows * row + c * N : nullptr, int32_t(F), b->s)
                 : CRLOT_EUNSUPPORTED;
    if (rc == CRLOT_OK) {
        spec_r_host = zc_out;
    } else if (rc == CRLOT_EUNSUPPORTED) {
        rc = crlot_rfft_batched(inner, d_in, spec_dev, int32_t(F), int64_t(N), 1, int64_t(row), 1, b->s);
        CRLOT_LAP(3);
        const float* inv_in = spec_dev;
        if (rc == CRLOT_OK && gained) {
            if ((e = dgrow(&b->d_specg, &b->c_specg, rows * row)) ||
                (e = launch_bin_gain(spec_dev, b->d_specg, b->d_sgain, int64_t(F), int64_t(row), int64_t(N / 2 + 1),
                                     b->s)))
                return hip_fail(e, "batch spectral gain");
            inv_in = b->d_specg;
        }
        if (rc == CRLOT_OK)
            rc = crlot_irfft_batched(inner, inv_in, r_dev, int32_t(F), int64_t(row), 1, int64_t(N), 1, b->s);
    }
    if (rc != CRLOT_OK) return rc;
    CRLOT_LAP(4);
    if (!spec_r_host &&
        ((e = hipMemcpyAsync(b->h_spec + c * row, spec_dev, sizeof(float) * F * row, hipMemcpyDeviceToHost, b->s)) ||
         (e = hipMemcpyAsync(b->h_r + c * N, r_dev, sizeof(float) * F * N, hipMemcpyDeviceToHost, b->s))))
        return hip_fail(e, "batch results");
    if ((e = b->ola ? launch_ola_window(b, zc_out) : launch_spec_ola(b, dev, zc_out)))
        return hip_fail(e, "batch overlap-add");
    CRLOT_LAP(5);
    if ((e = hipEventRecord(b->ev, b->s))) return hip_fail(e, "batch results");
    CRLOT_LAP(6);
    g_stats[kStatFrames].fetch_add(int64_t(F), std::memory_order_relaxed);
    return CRLOT_OK;
}

int run_chain(BatchSpec* b, crlot_plan* inner, int64_t carry) {
    const int rc = launch_chain(b, inner, carry);
    if (rc != CRLOT_OK) return rc;
    const hipError_t e = hipEventSynchronize(b->ev);
    if (e != hipSuccess) return hip_fail(e, "batch results");
    if (b->ola) b->y_waited = true;
    CRLOT_LAP(7);
    return CRLOT_OK;
}

// frame 0 of a source against the caller's input: (frame * w) bit for bit, for
// one of the library's windows
const std::vector<float>* window_match(const float* frame0, const float* in, int64_t n,
                                       const std::vector<std::vector<float>>& wins) {
    for (const auto& w : wins) {
        bool ok = true;
        for (int64_t i = 0; i < n && ok; ++i) {
            const float v = frame0[i] * w[size_t(i)];
            ok = std::memcmp(&v, in + i, sizeof(float)) == 0;
        }
        if (ok) return &w;
    }
    return nullptr;
}

// the pinned staging rows of the FrameQueue source (mapped for zero-copy reads)
float* stage_rows(BatchSpec* b, size_t floats, hipError_t* he) {
    const size_t had = b->c_hs;
    *he = hgrow(&b->h_stage, &b->c_hs, floats);
    if (*he != hipSuccess) return nullptr;
    if (b->c_hs != had || !b->m_stage) {
        void* m = nullptr;
        b->m_stage = hipHostGetDevicePointer(&m, b->h_stage, 0) == hipSuccess ? static_cast<float*>(m) : nullptr;
    }
    return b->h_stage;
}

// A speculation that could not start or continue: the caller's own path runs.
// Clears the error a failed allocation or launch recorded.
int decline(BatchSpec* b) {
    b->active = false;
    b->inv_ready = b->pushed = -1;
    b->we = b->next_fwd;  // nothing more is served from this batch
    b->M = b->we;
    (void)hipGetLastError();
    g_stats[kStatDeclined].fetch_add(1, std::memory_order_relaxed);
    return 0;
}

// The next window of a running batch: the forward of frame we, read from the
// same source.  1: served; 0: not a continuation (or declined); < 0: error.
int continue_window(SharedServer* sh, BatchSpec* b, crlot_plan* inner, int64_t n, const float* in, float* out) {
    int64_t hop = 0, F = 0, total = 0;
    uint64_t src = 0;
    if (!b->rows_src) {
        std::vector<float> sig;
        const std::vector<float>* w = &b->win;
        auto accept = [&](const float* f0, int64_t h) { return h == b->h && window_match(f0, in, n, {*w}) != nullptr; };
        if (!framer_last_signal(n, kBatchWindow, accept, &sig, &hop, &F, &total, &src)) return 0;
        if (src != b->source || total != b->M - b->we) return 0;
        b->sig.swap(sig);
    } else {
        int qdev = -1;
        int64_t first = 0;
        hipError_t he = hipSuccess;
        auto accept = [&](const float* r0) { return std::memcmp(r0, in, sizeof(float) * size_t(n)) == 0; };
        auto dst = [&](size_t floats) { return stage_rows(b, floats, &he); };
        const bool got = framequeue_last_rows(n, kBatchWindow, accept, &hop, &F, &total, &qdev, &src, &first, dst);
        if (he != hipSuccess) return decline(b);
        if (!got) return 0;
        if (src != b->source || first != b->src_first + b->we || hop != b->h || total != b->M - b->we) return 0;
    }
    // the attached object: carry its last frames' inverse outputs over, or rebuild
    // its ring now, while the frames it needs are still in the buffers
    int64_t carry = 0;
    if (b->ola) {
        const int64_t P = (b->n + b->h - 1) / b->h - 1, first = std::max(b->we - P, b->j0);
        const bool keep = P <= kBatchWarm && first >= b->cb && b->row(first) >= size_t(b->we - first) &&
                          size_t(b->we - first) + size_t(F) <= b->rows_cap && ola_can_continue(b->ola, b);
        if (keep) {
            carry = b->we - first;
        } else {
            crlot_ola* o = b->ola;
            b->ola = nullptr;
            const int rc = ola_materialize_locked(o);
            if (rc != CRLOT_OK) return rc;
        }
    }
    if (carry > 0) {
        const hipError_t e = hipMemcpyAsync(b->d_r, b->d_r + b->row(b->we - carry) * size_t(n),
                                            sizeof(float) * size_t(carry) * size_t(n), hipMemcpyDeviceToDevice, b->s);
        if (e != hipSuccess) {
            crlot_ola* o = b->ola;  // (its frames are still in place)
            b->ola = nullptr;
            const int rc = ola_materialize_locked(o);
            return rc != CRLOT_OK ? rc : decline(b);
        }
    }
    b->cb = b->we - carry;
    b->wb = b->we;
    b->we = b->wb + F;
    b->next_fwd = b->wb;
    b->pushed = -1;
    if (size_t(carry) + size_t(F) > b->rows_cap || run_chain(b, inner, carry) != CRLOT_OK) {
        if (b->ola) {  // the frames it still needs are the carried rows [0, carry)
            crlot_ola* o = b->ola;
            b->ola = nullptr;
            // the carry copy above runs on b->s; the rebuild reads those rows on the
            // object's own stream, which nothing orders after b->s
            (void)hipStreamSynchronize(b->s);
            const int rc = ola_materialize_locked(o);
            if (rc != CRLOT_OK) return rc;
        }
        return decline(b);
    }
    sh->fft.valid = false;
    sh->chain.valid = false;
    b->active = true;
    spec_count(kStatWindows);
    spec_count(kStatForward);
    std::memcpy(out, b->h_spec + b->row(b->wb) * (size_t(n) + 2), sizeof(float) * (size_t(n) + 2));
    b->next_fwd = b->wb + 1;
    b->inv_ready = b->wb;
    if (b->next_fwd == b->we) b->active = false;
    return 1;
}

}  // namespace

int spec_mode() { return g_mode.load(std::memory_order_relaxed); }
void spec_count(int what) { g_stats[what].fetch_add(1, std::memory_order_relaxed); }

void note_window(const float* w, int64_t n) {
    if (!w || n <= 0) return;
    std::lock_guard<std::mutex> lk(g_win_mu);
    for (size_t i = 0; i < g_windows.size(); ++i) {
        const auto& v = g_windows[i];
        if (int64_t(v.size()) == n && std::memcmp(v.data(), w, sizeof(float) * size_t(n)) == 0) {
            std::rotate(g_windows.begin(), g_windows.begin() + int64_t(i), g_windows.begin() + int64_t(i) + 1);
            return;
        }
    }
    g_windows.insert(g_windows.begin(), std::vector<float>(w, w + n));
    if (g_windows.size() > kMaxWindows) g_windows.pop_back();
}

std::vector<std::vector<float>> windows_of_size(int64_t n) {
    std::lock_guard<std::mutex> lk(g_win_mu);
    std::vector<std::vector<float>> out;
    for (const auto& v : g_windows)
        if (int64_t(v.size()) == n) out.push_back(v);
    return out;
}

int batch_abort(SharedServer* sh) {
    BatchSpec* b = sh->batch;
    if (!b) return CRLOT_OK;
    b->active = false;
    b->inv_ready = b->pushed = -1;
    if (b->ola) {
        const int rc = ola_materialize_locked(b->ola);  // detaches it
        b->ola = nullptr;
        return rc;
    }
    return CRLOT_OK;
}

int batch_serve_forward(SharedServer* sh, int64_t n, const float* in, float* out) {
    BatchSpec* b = sh->batch;
    if (!b || spec_mode() < 2 || !b->active || b->n != n) return 0;
    const int64_t j = b->next_fwd;
    if (j >= b->we || !input_matches(*b, j, in)) return 0;
    const size_t row = size_t(n) + 2;
    std::memcpy(out, b->h_spec + b->row(j) * row, sizeof(float) * row);
    b->next_fwd = j + 1;
    b->inv_ready = j;
    spec_count(kStatForward);
    if (b->next_fwd == b->we) b->active = false;  // window end: its inverse / push / produce still served
    return 1;
}

int batch_forward(SharedServer* sh, crlot_plan* inner, int64_t n, const float* in, float* out) {
    if (spec_mode() < 2) return 0;
    if (!sh->batch) sh->batch = new BatchSpec();
    BatchSpec* b = sh->batch;
    const size_t row = size_t(n) + 2;
    if (batch_serve_forward(sh, n, in, out)) return 1;
    CRLOT_LAP_START();
    if (!inner) return 0;
    // the next window of the running batch
    if (b->gen != 0 && b->n == n && b->next_fwd == b->we && b->we < b->M) {
        const int rc = continue_window(sh, b, inner, n, in, out);
        if (rc != 0) return rc;
    }
    // a forward the batch did not predict: end it, then try to start one here
    if (b->active || b->ola) {
        const int rc = batch_abort(sh);
        if (rc != CRLOT_OK) return rc;
    }
    b->inv_ready = b->pushed = -1;
    b->M = b->we = b->next_fwd = 0;
    // source 1: the Framer popped last, frame * a library window (the window
    // search on frame 0 before anything is copied)
    std::vector<float> sig;
    int64_t hop = 0, F = 0, total = 0, first = 0;
    uint64_t src = 0;
    const std::vector<float>* found = nullptr;
    std::vector<std::vector<float>> wins = windows_of_size(n);
    {
        auto accept = [&](const float* f0, int64_t) { return (found = window_match(f0, in, n, wins)) != nullptr; };
        if (!framer_last_signal(n, kBatchWindow, accept, &sig, &hop, &F, &total, &src) || total < 4) found = nullptr;
    }
    // source 2: the FrameQueue read last, its frame as it is (no window),
    // copied straight into the pinned staging block the upload reads
    if (!found) {
        int qdev = -1, cur = -1;
        hipError_t he = hipSuccess;
        auto accept = [&](const float* r0) { return std::memcmp(r0, in, sizeof(float) * size_t(n)) == 0; };
        auto dst = [&](size_t floats) { return stage_rows(b, floats, &he); };
        const bool got = framequeue_last_rows(n, kBatchWindow, accept, &hop, &F, &total, &qdev, &src, &first, dst);
        if (he != hipSuccess) return decline(b);
        if (!got || total < 4 || hipGetDevice(&cur) != hipSuccess || cur != qdev) return 0;
    }
    b->gen += 1;
    b->n = n;
    b->h = hop;
    b->M = total;
    b->cb = b->wb = 0;
    b->we = F;
    b->source = src;
    b->src_first = first;
    b->rows_src = found == nullptr;
    if (found) {
        b->sig.swap(sig);
        b->win = *found;
    } else {
        b->sig.clear();
        b->win.clear();
    }
    b->next_fwd = 0;
    b->y_ready = b->y_waited = false;
    b->ola = nullptr;
    b->sgain_from = 0;  // (a gain learned earlier is applied from the start: the likeliest caller)
    b->learn_after = -1;
    // a different gain at a new signal's first frames is a new caller's gain, not a
    // per-frame edit: it is learned at once (churn is judged within a signal)
    b->gain_served = kGainMinRun;
    b->learn_backoff = 16;
    if (!b->sgain.empty()) {
        const size_t bins = size_t(n) / 2 + 1;
        hipError_t ge = b->sgain.size() == bins ? dgrow(&b->d_sgain, &b->c_sgain, bins) : hipErrorInvalidValue;
        if (ge == hipSuccess && b->s)
            ge = hipMemcpyAsync(b->d_sgain, b->sgain.data(), sizeof(float) * bins, hipMemcpyHostToDevice, b->s);
        if (ge != hipSuccess || !b->s) b->sgain.clear();
    }
    CRLOT_LAP(0);
    // buffers for one window, plus the frames a continuing object carries over
    // when the batch has more than one
    const size_t rows = size_t(F) + (total > F ? size_t(kBatchWarm) : 0);
    if (ensure_rows(b, rows) != hipSuccess || run_chain(b, inner, 0) != CRLOT_OK) return decline(b);
    sh->fft.valid = false;  // the call server's own per-call speculation is not used meanwhile
    sh->chain.valid = false;
    b->active = true;
    spec_count(kStatStart);
    spec_count(kStatForward);
    std::memcpy(out, b->h_spec, sizeof(float) * row);
    b->next_fwd = 1;
    b->inv_ready = 0;
    if (b->next_fwd == b->we) b->active = false;
    return 1;
}

namespace {
// the inverse input the batch predicts for frame j: its spectrum, or the
// products with the learned gain (the caller's std::complex<float> *= float)
bool inverse_input_matches(const BatchSpec* b, int64_t j, const float* in) {
    const size_t row = size_t(b->n) + 2;
    const float* X = b->h_spec + b->row(j) * row;
    if (b->sgain.empty() || j < b->sgain_from) return std::memcmp(in, X, sizeof(float) * row) == 0;
    // bin by bin, stopping at the first difference (an edit that changes every
    // frame differs in the first bins: no full product row per call)
    const float* g = b->sgain.data();
    for (size_t k = 0; k < row / 2; ++k) {
        const float p[2] = {X[2 * k] * g[k], X[2 * k + 1] * g[k]};
        if (std::memcmp(p, in + 2 * k, sizeof(p)) != 0) return false;
    }
    return true;
}

// A real gain per bin that maps frame j's spectrum X onto the caller's input Y
// bit for bit (Y = X * g in float): g[k] = Y / X, checked, with its float
// neighbours as a fallback for the rounding of the division.  Bins where X is
// zero keep the previous gain (or 1): any gain reproduces them.
bool learn_gain(const BatchSpec* b, int64_t j, const float* Y, std::vector<float>* g) {
    const size_t bins = size_t(b->n) / 2 + 1;
    const float* X = b->h_spec + b->row(j) * (size_t(b->n) + 2);
    g->resize(bins);
    auto same = [](float a, float c) { return std::memcmp(&a, &c, sizeof(float)) == 0; };
    for (size_t k = 0; k < bins; ++k) {
        const float xr = X[2 * k], xi = X[2 * k + 1], yr = Y[2 * k], yi = Y[2 * k + 1];
        float q = b->sgain.size() == bins ? b->sgain[k] : 1.0f;
        if (same(xr * q, yr) && same(xi * q, yi)) {  // one frame need not pin a gain: keep the one
            (*g)[k] = q;                              // that reproduces the earlier frames too
            continue;
        }
        if (xr != 0.0f)
            q = yr / xr;
        else if (xi != 0.0f)
            q = yi / xi;
        if (!std::isfinite(q)) return false;
        const float cand[3] = {q, std::nextafter(q, INFINITY), std::nextafter(q, -INFINITY)};
        bool ok = false;
        for (float c : cand)
            if (same(xr * c, yr) && same(xi * c, yi)) {
                (*g)[k] = c;
                ok = true;
                break;
            }
        if (!ok) return false;
    }
    return true;
}

// the inverses of frames j .. we-1 of the buffers redone with the gain (and the
// attached object's produce blocks over them), waited for
int apply_gain(BatchSpec* b, crlot_plan* inner, int64_t j) {
    const size_t N = size_t(b->n), row = N + 2, bins = N / 2 + 1, F = size_t(b->we - j);
    hipError_t e;
    // the spectra as served (h_spec): the fused zero-copy chain wrote them to the
    // mapped host block only, so d_spec's rows may be stale
    float* spec = b->d_spec + b->row(j) * row;
    if ((e = dgrow(&b->d_sgain, &b->c_sgain, bins)) || (e = dgrow(&b->d_specg, &b->c_specg, b->rows_cap * row)) ||
        (e = hipMemcpyAsync(spec, b->h_spec + b->row(j) * row, sizeof(float) * F * row, hipMemcpyHostToDevice, b->s)) ||
        (e = hipMemcpyAsync(b->d_sgain, b->sgain.data(), sizeof(float) * bins, hipMemcpyHostToDevice, b->s)) ||
        (e = launch_bin_gain(spec, b->d_specg, b->d_sgain, int64_t(F), int64_t(row),
                             int64_t(bins), b->s)))
        return hip_fail(e, "batch spectral gain");
    float* r_dev = b->d_r + b->row(j) * N;
    int rc = crlot_irfft_batched(inner, b->d_specg, r_dev, int32_t(F), int64_t(row), 1, int64_t(N), 1, b->s);
    if (rc != CRLOT_OK) return rc;
    if ((e = hipMemcpyAsync(b->h_r + b->row(j) * N, r_dev, sizeof(float) * F * N, hipMemcpyDeviceToHost, b->s)))
        return hip_fail(e, "batch spectral gain");
    if (b->ola) {
        // the attached object's produce blocks over the redone rows; its wrapped ring
        // (the push-everything-first order) was precomputed from the inverses without
        // the gain when it attached with the chain: batch_alias rebuilds it from d_r
        b->spec_used = false;
        b->spec_y = false;
        if ((e = launch_ola_window(b, false))) return hip_fail(e, "batch overlap-add");
    } else {
        b->spec_y = false;  // a fresh object's blocks were of the inverses without the gain
    }
    if ((e = hipEventRecord(b->ev, b->s)) || (e = hipEventSynchronize(b->ev))) return hip_fail(e, "batch spectral gain");
    if (b->ola) b->y_waited = true;
    return CRLOT_OK;
}
}  // namespace

int batch_inverse(SharedServer* sh, crlot_plan* inner, int64_t n, const float* in, float* out) {
    BatchSpec* b = sh->batch;
    if (!b || spec_mode() < 2 || b->n != n || b->inv_ready < 0) return 0;
    const int64_t j = b->inv_ready;
    if (!inverse_input_matches(b, j, in)) {
        // a spectral step the batch does not know: learn it if it is a fixed real
        // gain per bin, and redo this window's remaining inverses with it
        if (!inner || j < b->learn_after) return 0;
        std::vector<float> g;
        if (!learn_gain(b, j, in, &g)) {
            b->learn_after = j + 16;
            return 0;
        }
        // A new gain right after the last one, different in many bins: the edit
        // changes from frame to frame (a time-varying mask), so redoing the
        // window's inverses for each would cost a chain per frame.  Those frames
        // take the per-call path; learning resumes after a backoff that doubles
        // each time (up to a window).  A gain that changes in a few bins only is
        // the same gain settling (bins one frame does not pin), applied at once.
        if (!b->sgain.empty() && b->gain_served < kGainMinRun) {
            size_t changed = 0;
            for (size_t k = 0; k < g.size(); ++k) changed += g[k] != b->sgain[k];
            if (changed * 8 > g.size()) {
                b->learn_after = j + b->learn_backoff;
                b->learn_backoff = std::min<int64_t>(2 * b->learn_backoff, kBatchWindow);
                g_stats[kStatGainBackoffs].fetch_add(1, std::memory_order_relaxed);
                return 0;
            }
        } else {
            b->learn_backoff = 16;
        }
        const std::vector<float> old = b->sgain;
        const int64_t old_from = b->sgain_from;
        b->sgain.swap(g);
        b->sgain_from = j;
        if (apply_gain(b, inner, j) != CRLOT_OK) {  // nothing served: the buffers hold the old inverses
            b->sgain = old;
            b->sgain_from = old_from;
            b->learn_after = j + 16;
            return decline(b);
        }
        spec_count(kStatGains);
        b->gain_served = 0;
        if (std::all_of(b->sgain.begin(), b->sgain.end(), [](float v) { return v == 1.0f; }))
            b->sgain.clear();  // the identity again (x * 1 is exact: the rows redone are its bits)
        if (!inverse_input_matches(b, j, in)) return 0;
    }
    std::memcpy(out, b->h_r + b->row(j) * size_t(n), sizeof(float) * size_t(n));
    b->inv_ready = -1;
    b->pushed = j;
    if (!b->sgain.empty()) b->gain_served += 1;
    spec_count(kStatInverse);
    return 1;
}

int batch_attach(SharedServer* sh, crlot_ola* o, int64_t j0, int64_t R, const float* d_ws, const float* d_den,
                 float gain, hipStream_t tables_stream, uint64_t tgen) {
    BatchSpec* b = sh->batch;
    b->ola_ws = d_ws;
    b->ola_den = d_den;
    b->ola_R = R;
    if (b->spec_y && b->spec_ola.o == o && b->spec_ola.tgen == tgen && b->spec_ola.R == R && j0 == 0 &&
        std::memcmp(&gain, &kOne, sizeof(float)) == 0) {  // computed with the chain (run_chain)
        b->ola = o;
        b->j0 = 0;
        b->gain = gain;
        b->y_ready = b->y_waited = true;
        b->y_base = b->y_lo = 0;
        b->spec_used = true;
        b->ya = b->h_y + y_floats(b, size_t(b->we));
        return CRLOT_OK;
    }
    b->spec_used = false;
    // blocks of the window's frames j0 .. we-1 and the tail only they reach (no
    // later frame is in the window; a produce there needs the last frame pushed)
    const size_t F = size_t(b->we - j0), len = y_floats(b, F);
    hipError_t e;
    if ((e = hipStreamSynchronize(tables_stream)) != hipSuccess) return hip_fail(e, "OLA tables");
    Geometry g;
    g.n = int(b->n);
    g.h = int(b->h);
    g.ring_len = int(R);
    g.gain = gain;
    DevTables t;
    t.ws = d_ws;
    t.den = d_den;
    if ((e = launch_ola_gather(g, t, b->d_r + b->row(j0) * size_t(b->n), b->n, b->d_y, 1, int64_t(F),
                               int64_t(len), int64_t(len), b->s)) ||
        (e = hipMemcpyAsync(b->h_y, b->d_y, sizeof(float) * len, hipMemcpyDeviceToHost, b->s)) ||
        (e = hipEventRecord(b->ev, b->s)))
        return hip_fail(e, "batch overlap-add");
    b->ola = o;
    b->j0 = j0;
    b->gain = gain;
    b->y_ready = true;
    b->y_waited = false;
    b->y_base = b->y_lo = 0;
    return CRLOT_OK;
}

int batch_wait_y(BatchSpec* b) {
    if (b->y_waited) return CRLOT_OK;
    const hipError_t e = hipEventSynchronize(b->ev);
    if (e != hipSuccess) return hip_fail(e, "batch overlap-add");
    b->y_waited = true;
    return CRLOT_OK;
}

int batch_alias(BatchSpec* b, int64_t R, const float* d_ws, const float* d_den) {
    if (b->spec_used) return CRLOT_OK;  // computed with the chain (b->ya)
    if (!b->single()) return set_error(CRLOT_ERUNTIME, "wrapped ring of a windowed batch");
    const int64_t F = b->M - b->j0, len = F * b->h + std::max<int64_t>(0, b->n - b->h);
    hipError_t e;
    if ((e = dgrow(&b->d_acc, &b->c_acc, size_t(R))) || (e = dgrow(&b->d_ya, &b->c_ya, size_t(R))) ||
        (e = hgrow(&b->h_ya, &b->c_hya, size_t(R))))
        return hip_fail(e, "batch buffers");
    Geometry g;
    g.n = int(b->n);
    g.h = int(b->h);
    g.ring_len = int(R);
    g.gain = b->gain;
    DevTables t;
    t.ws = d_ws;
    t.den = d_den;
    if ((e = launch_ola_gather_wrap(g, t, b->d_r + b->row(b->j0) * size_t(b->n), b->n, F, len, b->d_acc, b->d_ya,
                                    b->s)) ||
        (e = hipMemcpyAsync(b->h_ya, b->d_ya, sizeof(float) * size_t(R), hipMemcpyDeviceToHost, b->s)) ||
        (e = hipEventRecord(b->ev, b->s)) || (e = hipEventSynchronize(b->ev)))
        return hip_fail(e, "batch overlap-add (wrapped)");
    b->ya = b->h_ya;
    return CRLOT_OK;
}

}  // namespace crlot

extern "C" int crlot_call_speculation_stats(int64_t* out6) {
    if (!out6) return crlot::set_error(CRLOT_EINVAL, "null argument");
    for (int i = 0; i < 6; ++i) out6[i] = crlot::g_stats[i].load(std::memory_order_relaxed);
    return CRLOT_OK;
}

extern "C" int crlot_call_speculation_stats_ex(int64_t* out, int32_t count) {
    if (!out || count < 0) return crlot::set_error(CRLOT_EINVAL, "null argument");
    for (int i = 0; i < count; ++i)
        out[i] = i < crlot::kStatCount ? crlot::g_stats[i].load(std::memory_order_relaxed) : 0;
    return CRLOT_OK;
}

extern "C" int crlot_call_batch_capacity(int64_t* window_frames, int64_t* device_bytes, int64_t* pinned_bytes,
                                         int64_t* pinned_peak) {
    if (window_frames) *window_frames = crlot::kBatchWindow;
    if (device_bytes) *device_bytes = crlot::g_dev_bytes.load();
    if (pinned_bytes) *pinned_bytes = crlot::g_pin_bytes.load();
    if (pinned_peak) *pinned_peak = crlot::g_pin_peak.load();
    return CRLOT_OK;
}

extern "C" int crlot_test_inject(int32_t what, int32_t count) {
    if (count < 0) return crlot::set_error(CRLOT_EINVAL, "negative injection count");
    if (what == CRLOT_INJECT_BATCH_ALLOC) {
        crlot::g_fail_alloc.store(count, std::memory_order_relaxed);
    } else if (what == CRLOT_INJECT_CALL_TIMEOUT) {
        crlot::test_inject_timeouts(count);
    } else {
        return crlot::set_error(CRLOT_EINVAL, "unknown injection");
    }
    return CRLOT_OK;
}

extern "C" int crlot_set_call_speculation(int32_t mode) {
    if (mode < 1 || mode > 2) return crlot::set_error(CRLOT_EINVAL, "speculation mode is 1 or 2");
    crlot::g_mode.store(mode, std::memory_order_relaxed);
    return CRLOT_OK;
}
