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
std::atomic<int64_t> g_stats[6];

std::mutex g_win_mu;
std::vector<std::vector<float>> g_windows;  // newest first
constexpr size_t kMaxWindows = 16;

// grow-only device and pinned buffers
hipError_t dgrow(float** p, size_t* cap, size_t need) {
    if (*cap >= need) return hipSuccess;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    hipError_t e = hipMalloc(p, sizeof(float) * need);
    if (e == hipSuccess) *cap = need;
    return e;
}
hipError_t hgrow(float** p, size_t* cap, size_t need) {
    if (*cap >= need) return hipSuccess;
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    *cap = 0;
    hipError_t e = hipHostMalloc(p, sizeof(float) * need, hipHostMallocDefault);
    if (e == hipSuccess) *cap = need;
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
    if (b.rows_src) return std::memcmp(in, b.h_stage + size_t(j) * size_t(b.n), sizeof(float) * size_t(b.n)) == 0;
    // the products into a scratch row, then one compare (a loop the compiler
    // vectorises; the same IEEE products)
    const int64_t L = int64_t(b.sig.size()), base = j * b.h, n = b.n;
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

// run frames 0 .. M-1 of the found chain: products, forward, inverse (and the
// overlap-add of a fresh OLA object); results to pinned memory in one copy
// the overlap-add of a fresh OLA object (fresh_ola) after the chain's inverse
// frames, both ways its produces may come (after each push; after every push,
// the ring wrapped): into the result block (zero-copy: its host side)
hipError_t launch_spec_ola(BatchSpec* b, int dev, bool zc_out) {
    b->spec_y = b->spec_used = false;
    if (!fresh_ola(b->n, b->h, dev, b->s, &b->spec_ola)) return hipSuccess;
    const size_t N = size_t(b->n), M = size_t(b->M), row = N + 2, R = size_t(b->spec_ola.R);
    const size_t ylen = M * size_t(b->h) + size_t(std::max<int64_t>(0, b->n - b->h));
    if (M * row + M * N + ylen + R > b->c_blk || M * row + M * N + ylen + R > b->c_hblk) return hipSuccess;
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
    float* yout = zc_out ? b->m_blk + (M * row + M * N) : b->d_y;
    if ((e = launch_ola_gather_wrap(g, t, b->d_r, b->n, b->M, int64_t(ylen), b->d_acc, yout + ylen, b->s, yout)) ||
        (!zc_out && (e = hipMemcpyAsync(b->h_y, b->d_y, sizeof(float) * (ylen + R), hipMemcpyDeviceToHost, b->s))))
        return e;
    b->spec_y = true;
    return hipSuccess;
}

// frames 0 .. M-1 of the found chain: products, forward, inverse (and the
// overlap-add of a fresh OLA object), results to pinned memory; enqueued on
// b->s up to the event b->ev (run_chain waits for it)
int launch_chain(BatchSpec* b, crlot_plan* inner) {
    const size_t L = b->sig.size(), N = size_t(b->n), M = size_t(b->M), row = N + 2;
    const size_t ylen = M * size_t(b->h) + size_t(std::max<int64_t>(0, b->n - b->h));
    hipError_t e;
    if (!b->s && (e = hipStreamCreateWithFlags(&b->s, hipStreamNonBlocking)) != hipSuccess)
        return hip_fail(e, "batch stream");
    if (!b->ev && (e = hipEventCreateWithFlags(&b->ev, hipEventDisableTiming)) != hipSuccess)
        return hip_fail(e, "batch event");
    b->spec_y = b->spec_used = false;
    int dev = -1;
    if ((e = hipGetDevice(&dev))) return hip_fail(e, "batch device");
    // room for a fresh object's overlap-adds, whenever one comes (its ring: crlot_ring_len)
    const size_t R = size_t(crlot_ring_len(b->n, b->h)), blk = M * row + M * N + ylen + R;
    const size_t had = b->c_hblk;
    if ((e = dgrow(&b->d_p, &b->c_p, M * N)) || (e = dgrow(&b->d_blk, &b->c_blk, blk)) ||
        (e = hgrow(&b->h_blk, &b->c_hblk, blk)))
        return hip_fail(e, "batch buffers");
    if (b->c_hblk != had || !b->m_blk) {
        void* m = nullptr;
        b->m_blk = hipHostGetDevicePointer(&m, b->h_blk, 0) == hipSuccess ? static_cast<float*>(m) : nullptr;
    }
    b->d_spec = b->d_blk;
    b->d_r = b->d_spec + M * row;
    b->d_y = b->d_r + M * N;
    b->h_spec = b->h_blk;
    b->h_r = b->h_spec + M * row;
    b->h_y = b->h_r + M * N;
    // zero-copy (default): the kernels read the pinned rows and write the host
    // copies of their results themselves -- no copy engine, one dependent launch
    // fewer per copy
    const bool zc_out = zero_copy_out() && b->m_blk;
    CRLOT_LAP(1);
    const float* d_in = b->d_p;
    if (b->rows_src) {  // the FrameQueue's rows (already in h_stage) are the forward inputs
        if (zero_copy_in() && b->m_stage)
            d_in = b->m_stage;
        else if ((e = hipMemcpyAsync(b->d_p, b->h_stage, sizeof(float) * M * N, hipMemcpyHostToDevice, b->s)))
            return hip_fail(e, "batch frames");
    } else {
        b->m_stage = nullptr;  // (h_stage may move; the rows source maps it again)
        if ((e = dgrow(&b->d_sig, &b->c_sig, L + N)) || (e = hgrow(&b->h_stage, &b->c_hs, L + N)))
            return hip_fail(e, "batch buffers");
        std::memcpy(b->h_stage, b->sig.data(), sizeof(float) * L);
        std::memcpy(b->h_stage + L, b->win.data(), sizeof(float) * N);
        if ((e = hipMemcpyAsync(b->d_sig, b->h_stage, sizeof(float) * (L + N), hipMemcpyHostToDevice, b->s)) ||
            (e = launch_windowed_frames(b->d_sig, int64_t(L), b->d_sig + L, b->d_p, b->M, b->n, b->h, b->s)))
            return hip_fail(e, "batch frames");
    }
    CRLOT_LAP(2);
    // forward + inverse: one launch where the plan has the fused kernel
    bool spec_r_host = false;
    int rc = fuse_fft() ? plan_rfft_irfft(inner, d_in, zc_out ? b->m_blk : b->d_spec, b->d_r,
                                          zc_out ? b->m_blk + M * row : nullptr, int32_t(M), b->s)
                        : CRLOT_EUNSUPPORTED;
    if (rc == CRLOT_OK) {
        spec_r_host = zc_out;
    } else if (rc == CRLOT_EUNSUPPORTED) {
        rc = crlot_rfft_batched(inner, d_in, b->d_spec, int32_t(M), int64_t(N), 1, int64_t(row), 1, b->s);
        CRLOT_LAP(3);
        if (rc == CRLOT_OK)
            rc = crlot_irfft_batched(inner, b->d_spec, b->d_r, int32_t(M), int64_t(row), 1, int64_t(N), 1, b->s);
    }
    if (rc != CRLOT_OK) return rc;
    CRLOT_LAP(4);
    if (!spec_r_host &&
        (e = hipMemcpyAsync(b->h_blk, b->d_blk, sizeof(float) * (M * row + M * N), hipMemcpyDeviceToHost, b->s)))
        return hip_fail(e, "batch results");
    if ((e = launch_spec_ola(b, dev, zc_out))) return hip_fail(e, "batch overlap-add");
    CRLOT_LAP(5);
    if ((e = hipEventRecord(b->ev, b->s))) return hip_fail(e, "batch results");
    CRLOT_LAP(6);
    return CRLOT_OK;
}

int run_chain(BatchSpec* b, crlot_plan* inner) {
    const int rc = launch_chain(b, inner);
    if (rc != CRLOT_OK) return rc;
    const hipError_t e = hipEventSynchronize(b->ev);
    if (e != hipSuccess) return hip_fail(e, "batch results");
    CRLOT_LAP(7);
    return CRLOT_OK;
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
    if (j >= b->M || !input_matches(*b, j, in)) return 0;
    const size_t row = size_t(n) + 2;
    std::memcpy(out, b->h_spec + size_t(j) * row, sizeof(float) * row);
    b->next_fwd = j + 1;
    b->inv_ready = j;
    spec_count(kStatForward);
    if (b->next_fwd == b->M) b->active = false;  // last frame: its inverse / push / produce still served
    return 1;
}

int batch_forward(SharedServer* sh, crlot_plan* inner, int64_t n, const float* in, float* out) {
    if (spec_mode() < 2) return 0;
    if (!sh->batch) sh->batch = new BatchSpec();
    BatchSpec* b = sh->batch;
    const size_t row = size_t(n) + 2;
    if (batch_serve_forward(sh, n, in, out)) return 1;
    // a forward the batch did not predict: end it, then try to start one here
    if (b->active || b->ola) {
        const int rc = batch_abort(sh);
        if (rc != CRLOT_OK) return rc;
    }
    b->inv_ready = b->pushed = -1;
    CRLOT_LAP_START();
    if (!inner) return 0;
    // source 1: the Framer popped last, frame * a library window
    std::vector<float> sig;
    int64_t hop = 0, M = 0;
    const std::vector<float>* found = nullptr;
    std::vector<std::vector<float>> wins;
    if (framer_last_signal(n, &sig, &hop, &M) && M >= 4) {
        wins = windows_of_size(n);
        for (const auto& w : wins) {
            bool ok = true;
            for (int64_t i = 0; i < n && ok; ++i) {
                const float v = (i < int64_t(sig.size()) ? sig[size_t(i)] : 0.0f) * w[size_t(i)];
                ok = std::memcmp(&v, in + i, sizeof(float)) == 0;
            }
            if (ok) {
                found = &w;
                break;
            }
        }
    }
    // source 2: the FrameQueue read last, its frame as it is (no window),
    // copied straight into the pinned staging block the upload reads
    if (!found) {
        int qdev = -1, cur = -1;
        hipError_t he = hipSuccess;
        auto dst = [&](size_t floats) -> float* {
            const size_t had = b->c_hs;
            he = hgrow(&b->h_stage, &b->c_hs, floats);
            if (he != hipSuccess) return nullptr;
            if (b->c_hs != had || !b->m_stage) {
                void* m = nullptr;
                b->m_stage = hipHostGetDevicePointer(&m, b->h_stage, 0) == hipSuccess ? static_cast<float*>(m) : nullptr;
            }
            return b->h_stage;
        };
        const bool got = framequeue_last_rows(n, &hop, &M, &qdev, dst);
        if (he != hipSuccess) return hip_fail(he, "batch buffers");
        if (!got || M < 4 || hipGetDevice(&cur) != hipSuccess || cur != qdev ||
            std::memcmp(b->h_stage, in, sizeof(float) * size_t(n)) != 0)
            return 0;
    }
    b->gen += 1;
    b->n = n;
    b->h = hop;
    b->M = M;
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
    CRLOT_LAP(0);
    const int rc = run_chain(b, inner);
    if (rc != CRLOT_OK) {
        b->active = false;
        return rc;
    }
    sh->fft.valid = false;  // the call server's own per-call speculation is not used meanwhile
    sh->chain.valid = false;
    b->active = true;
    spec_count(kStatStart);
    spec_count(kStatForward);
    std::memcpy(out, b->h_spec, sizeof(float) * row);
    b->next_fwd = 1;
    b->inv_ready = 0;
    return 1;
}

int batch_inverse(SharedServer* sh, int64_t n, const float* in, float* out) {
    BatchSpec* b = sh->batch;
    if (!b || spec_mode() < 2 || b->n != n || b->inv_ready < 0) return 0;
    const int64_t j = b->inv_ready;
    const size_t row = size_t(n) + 2;
    if (std::memcmp(in, b->h_spec + size_t(j) * row, sizeof(float) * row) != 0) return 0;
    std::memcpy(out, b->h_r + size_t(j) * size_t(n), sizeof(float) * size_t(n));
    b->inv_ready = -1;
    b->pushed = j;
    spec_count(kStatInverse);
    return 1;
}

int batch_attach(SharedServer* sh, crlot_ola* o, int64_t j0, int64_t R, const float* d_ws, const float* d_den,
                 float gain, hipStream_t tables_stream, uint64_t tgen) {
    BatchSpec* b = sh->batch;
    if (b->spec_y && b->spec_ola.o == o && b->spec_ola.tgen == tgen && b->spec_ola.R == R && j0 == 0 &&
        std::memcmp(&gain, &kOne, sizeof(float)) == 0) {  // computed with the chain (run_chain)
        b->ola = o;
        b->j0 = 0;
        b->gain = gain;
        b->y_ready = b->y_waited = true;
        b->spec_used = true;
        b->ya = b->h_y + (size_t(b->M) * size_t(b->h) + size_t(std::max<int64_t>(0, b->n - b->h)));
        return CRLOT_OK;
    }
    b->spec_used = false;
    // blocks of frames j0 .. M-1 and the tail only they reach (no later frame
    // exists in the batch; a produce there needs the last frame pushed)
    const size_t F = size_t(b->M - j0), len = F * size_t(b->h) + size_t(std::max<int64_t>(0, b->n - b->h));
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
    if ((e = launch_ola_gather(g, t, b->d_r + size_t(j0) * size_t(b->n), b->n, b->d_y, 1, int64_t(F),
                               int64_t(len), int64_t(len), b->s)) ||
        (e = hipMemcpyAsync(b->h_y, b->d_y, sizeof(float) * len, hipMemcpyDeviceToHost, b->s)) ||
        (e = hipEventRecord(b->ev, b->s)))
        return hip_fail(e, "batch overlap-add");
    b->ola = o;
    b->j0 = j0;
    b->gain = gain;
    b->y_ready = true;
    b->y_waited = false;
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
    if ((e = launch_ola_gather_wrap(g, t, b->d_r + size_t(b->j0) * size_t(b->n), b->n, F, len, b->d_acc, b->d_ya,
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

extern "C" int crlot_set_call_speculation(int32_t mode) {
    if (mode < 1 || mode > 2) return crlot::set_error(CRLOT_EINVAL, "speculation mode is 1 or 2");
    crlot::g_mode.store(mode, std::memory_order_relaxed);
    return CRLOT_OK;
}
