// kernels.h -- host-side launch interface of the HIP kernels (internal).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "ab.h"
#include "crlot_dsp.h"

namespace crlot {

// Device-resident per-plan tables.
struct DevTables {
    const float* wa = nullptr;   // analysis window [N] (all ones if disabled)
    const float* ws = nullptr;   // synthesis window [N] (all ones if none)
    const float* den = nullptr;  // max(norm, eps) [ring_len]
    const float* tw = nullptr;   // per-pass Stockham twiddles (build_pass_twiddles)
    const float* st = nullptr;   // exp(-i pi (k/P + 1/2)), k < P, float pairs
    const float* gain = nullptr; // spectral gain [P+1] or nullptr
    // Exact-rewrite tables of the fused kernels (nullptr when the plan's tables
    // fall outside the ranges where the rewrites are bit-identical):
    const float* wsn = nullptr;  // ws * (1/N): folds the inverse's 1/N into the window
    const float* rden = nullptr; // RN(1 / den): Markstein division
    // {den, RN(1 / den)} pairs [ring_len] whenever every den lies in [2^-40, 2^40]
    // (Markstein's exact range), whatever the window rewrite says (K_pair15 keeps
    // the window and 1/N apart)
    const float* den_rden = nullptr;
    // Frame-pair transform tables (N = 1024 plans with pairing on, else nullptr):
    // W1024^{l k1} (15 x 64, fft_pair.h pair_t1_index) then W64^{b c} [c-1][b] (3 x 16), float pairs.
    const float* ptw = nullptr;
    // K_pair per-block divisors: [ring_len/H][64 lanes][den (SH) | rden (SH)], SH = H/64,
    // den at block offset lane + 64 q (nullptr when the pair kernel is off).
    const float* pden = nullptr;
    // ... and the same divisors by block pair: [ring_len/H][L lanes][(den_k, den_k+1) (SH pairs) |
    // (rden_k, rden_k+1) (SH pairs)] for every block k (k+1 modulo the ring), so the hot walkers
    // divide the blocks of a frame pair with packed operations (N = 512, 1024, 2048, 4096;
    // L = 64, 64, 128, 256).
    const float* pden2 = nullptr;
    // K_pair paired regime: samples x with x == 0 or px_lo <= |x| <= px_hi keep
    // sanitize(x * wa) == x * wa and the transforms finite (kernels.hip K_pair).
    float px_lo = 0.f, px_hi = 0.f;
    // K_pair4k (N = 4096) / K_pair2k (N = 2048): twiddles (fft_pair4k.h kP4Tw /
    // fft_pair2k.h kP2Tw float pairs) and divisors [ring_len/H][L lanes][den SH | rden SH],
    // L = 256 / 128, SH = H/L.
    const float* ptw4 = nullptr;
    const float* pden4 = nullptr;
    // K_pairN's pass twiddles for the spectral entries (pairn_spec.hip): ptw at its
    // sizes, a table of their own where ptw holds another transform's (1920 at even
    // hops: K_pair30's)
    const float* ptwn = nullptr;
    // K_pair (N = 1024): one flag per walker wave, written by the paired-only
    // walker (1 = a pair of its chunk left the paired regime) and read by the
    // fix-up walker that redoes those chunks; pflags_len flags of capacity.
    uint32_t* pflags = nullptr;
    int64_t pflags_len = 0;
    // 0: the paired-only hot walkers stay off and the two-regime walkers run every
    // chunk (crlot_plan_set_frame_pairing(plan, 2): parity diagnostics)
    int hot = 1;
};

// Launch knobs and the record of what one ABI call launched (crlot_plan_set_chunks,
// crlot_plan_last_launch).  The ABI installs a LaunchCtl on the calling thread for
// the duration of a call (LaunchScope in abi.cpp); the launch functions read the
// knobs from it and append every kernel they launch.  Kernel ids: CRLOT_K_* in
// include/crlot_dsp.h.
constexpr int kLaunchRecordMax = 8;
struct LaunchRecord {
    int32_t n = 0;                      // kernels launched (first kLaunchRecordMax kept)
    int32_t id[kLaunchRecordMax] = {};  // CRLOT_K_* in launch order
    int64_t grid[kLaunchRecordMax] = {};  // workgroups of each launch
    int32_t n_chunks = 0;               // chunks per stream of the walk (0: not a chunked walk)
};
struct LaunchCtl {
    int chunks = 0;  // chunks per stream forced on the chunked walkers (0: the chooser's)
    LaunchRecord rec;
};
LaunchCtl* launch_ctl();                  // the calling thread's, or nullptr
void set_launch_ctl(LaunchCtl* c);
void note_launch(int32_t id, int64_t grid);  // no-op without a LaunchCtl
void note_chunks(int64_t n_chunks);
// chunks per stream a walker over F frames uses given its chooser's dflt: the
// plan's knob clamped to [1, max_chunks] (max_chunks <= F), else dflt
int64_t chunks_or(int64_t dflt, int64_t max_chunks);

// Tables of the frame-pair transform (fft_pair.h) for N = 1024, float pairs.
std::vector<float> build_pair_twiddles();
// ... and of the 4096- and 512-point ones (fft_pair4k.h, fft_pair512.h).
std::vector<float> build_pair4k_twiddles();
std::vector<float> build_pair512_twiddles();
std::vector<float> build_pair2k_twiddles();  // fft_pair2k.h (N = 2048; stored in DevTables::ptw4)

// Per-pass Stockham twiddles for an N-point real frame (P = N/2 complex points),
// laid out as the device reads them (fft_wave.h twiddle_table_size), computed in
// double and rounded to float.  Returns float pairs.
std::vector<float> build_pass_twiddles(int n);

struct Geometry {
    int n = 0;          // frame size N
    int h = 0;          // hop H
    int ring_len = 0;   // OLA ring length
    float inv_n = 0.f;  // 1.0f / N (kissfft_adapter.cc:154)
    float gain = 1.f;   // push gain
    // framing source: frame k covers x[k*h - pad, k*h - pad + n); samples outside
    // [0, T) come from pad_mode (0 zeros, 1 reflect101, 2 edge; FrameQueue,
    // Indexing.h:18-70).  The Framer modes have pad = 0, pad_mode = 0.
    int pad = 0;
    int pad_mode = 0;
};

// Fused fast path: N in {256..2048}, H % 128 == 0, N % H == 0, ring_len % H == 0,
// 8-byte aligned streams.  Returns false if this shape has no instantiation.
bool fused_supported(int n, int h);
hipError_t launch_fused(const Geometry& g, const DevTables& t, const float* x, float* y,
                        int n_streams, int64_t T, int64_t ld_x, int64_t ld_y, int64_t F,
                        int64_t out_len, hipStream_t stream);
// K_pair on interleaved groups (crlot_roundtrip_interleaved's direct path);
// hipErrorNotSupported when the plan's kernel is not K_pair (N = 1024, zero padding)
hipError_t launch_pair_interleaved(const Geometry& g, const DevTables& t, const float* x, float* y, int n_groups,
                                   int channels, int64_t T, int64_t ld_x, int64_t ld_y, int64_t F,
                                   int64_t out_len, hipStream_t stream);

// Fused workgroup-walker path for frames too large for one wave: N = 4096
// (256 lanes per frame), H % 512 == 0, N % H == 0; same preconditions otherwise.
bool fused_wg_supported(int n, int h);
hipError_t launch_fused_wg(const Geometry& g, const DevTables& t, const float* x, float* y,
                           int n_streams, int64_t T, int64_t ld_x, int64_t ld_y, int64_t F,
                           int64_t out_len, hipStream_t stream);

// Staged general path.
bool synth_supported(int n);
hipError_t launch_synth_frames(const Geometry& g, const DevTables& t, const float* x,
                               int n_streams, int64_t T, int64_t ld_x, int64_t F, float* frames,
                               float* spec, hipStream_t stream);
hipError_t launch_ola_gather(const Geometry& g, const DevTables& t, const float* frames,
                             int64_t ld_frames, float* y, int n_streams, int64_t F,
                             int64_t ld_y, int64_t out_len, hipStream_t stream);
// the ring slots [0, ring_len) after F frames pushed from position 0 with no
// produce between (len = F h + max(0, n - h) positions; later positions wrap
// onto earlier slots): acc = the slots, y = acc / den (k_ola_gather_wrap);
// y_blocks (nullable): launch_ola_gather's produce blocks [len] too, same launch
hipError_t launch_ola_gather_wrap(const Geometry& g, const DevTables& t, const float* frames, int64_t ld_frames,
                                  int64_t F, int64_t len, float* acc, float* y, hipStream_t stream,
                                  float* y_blocks = nullptr);
// K_rfft then K_irfft of `batch` contiguous rows (power-of-two n, 256..2048) in
// one launch (k_rfft_irfft): spectra [batch][ld_spec], inverse frames into r
// (and r_host when not null), rows ld_r apart
hipError_t launch_rfft_irfft(const Geometry& g, const DevTables& t, const float* in, int64_t ld_in, float* spec,
                             int64_t ld_spec, float* r, float* r_host, int64_t ld_r, int batch, hipStream_t stream);

// Any-size path (fft_any.h): any P = N/2 in 1..8192.  twany = build_any_twiddles(P)
// on device.  kind: 0 rfft, 1 irfft, 2 cfft, 3 icfft; p = complex points of the
// transform (N/2 for the real kinds, nfft for the complex ones); inv_scale = 1/nfft.
bool any_supported(int p);
std::vector<float> build_any_twiddles(int p);
std::vector<uint8_t> build_any_plan_blob(int p);  // dev::any::Plan bytes (fft_any.h)
hipError_t launch_synth_any(const Geometry& g, const DevTables& t, const float* twany,
                            const float* x, int n_streams, int64_t T, int64_t ld_x, int64_t F,
                            float* frames, float* spec, hipStream_t stream);
// Any-shape streaming hop (DROP Framer, one wave per channel).  hist: [C][hl],
// acc: [C][rl] floats (zeroed at creation); k = frame completed by hop q or -1.
int stream_any_hist_len(int n, int h);
int stream_any_ring_len(int n, int h);
hipError_t launch_stream_any(const Geometry& g, const DevTables& t, const float* twany,
                             const float* in, int64_t in_ld, int64_t in_inc, float* out,
                             int64_t out_ld, int64_t out_inc, float* hist, float* acc, int channels,
                             int64_t q, int64_t k, hipStream_t stream);

// Fused any-size walker (OLA ring in LDS): bit-identical to synth_any + ola_gather.
// mask (optional): per-walker flags of a K_pair15 launch, [stream / mask_div][mask_chunks],
// bit (stream % mask_div) for the stream; only streams with a flagged walker are walked.
bool fused_any_fits(int n, int h);
hipError_t launch_fused_any(const Geometry& g, const DevTables& t, const float* twany,
                            const float* x, float* y, int n_streams, int64_t T, int64_t ld_x,
                            int64_t ld_y, int64_t F, hipStream_t stream,
                            const uint32_t* mask = nullptr, int mask_chunks = 0, int mask_div = 1);

// K_pair15 (pair_any.hip): N = 960 / 480 frame pairs, paired regime only; flags
// per walker in t.pflags ([stream / *streams_per_walk][*n_chunks]); table t.ptw =
// build_pair15_twiddles(N).
bool pair15_supported(int n, int h, int ring_len);
hipError_t launch_pair15(const Geometry& g, const DevTables& t, const float* x, float* y, int n_streams,
                         int64_t T, int64_t ld_x, int64_t ld_y, int64_t F, int64_t out_len, int* n_chunks,
                         int* streams_per_walk, hipStream_t stream);
std::vector<float> build_pair15_twiddles(int n);
// K_pairN (pair_n.hip): frame pairs for N in {320, 400, 640, 882, 1000, 1764}
// (fft_pairn.h), paired regime only; flags per walker in t.pflags like K_pair15,
// n_chunks walkers per stream.  Tables: t.ptw = build_pairn_twiddles(N).
bool pairn_size(int n);
bool pairn_over_pair15(int n);
bool pairn_supported(int n, int h, int ring_len);
hipError_t launch_pairn(const Geometry& g, const DevTables& t, const float* x, float* y, int n_streams, int64_t T,
                        int64_t ld_x, int64_t ld_y, int64_t F, int64_t out_len, int* n_chunks, hipStream_t stream);
std::vector<float> build_pairn_twiddles(int n);
// K_pair30 (pair30.hip): N = 1920 frame pairs as two 960-point transforms on two
// waves, even hops; flags per walk as launch_pairn.  Tables: t.ptw = build_pair30_twiddles().
bool pair30_supported(int n, int h, int ring_len);
hipError_t launch_pair30(const Geometry& g, const DevTables& t, const float* x, float* y, int n_streams, int64_t T,
                         int64_t ld_x, int64_t ld_y, int64_t F, int64_t out_len, int* n_chunks, hipStream_t stream);
std::vector<float> build_pair30_twiddles();
hipError_t launch_fft_any(int kind, int p, float inv_scale, const DevTables& t, const float* twany,
                          const float* in, float* out, int batch, int64_t ld_in, int64_t inc_in,
                          int64_t ld_out, int64_t inc_out, hipStream_t stream);

// Streaming per-hop path (shapes as the fused path).  hist/acc: [channels][N].
hipError_t launch_stream_hop(const Geometry& g, const DevTables& t, const float* in, int64_t in_ld,
                             int64_t in_inc, float* out, int64_t out_ld, int64_t out_inc,
                             float* hist, float* acc, int channels, int64_t q, hipStream_t stream);

// Resident streaming kernel (stream_rt.hip, BASELINE config 4).  The control
// block and the hop rings live in pinned host memory; the host writes hop q
// into in_ring slot q % depth, then seq = q + 1; workgroup w publishes
// done[w] = q + 1 once its channels' output block is in out_ring slot q % depth.
constexpr int kRtMaxChannels = 1024;
constexpr int kRtMaxWg = kRtMaxChannels / 4;
struct alignas(64) RtCtl {
    uint64_t seq;             // hops submitted (host, release)
    uint64_t stop;            // nonzero: every workgroup exits at its next poll (host: 1 =
                              // stop; device: 2 = a workgroup's idle timer expired)
    uint64_t pad0[6];
    uint64_t done[kRtMaxWg];  // hops completed per workgroup (device, release)
    uint64_t ticks[kRtMaxWg]; // s_memrealtime ticks (100 MHz) of the last hop per workgroup
    uint64_t phase[8];        // CRLOT_RT_PHASES diagnostic builds: workgroup 0's phase stamps
};
struct RtArgs {
    DevTables t;
    RtCtl* ctl;
    const float* in_ring;     // [depth][C * H] host-pinned
    float* out_ring;          // [depth][C * H] host-pinned
    float* state;             // [C][2N] device: hist | acc, saved at exit, restored at launch
    int channels = 0, interleaved = 0, depth = 0, ring_len = 0;
    float inv_n = 0.f, gain = 1.f;
    uint64_t idle_ticks = 0;  // exit after this long without a hop
};
int stream_rt_workgroups(int channels);
hipError_t launch_stream_rt(const Geometry& g, const RtArgs& a, hipStream_t stream);

// Batched adapter-semantics real FFTs.
hipError_t launch_rfft(const Geometry& g, const DevTables& t, const float* in, float* out,
                       int batch, int64_t ld_in, int64_t inc_in, int64_t ld_out,
                       int64_t inc_out, hipStream_t stream);
hipError_t launch_irfft(const Geometry& g, const DevTables& t, const float* in, float* out,
                        int batch, int64_t ld_in, int64_t inc_in, int64_t ld_out,
                        int64_t inc_out, hipStream_t stream);
// Batched complex FFT of P = g.n / 2 points (forward: raw DFT; inverse: *1/P, sanitize).
hipError_t launch_cfft(const Geometry& g, const DevTables& t, const float* in, float* out, int batch,
                       int64_t ld_in, int64_t inc_in, int64_t ld_out, int64_t inc_out, bool inverse,
                       hipStream_t stream);

// OLAAccumulator object (ola.hip): ring [C][R], den [R].  add: source element
// (c, j) at src[c*cs + j*js], window win[j] or nullptr, ring position
// (start + j) mod R for j < len <= R.  produce: out[c*ldo + j] = ring / den at
// (rp + j) mod R, j < len, ring cleared; peak (nullable) = running max |out|
// over channel 0's first n_total samples, as float bits.
// PCM layout: groups of T rows x C interleaved samples <-> channel planes [g][c][T].
hipError_t launch_deinterleave(const float* x, int64_t ld_x, float* planes, int groups, int64_t T, int C,
                               hipStream_t s);
hipError_t launch_interleave(const float* planes, int64_t L, float* y, int64_t ld_y, int groups, int C,
                             hipStream_t s);
hipError_t launch_ola_add(float* ring, int channels, int64_t R, const float* src, int64_t cs,
                          int64_t js, const float* win, int64_t start, int64_t len, float gain,
                          hipStream_t s);
hipError_t launch_ola_produce(float* ring, int channels, int64_t R, const float* den, float* out,
                              int64_t ldo, int64_t rp, int64_t len, int64_t n_total, unsigned* peak,
                              hipStream_t s);

// Resident call server (call_rt.hip, host side call.cpp): the reference's
// host-pointer calls as request descriptors.  Ops and flags:
enum : uint32_t {
    kCallRfft = 1, kCallIrfft, kCallCfft, kCallIcfft,  // IFftPlan forward / inverse / _complex
    kCallOlaAdd, kCallOlaProduce,                      // OLAAccumulator add_frame_SoA|push_frame_AoS / produce
    kCallAxpy, kCallAxpyWin, kCallNormalize            // dsp::axpy / axpy_windowed / normalize_and_clear
};  // op 0: nothing but the request's deferred ring work (CallPend)
// kCallChain (on a speculating forward): also keep the speculated inverse frame
// and compute the produce block the target OLA object would give after pushing it
// kCallPendLate (on a chained single-frame request whose deferred commit pushes
// into the chain's own ring, its clear disjoint from the produce block): the
// produce block adds that commit's frame itself, and the deferred ring work runs
// after chain_done, published as ring_done
enum : uint32_t { kCallSpec = 1, kCallClearOnly = 2, kCallAcquire = 4, kCallChain = 8, kCallPendLate = 16 };
struct alignas(512) CallReq {
    uint32_t op, flags;
    int32_t batch, channels;
    int64_t in_off, out_off, spec_off, win_off;  // floats into in_arena (device) / out_arena (host); win_off < 0: none
    const float* p0;  // FFT: pass twiddles   | OLA add: the object's window (nullable)
    const float* p1;  // FFT: super twiddles  | OLA: den = max(norm, eps)
    float* p2;        // OLA (and chain): ring [C][R]
    int64_t i[6];     // OLA: R, ring start / read pos, len, AoS?, speculated read pos, speculated count
    float f0, f1;     // FFT: 1/N (1/P complex) | OLA add: gain | axpy: g | normalize: eps; f1: chain gain
    const float* p3;  // chain: den
    const float* p4;  // chain: the object's window (nullable)
    int64_t j[8];     // chain: R, push start (ring pos), produce read pos, produce count
    const void* p5;   // FFT of any size (K_call<-1>): the pass plan (dev::any::Plan, device)
    uint64_t pad[5];
    // Ring work the host deferred onto this request, applied before it (in this
    // order): the push of the frame the last chained forward kept (kPendCommit),
    // then the clear of a produce block served from a speculation (kPendClear).
    struct Pend {
        uint32_t flags;
        float gain;
        float* ring;
        const float* win;   // commit: the object's window or null
        int64_t R, start, len;  // commit: ring position and length
        int64_t rp, n;          // clear: ring position and length (mono)
        // commit: the chained forward that kept the frame (1-based request
        // number) and the frame's copy in out_arena (its speculated inverse,
        // floats from out_arena): a kernel launched after that forward has lost
        // the LDS copy and reads this one
        uint64_t src_index;
        int64_t src_off;
    } pend;
    uint64_t pad2[22];
};
enum : uint32_t { kPendCommit = 1, kPendClear = 2 };
static_assert(sizeof(CallReq) == 512, "one descriptor = 64 lanes x 8 bytes");
struct alignas(64) CallCtl {  // fine-grained device memory, written by the host (BAR)
    uint64_t seq;             // requests submitted
    uint64_t pad0[7];
    uint64_t stop;            // host: 1 = stop; kernel: 2 = idle exit
    uint64_t pad1[7];
};
struct alignas(64) CallHostCtl {  // pinned host memory, written by the kernel
    uint64_t done;                // requests completed
    uint64_t pad0[7];
    uint64_t spec_done;           // requests whose speculation slot is written
    uint64_t pad1[7];
    uint64_t chain_done;          // forwards whose chained produce block is written
    uint64_t pad2[7];
    uint64_t ring_done;           // requests whose late deferred ring work (kCallPendLate) is done
    uint64_t pad3[7];
    uint64_t ph[8];               // -DCRLOT_CALL_PHASES builds: the last request's phase stamps
};
struct CallArgs {
    CallCtl* ctl = nullptr;
    CallHostCtl* hctl = nullptr;
    const CallReq* reqs = nullptr;  // [depth], fine-grained device memory
    const float* in_arena = nullptr;
    float* out_arena = nullptr;     // pinned host memory
    int depth = 0;
    int64_t in_cap = 0;             // floats per input slot (slot q % depth at q * in_cap)
    uint64_t first = 0;             // requests completed before this launch
    uint64_t idle_ticks = 0;
    int any_p = 0, any_waves = 0, any_tw = 0;  // e < 0: complex points, FFT waves, twiddles (launch_call)
    int any_two = 0;                           // e < 0: two chained frames in LDS (call_any_two)
};
// e = 0 (OLA / kernel ops only), the FFT's E = P / 64 in {2, 4, 8, 16, 32}, or
// -P for any other complex size P (fft_any.h; call_any_waves(P) > 0)
size_t call_lds_bytes(int e);
int call_any_waves(int p);
bool call_any_two(int p);
hipError_t launch_call(int e, const CallArgs& a, hipStream_t s);

// dsp::axpy / axpy_windowed (win != nullptr) / normalize_and_clear over `batch`
// rows of n elements (ola.hip); the window / norm row is shared by every row.
hipError_t launch_axpy(float* dst, int64_t ld_dst, const float* src, int64_t ld_src, const float* win, float g,
                       int64_t n, int64_t batch, hipStream_t s);
hipError_t launch_normalize_and_clear(float* out, int64_t ld_out, float* acc, int64_t ld_acc, const float* norm,
                                      float eps, int64_t n, int64_t batch, hipStream_t s);
// p[k][j] = x[k H + j] * w[j] (0 * w[j] past T), k < F: the host loop's analysis
// products for the batched drop-in speculation (batch.cpp)
hipError_t launch_windowed_frames(const float* x, int64_t T, const float* w, float* p, int64_t F, int64_t N,
                                  int64_t H, hipStream_t s);
// out[k][2b + c] = spec[k][2b + c] * g[b] (k < rows, b < bins, rows ld floats apart):
// a caller's per-bin real spectral gain (batch.cpp), one plain multiply
hipError_t launch_bin_gain(const float* spec, float* out, const float* g, int64_t rows, int64_t ld, int64_t bins,
                           hipStream_t s);
// ---- stft.hip: the round trip split at the spectral step (crlot_stft / crlot_istft_ola)
// Per-frame real mask rows: row (stream s, frame k) at p + s ld_stream + k ld_frame,
// N/2+1 floats (ld_stream 0: one row per frame for every stream).
struct SpecMask {
    const float* p = nullptr;
    int64_t ld_frame = 0, ld_stream = 0;
};
// K_stft: power-of-two N 256..4096, any hop and framing; spectra (s, k) at
// spec + s ld_spec + k ld_frame, N/2+1 float pairs (8-byte aligned rows)
bool stft_supported(int n);
hipError_t launch_stft(const Geometry& g, const DevTables& t, const float* x, int n_streams, int64_t T,
                       int64_t ld_x, int64_t F, float* spec, int64_t ld_spec, int64_t ld_frame, hipStream_t s);
// K_istft walker shapes: stft_supported(n), H % 128 == 0, N % H == 0; also needs the
// exact-rewrite tables (t.wsn, t.rden), ring_len % H == 0 and 8-byte aligned y rows
bool istft_walk_supported(int n, int h);
hipError_t launch_istft(const Geometry& g, const DevTables& t, const SpecMask& m, const float* spec,
                        int64_t ld_spec, int64_t ld_frame, float* y, int n_streams, int64_t F, int64_t ld_y,
                        hipStream_t s);
// The round trip with the spectral step (gain, mask) on K_istft's walk from x
// (8-byte aligned x rows as well): bit-identical to launch_istft(launch_stft(x))
hipError_t launch_roundtrip_masked(const Geometry& g, const DevTables& t, const SpecMask& m, const float* x,
                                   float* y, int n_streams, int64_t T, int64_t ld_x, int64_t ld_y, int64_t F,
                                   hipStream_t s);
// ... as frame pairs (K_pair_mask, pair_mask.hip: N = 1024, H = 128 / 256 / 512, the
// pair tables; equal to the per-frame walk within float32 rounding)
bool pair_mask_supported(int n, int h);
bool pair_spec_supported(int n, int h);  // K_pair_stft / K_pair_istft: N = 1024 (H 128-512), 512 (H 128, 256),
                                         // 2048 (H 256, 512), 4096 (H 512, 1024)
bool pair_tables(const Geometry& g, const DevTables& t);  // the tables those kernels read are there
// ... and at N = 960 / 480 (K_pair15's transforms, any hop >= 32 with ring_len % H == 0; pair15_spec.hip)
bool pair15_spec_supported(int n, int h, int ring_len);
bool pair15_spec_fits(int n, int64_t ld, int64_t len);  // the walks' 32-bit buffer offsets cover (ld, len)
// ... and at K_pairN's one-wave sizes 882, 1000, 640, 400, 320 (pairn_spec.hip)
bool pairn_spec_supported(int n, int h, int ring_len);
hipError_t launch_pairn_stft(const Geometry& g, const DevTables& t, const float* x, int n_streams, int64_t T,
                             int64_t ld_x, int64_t F, float* spec, int64_t ld_spec, int64_t ld_frame,
                             hipStream_t stream);
hipError_t launch_pairn_istft(const Geometry& g, const DevTables& t, const SpecMask& m, const float* spec,
                              int64_t ld_spec, int64_t ld_frame, float* y, int n_streams, int64_t F, int64_t ld_y,
                              hipStream_t stream);
hipError_t launch_pairn_masked(const Geometry& g, const DevTables& t, const SpecMask& m, const float* x, float* y,
                               int n_streams, int64_t T, int64_t ld_x, int64_t ld_y, int64_t F, int64_t out_len,
                               hipStream_t stream);
hipError_t launch_pair15_stft(const Geometry& g, const DevTables& t, const float* x, int n_streams, int64_t T,
                              int64_t ld_x, int64_t F, float* spec, int64_t ld_spec, int64_t ld_frame,
                              hipStream_t stream);
hipError_t launch_pair15_istft(const Geometry& g, const DevTables& t, const SpecMask& m, const float* spec,
                               int64_t ld_spec, int64_t ld_frame, float* y, int n_streams, int64_t F, int64_t ld_y,
                               hipStream_t stream);
hipError_t launch_pair15_masked(const Geometry& g, const DevTables& t, const SpecMask& m, const float* x, float* y,
                                int n_streams, int64_t T, int64_t ld_x, int64_t ld_y, int64_t F, int64_t out_len,
                                hipStream_t stream);
// crlot_stft / crlot_istft_ola as frame pairs (K_pair_stft / K_pair_istft, pair_stft.hip:
// N = 1024, H = 128 / 256 / 512, the pair tables; within float32 rounding of the per-frame kernels)
hipError_t launch_pair_stft(const Geometry& g, const DevTables& t, const float* x, int n_streams, int64_t T,
                            int64_t ld_x, int64_t F, float* spec, int64_t ld_spec, int64_t ld_frame, hipStream_t s);
hipError_t launch_pair_istft(const Geometry& g, const DevTables& t, const SpecMask& m, const float* spec,
                             int64_t ld_spec, int64_t ld_frame, float* y, int n_streams, int64_t F, int64_t ld_y,
                             hipStream_t s);
hipError_t launch_pair_masked(const Geometry& g, const DevTables& t, const SpecMask& m, const float* x, float* y,
                              int n_streams, int64_t T, int64_t ld_x, int64_t ld_y, int64_t F, int64_t out_len,
                              hipStream_t s);
// staged forms: frames[s F + k][N] = x frame * analysis window; out rows (s F + k) of
// 2 bins floats = spectrum * gain * mask (in place when out aliases the same layout)
hipError_t launch_frames_windowed(const Geometry& g, const DevTables& t, const float* x, int n_streams, int64_t T,
                                  int64_t ld_x, int64_t F, float* frames, hipStream_t s);
hipError_t launch_spec_step(const DevTables& t, const SpecMask& m, const float* spec, int64_t ld_spec,
                            int64_t ld_frame, float* out, int n_streams, int64_t F, int bins, hipStream_t s);

// dsp::FrameQueue frames on the device: [stream][F][N] from x [stream][ld_x]
hipError_t launch_fq_frames(const float* x, int64_t T, int64_t ld_x, int n_streams, float* frames, int64_t F,
                            int64_t N, int64_t H, int64_t pad, int pad_mode, hipStream_t s);

}  // namespace crlot
