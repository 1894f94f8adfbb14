/*
 * crlot_dsp.h -- C ABI of the MI355X (gfx950) batched STFT -> iSTFT -> OLA engine.
 *
 * Replaces, for the hot path, the reference's host objects (file:line in
 * /root/reference):
 *   dsp::Framer                  dsp/frame/framer.h:26-127, framer.cc:15-181
 *   dsp::WindowLUT               dsp/window/WindowLUT.h:80-287, WindowLUT.cc:215-388
 *   dsp::fft::IFftPlan           dsp/fft/api/fft_api.h:16-51,
 *                                dsp/fft/backends/kissfft_adapter.cc:11-269
 *   dsp::OLAAccumulator          dsp/ola/OLAAccumulator.h:15-217, OLAAccumulator.cc:13-295
 *   dsp::ola::build_norm_linear  dsp/ola/norm_builder.cc:8-52
 *   axpy_windowed / normalize_and_clear   dsp/ola/kernels.cc:18-52
 * and the round trip the harness assembles from them
 * (bench/e2e_benchmark.cc:138-186, streaming-interleaved order: push frame k,
 * then produce(H)).
 *
 * Conventions: plain C types only.  Device pointers (d_*) are caller-owned HIP
 * device memory; host pointers are plain host memory.  `stream` is a hipStream_t
 * passed as void* (NULL = default stream).  Every entry returns 0 on success or
 * a negative CRLOT_E* code; crlot_last_error() gives the message of the last
 * failure on the calling thread.  Nothing throws across this boundary.
 * Streams and threads: a plan may serve several HIP streams at once.  Its
 * launch scratch (K_pair's regime flags, the staged path's frame workspace, the
 * interleaved path's channel planes) is kept per stream handle, so round trips
 * issued on different streams never share device scratch, and growth is
 * stream-ordered (hipMallocAsync / hipFreeAsync on the calling stream: no
 * device-wide synchronisation).  Host-side entry points take the plan's lock,
 * so several host threads may also share a plan (the reference's KissFftPlan
 * is non-reentrant: kissfft_adapter.cc:256-263).  Streaming objects
 * (crlot_stream*, crlot_stream_rt*, crlot_ola*) are single-owner objects.
 */
#ifndef CRLOT_DSP_H_
#define CRLOT_DSP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CRLOT_ABI_VERSION 2

/* error codes */
#define CRLOT_OK 0
#define CRLOT_EINVAL (-1)       /* bad argument (reference: std::invalid_argument) */
#define CRLOT_EUNSUPPORTED (-2) /* valid for the reference, not on this device path */
#define CRLOT_EHIP (-3)         /* HIP runtime error */
#define CRLOT_ENOMEM (-4)       /* allocation failed (reference: std::bad_alloc) */
#define CRLOT_ERUNTIME (-5)     /* reference: std::runtime_error */
#define CRLOT_ERANGE (-6)       /* reference: std::out_of_range */

/* dsp::WindowType (WindowLUT.h:14-20) */
#define CRLOT_WIN_HANN 0
#define CRLOT_WIN_HAMMING 1
#define CRLOT_WIN_BLACKMAN 2
#define CRLOT_WIN_RECT 3
#define CRLOT_WIN_BLACKMAN_HARRIS 4 /* rejected, as in WindowLUT.cc:241-242 */
/* dsp::NormalizationType (WindowLUT.h:25-31) */
#define CRLOT_NORM_NONE 0
#define CRLOT_NORM_SUM_TO_ONE 1
#define CRLOT_NORM_L2 2
#define CRLOT_NORM_OLA_UNITY_GAIN 3
#define CRLOT_NORM_OLA_SUM_WSQ 4
/* framing source: dsp::BoundaryMode (framer.h:11-14) of a whole-stream Framer
 * push, or dsp::FrameQueue (FrameQueue.h:26-96) with center / pad_mode */
#define CRLOT_ZERO_PAD 0
#define CRLOT_DROP 1
#define CRLOT_FRAMEQUEUE 2
/* dsp::PadMode (FrameQueue.h:8-12) */
#define CRLOT_PAD_CONSTANT 0
#define CRLOT_PAD_REFLECT 1
#define CRLOT_PAD_EDGE 2

typedef struct crlot_plan crlot_plan;
typedef struct crlot_stream crlot_stream;

/* Plan description: the union of OLAConfig (OLAAccumulator.h:15-29), the
 * Framer parameters (framer.h:46-47) and the window choice of the harness
 * (e2e_benchmark.cc:48-64).  Zero-initialise, then set the fields. */
typedef struct crlot_plan_desc {
    int32_t frame_size;          /* N: even, <= 16384 (powers of two 256..4096 run the
                                    register-resident kernels, other sizes the mixed-radix path) */
    int32_t hop_size;            /* H: 1..N */
    int32_t window_type;         /* CRLOT_WIN_* */
    int32_t periodic;            /* 0 = symmetric (reference default) */
    int32_t window_norm;         /* CRLOT_NORM_* */
    int32_t boundary_mode;       /* CRLOT_ZERO_PAD / CRLOT_DROP (Framer) or CRLOT_FRAMEQUEUE */
    int32_t analysis_window;     /* 1: frame * w before forward (e2e_benchmark.cc:154-156) */
    int32_t apply_window_inside; /* OLAConfig::apply_window_inside */
    float eps;                   /* OLAConfig::eps; 0 -> 1e-8f */
    float ola_gain;              /* push_frame_AoS gain; 0 -> 1.0f */
    int32_t ring_len;            /* 0 -> (ceil(N/H)+20)*H (OLAAccumulator.cc:249-258) */
    int32_t device;              /* HIP device ordinal, -1 = current */
    int32_t center;              /* CRLOT_FRAMEQUEUE: pad N/2 both sides (FrameQueue default: 1) */
    int32_t pad_mode;            /* CRLOT_FRAMEQUEUE: CRLOT_PAD_* */
} crlot_plan_desc;

const char* crlot_last_error(void);
int crlot_abi_version(void);
/* What this binary was built from: "src:<hash> arch:gfx950", the hash being
 * tools/src_hash.py's lib_hash() of the library's sources at build time (a
 * prebuilt library older than the tree it ships in shows a different hash). */
const char* crlot_build_info(void);

/* ---------------------------------------------------------------- plan */
int crlot_plan_create(const crlot_plan_desc* desc, crlot_plan** out);
void crlot_plan_destroy(crlot_plan* plan);
/* Replace the plan's window (N floats) and/or COLA norm table (ring_len floats)
 * with host-built ones (NULL keeps the plan's own, which are built on the host
 * by the reference formulas, bit-exact). */
int crlot_plan_upload_tables(crlot_plan* plan, const float* window, const float* norm);
/* Spectral hook between rfft and irfft: real per-bin gain, N/2+1 host floats;
 * NULL restores the identity step of the reference (e2e_benchmark.cc:161-162). */
int crlot_plan_set_spectral_gain(crlot_plan* plan, const float* gain);
/* Stream-ordered forms of the two table updates: the host data is staged in
 * pinned memory and copied with hipMemcpyAsync on `stream`, so work enqueued on
 * `stream` before the call sees the old tables and work after it the new ones
 * (the host arrays may be reused as soon as the call returns).  The stream-less
 * entries above first drain the device (hipDeviceSynchronize), so a round trip
 * in flight on any stream never reads a half-updated table. */
int crlot_plan_upload_tables_async(crlot_plan* plan, const float* window, const float* norm,
                                   void* stream);
int crlot_plan_set_spectral_gain_async(crlot_plan* plan, const float* gain, void* stream);
/* Frame pairing on the fused round trip (default on): two consecutive frames
 * (2j, 2j+1) of a stream share one complex FFT, z = frame_2j + i frame_2j+1,
 * whose real and imaginary round-trip outputs are the two frames' (exact for
 * the real, bin-symmetric spectral gain).  Used where those kernels exist
 * (N = 512, 1024, 2048, 4096 with the fused hop rules); a pair holding a NaN, Inf,
 * huge or tiny sample is transformed frame by frame instead, so no frame's
 * overflow reaches its neighbour.  Results equal the per-frame kissfft
 * formulation within float32 rounding, not bit for bit, and do not depend on
 * the batch or the chunking.  0 selects the per-frame (kiss_fftr split)
 * kernels, bit-identical to crlot_roundtrip_stages + crlot_ola_gather.  2 keeps
 * pairing but runs the power-of-two pair kernels' two-regime walkers on every
 * chunk (their paired-only hot walkers off): bit-identical to 1, for parity
 * diagnostics.  Other values: CRLOT_EINVAL. */
int crlot_plan_set_frame_pairing(crlot_plan* plan, int32_t enable);
/* Chunks per stream the chunked walkers of crlot_roundtrip /
 * crlot_roundtrip_interleaved split every stream into (every frame-pair walker
 * and the per-frame fused walkers).  0 (default) lets the library choose (whole
 * resident rounds of the device); n > 0 forces min(n, F) chunks (min(n, F/2) on
 * the two-wave K_pairN walks).  Output bits never depend on it (each chunk
 * recomputes its warm-up frames); it exists so parity tests can move the chunk
 * seams, and the launch record below reports the chunking a call used.
 * Negative: CRLOT_EINVAL. */
int crlot_plan_set_chunks(crlot_plan* plan, int32_t chunks_per_stream);
/* Speculation of the host-pointer drop-in calls (IFftPlan forward / inverse,
 * OLAAccumulator push / produce), process-wide.  1: each forward also computes
 * the inverse and the produce block that follow it on the call kernel.  2
 * (default): in addition, when a forward's input is bit for bit the frame a
 * dsp::Framer just popped times a window table the library built (or the
 * dsp::FrameQueue frame read last), the loop over that signal runs as batches
 * on the device, windows of at most `window_frames` frames
 * (crlot_call_batch_capacity), and the following calls are served from them
 * after a bitwise check of each call's input and arguments; an inverse input
 * that is the served spectrum times a fixed real gain per bin teaches the batch
 * that gain.  The first call that differs otherwise ends the batch and the OLA
 * object's ring is rebuilt from the frames it was served; a batch that cannot
 * allocate or launch declines and the call takes its ordinary path.  Results
 * are the same bits in both modes.  Other values: CRLOT_EINVAL. */
int crlot_set_call_speculation(int32_t mode);
/* Process-wide counters of the batched speculation: [0] batches started, [1]
 * forwards, [2] inverses, [3] pushes, [4] produces served from a batch, [5] OLA
 * rings rebuilt after a call the batch did not predict. */
int crlot_call_speculation_stats(int64_t* out6);
/* The same counters and more, out[0 .. count): [0..5] as above, [6] frames the
 * batches transformed, [7] window continuations (a batch is bounded: at most
 * `window_frames` frames per chain, below; the next window starts at the
 * forward of the first frame past it), [8] speculations declined because a
 * buffer or launch failed (the call then took the ordinary path), [9] spectral
 * gains learned (an inverse input that was the served spectrum times a fixed
 * real gain per bin, bit for bit: the batch's remaining inverses are then those
 * of the gained spectra, each still served only after a bitwise check), [10]
 * learned gains not applied because the previous one served fewer than four
 * inverses and differed in more than an eighth of the bins (a time-varying
 * edit: those frames take the per-call path, learning backs off for 16, 32, ..
 * frames); entries past the known ones are 0.  Negative: CRLOT_EINVAL. */
int crlot_call_speculation_stats_ex(int64_t* out, int32_t count);
/* Bounds of the batched speculation: frames per window, and the device and
 * pinned host bytes the batches hold now, with the pinned peak since load. */
int crlot_call_batch_capacity(int64_t* window_frames, int64_t* device_bytes, int64_t* pinned_bytes,
                              int64_t* pinned_peak);
/* Test-only fault injection: CRLOT_INJECT_BATCH_ALLOC makes the next `count`
 * buffer allocations of the batched speculation fail (a speculation that cannot
 * allocate declines and the call takes its ordinary path);
 * CRLOT_INJECT_CALL_TIMEOUT makes the next `count` waits on the resident call
 * kernel take their timeout path (the call fails with CRLOT_EHIP; the server
 * serves again once every request submitted before completed).  Other `what`:
 * CRLOT_EINVAL. */
#define CRLOT_INJECT_BATCH_ALLOC 1
#define CRLOT_INJECT_CALL_TIMEOUT 2
int crlot_test_inject(int32_t what, int32_t count);
/* What the plan's last call on `stream` launched: kernels in launch order
 * (CRLOT_K_* ids below; the first 8 are kept, n_kernels counts all), the
 * workgroups of each launch, and the chunks per stream of the walk (0 when the
 * call ran no chunked walker).  Recorded by crlot_roundtrip,
 * crlot_roundtrip_interleaved, crlot_roundtrip_stages, crlot_ola_gather and
 * the batched FFTs; a call that failed records what it launched before failing.
 * No call on `stream` yet: n_kernels = 0. */
#define CRLOT_K_PAIR_HOT 1       /* K_pair paired-only walker, N = 1024 */
#define CRLOT_K_PAIR_FIX 2       /* K_pair two-regime walker: the flagged chunks after the hot walker */
#define CRLOT_K_PAIR_ALL 3       /* K_pair two-regime walker over every chunk */
#define CRLOT_K_PAIR512_HOT 4
#define CRLOT_K_PAIR512 5        /* two-regime walker, N = 512 (flagged chunks or all, see fix_all) */
#define CRLOT_K_PAIR2K_HOT 6
#define CRLOT_K_PAIR2K 7
#define CRLOT_K_PAIR4K_HOT 8
#define CRLOT_K_PAIR4K 9
#define CRLOT_K_FUSED 10         /* per-frame fused walker, one frame per wave in flight */
#define CRLOT_K_FUSED2 11        /* ... two frames per wave in flight */
#define CRLOT_K_FUSED_WG 12      /* per-frame workgroup walker, N = 4096 */
#define CRLOT_K_PAIR15 13        /* N = 960 / 480 pairs */
#define CRLOT_K_PAIRN 14         /* N = 320 ... 1764 pairs (2, 3, 5, 7 factors) */
#define CRLOT_K_PAIR30 15        /* N = 1920 pairs, even hops */
#define CRLOT_K_FUSED_ANY 16     /* any-size per-frame walker (all streams, or the flagged ones) */
#define CRLOT_K_SYNTH 17         /* staged path: frames */
#define CRLOT_K_SYNTH_ANY 18
#define CRLOT_K_GATHER 19        /* staged path: overlap-add gather */
#define CRLOT_K_DEINTERLEAVE 20
#define CRLOT_K_INTERLEAVE 21
#define CRLOT_K_FFT 22           /* batched rfft / irfft / cfft */
#define CRLOT_K_FFT_ANY 23
#define CRLOT_K_STFT 24          /* crlot_stft: x -> spectra */
#define CRLOT_K_ISTFT 25         /* crlot_istft_ola: spectra -> step -> y */
#define CRLOT_K_STFT_MASKED 26   /* crlot_roundtrip with a spectral mask: one walk x -> y */
#define CRLOT_K_SPEC_STEP 27     /* staged spectral step (gain, mask) over spectra in HBM */
#define CRLOT_K_FRAMES_W 28      /* staged windowed frames (mixed-radix stft) */
#define CRLOT_K_PAIR_MASK 29     /* N = 1024 frame-pair walk with the per-frame mask */
#define CRLOT_K_PAIR_STFT 30     /* crlot_stft as frame pairs (N = 1024) */
#define CRLOT_K_PAIR_ISTFT 31    /* crlot_istft_ola as frame pairs (N = 1024) */
#define CRLOT_K_EXPERIMENT 99    /* experiment builds only */
typedef struct crlot_launch_info {
    int32_t n_kernels;
    int32_t kernels[8];
    int64_t grid[8];
    int32_t n_chunks;
    int32_t reserved;
} crlot_launch_info;
int crlot_plan_last_launch(const crlot_plan* plan, void* stream, crlot_launch_info* out);
/* Name of a CRLOT_K_* id ("k_pair_hot", ...); "unknown" otherwise. */
const char* crlot_kernel_name(int32_t kernel_id);
int crlot_plan_info(const crlot_plan* plan, int32_t* frame_size, int32_t* hop_size,
                    int32_t* ring_len);
/* Frames of a T-sample stream: Framer whole push (framer.cc:88-117) or
 * FrameQueue::calculateNumFrames on the padded length (FrameQueue.cc:98-115) */
int64_t crlot_frame_count(const crlot_plan* plan, int64_t T);
/* Samples the streaming-interleaved round trip emits: F*H */
int64_t crlot_output_length(const crlot_plan* plan, int64_t T);
/* Device workspace a non-fast-path crlot_roundtrip needs (bytes); reserve it
 * up front so the launch itself never allocates (graph capture).
 * crlot_plan_reserve grows the default (NULL) stream's slot and waits for it;
 * crlot_plan_reserve_stream grows `stream`'s slot (regime flags, frame
 * workspace, channel planes) for round trips of n_streams groups of `channels`
 * channels (1 = crlot_roundtrip) of T samples, stream-ordered. */
int64_t crlot_workspace_bytes(const crlot_plan* plan, int32_t n_streams, int64_t T);
int crlot_plan_reserve(crlot_plan* plan, int64_t bytes);
int crlot_plan_reserve_stream(crlot_plan* plan, int32_t n_streams, int64_t T, int32_t channels,
                              void* stream);

/* ---------------------------------------------------------------- hot path */
/* The round trip for n_streams independent mono streams: stream s reads
 * d_x[s*ld_x + t], t < T, and writes d_y[s*ld_y + n], n < crlot_output_length.
 * Equals, per stream, Framer(push whole) -> pop -> *w -> IFftPlan::forward ->
 * (spectral hook) -> IFftPlan::inverse -> OLAAccumulator::push_frame_AoS(k*H)
 * -> produce(H), frame after frame.  With CRLOT_FRAMEQUEUE the frames are
 * FrameQueue(x, T, N, H, center, pad_mode).getFrame(k) (output sample n is at
 * padded position n) -- the performance_benchmark.cc:174-246 pipeline, with
 * analysis_window = 0 there.  d_x may be NULL when T == 0. */
int crlot_roundtrip(crlot_plan* plan, const float* d_x, float* d_y, int32_t n_streams, int64_t T,
                    int64_t ld_x, int64_t ld_y, void* stream);

/* The same round trip for n_groups groups of `channels` interleaved channels
 * (the reference's multi-channel PCM: Framer::set_params(N, H, C) frames N*C
 * interleaved samples, push_frame_AoS deinterleaves them; framer.cc:15-35,
 * aos_to_soa.cc:7-18): group g's input is T rows of C samples at d_x + g*ld_x
 * (ld_x >= T*C), its output F*H rows of C samples at d_y + g*ld_y.  Every
 * channel is an independent stream, bit-identical to crlot_roundtrip on that
 * channel's plane.  N = 1024 plans with zero padding walk the interleaved rows
 * of up to 5 channels directly (K_pair with strided hop loads and stores: one
 * pass over HBM); other plans and wider rows run LDS-tiled deinterleave -> the
 * mono kernels -> interleave through a plan-owned workspace of
 * n_groups*C*(T + F*H) floats (two extra HBM passes). */
int crlot_roundtrip_interleaved(crlot_plan* plan, const float* d_x, float* d_y, int32_t n_groups,
                                int32_t channels, int64_t T, int64_t ld_x, int64_t ld_y, void* stream);

/* Per-stage outputs of the same path (parity/debug): d_frames gets, per
 * stream and frame, the N-sample push_frame_AoS input (sanitized inverse
 * output, before the synthesis window), [s][k][N]; d_spec (optional) the
 * forward spectrum [s][k][N/2+1] complex (float pairs). */
int crlot_roundtrip_stages(crlot_plan* plan, const float* d_x, int32_t n_streams, int64_t T,
                           int64_t ld_x, float* d_frames, float* d_spec, void* stream);

/* OLAAccumulator over precomputed frames: d_frames [s][k][ld_frames] (k < F)
 * pushed at k*H with the plan's synthesis window (apply_window_inside) and
 * gain, normalised by max(norm, eps) and produced in H-sample steps:
 * d_y[s*ld_y + n], n < F*H.  Bit-exact with the reference given equal frames. */
int crlot_ola_gather(crlot_plan* plan, const float* d_frames, float* d_y, int32_t n_streams,
                     int64_t F, int64_t ld_frames, int64_t ld_y, void* stream);

/* ---------------------------------------------------------------- the spectral step
 * The round trip split where the reference's harness leaves its spectral
 * processing step (e2e_benchmark.cc:160-162, identity there), so any
 * device-side processing -- masks, Wiener gains, a model -- can sit between
 * the halves with the spectra in HBM.
 *
 * crlot_stft: the analysis half.  Per stream and frame (framing exactly as
 * crlot_roundtrip: Framer ZERO_PAD / DROP or FrameQueue), frame * analysis
 * window, then IFftPlan::forward (sanitize, kiss_fftr; kissfft_adapter.cc
 * :83-122): spectrum k of stream s, N/2+1 complex bins as float pairs, at
 * d_spec[s*ld_spec + k*ld_frame + 2*b], b <= N/2.  ld_frame >= N+2 floats;
 * d_spec 8-byte aligned, ld_frame and ld_spec even.  F = crlot_frame_count(T)
 * frames per stream.  Bit-identical to crlot_rfft_batched on the windowed
 * frames.
 *
 * crlot_istft_ola: the synthesis half.  Spectra in that layout (F frames per
 * stream) -> the plan's spectral step (the per-bin gain of
 * crlot_plan_set_spectral_gain, then row k of the mask below) ->
 * IFftPlan::inverse (kiss_fftri, *1/N, sanitize; kissfft_adapter.cc:124-168)
 * -> push_frame_AoS(k*H) with the synthesis window and gain -> produce(H)
 * (OLAAccumulator.cc:124-221): d_y[s*ld_y + n], n < F*H.  Bit-identical to
 * crlot_irfft_batched of the stepped spectra + crlot_ola_gather.  The imaginary
 * parts of bins 0 and N/2 are ignored, as kiss_fftri ignores them.
 *
 * crlot_plan_set_spectral_mask: a time-varying spectral step.  Row (s, k) of
 * N/2+1 real floats at d_mask[s*ld_stream + k*ld_frame] multiplies frame k of
 * stream s after the per-bin gain (ld_stream = 0: one row per frame, shared by
 * every stream).  Device memory owned by the caller, read by every later
 * crlot_roundtrip, crlot_roundtrip_interleaved (stream = channel plane
 * g*C + c) and crlot_istft_ola on the plan until it is replaced or cleared
 * (NULL); it must hold a row for every frame those calls run.  With a mask,
 * crlot_roundtrip(x) equals crlot_istft_ola(crlot_stft(x)) bit for bit (one
 * walk over HBM where the shape allows it: power-of-two N, H % 128 == 0,
 * N % H == 0, 8-byte aligned output rows).  The streaming objects, the host-pointer
 * calls and crlot_roundtrip_stages keep the per-bin gain only. */
int crlot_plan_set_spectral_mask(crlot_plan* plan, const float* d_mask, int64_t ld_frame, int64_t ld_stream);
int crlot_stft(crlot_plan* plan, const float* d_x, float* d_spec, int32_t n_streams, int64_t T, int64_t ld_x,
               int64_t ld_spec, int64_t ld_frame, void* stream);
int crlot_istft_ola(crlot_plan* plan, const float* d_spec, float* d_y, int32_t n_streams, int64_t F,
                    int64_t ld_spec, int64_t ld_frame, int64_t ld_y, void* stream);

/* Batched IFftPlan::forward / inverse with the adapter's semantics
 * (kissfft_adapter.cc:83-168): forward sanitizes its input, inverse scales by
 * 1/N and sanitizes its output.  Element i of batch b lives at
 * [b*ld + i*inc] (float for real data, float pairs for spectra). */
int crlot_rfft_batched(crlot_plan* plan, const float* d_in, float* d_out_complex, int32_t batch,
                       int64_t ld_in, int64_t inc_in, int64_t ld_out, int64_t inc_out,
                       void* stream);
int crlot_irfft_batched(crlot_plan* plan, const float* d_in_complex, float* d_out, int32_t batch,
                        int64_t ld_in, int64_t inc_in, int64_t ld_out, int64_t inc_out,
                        void* stream);

/* ---------------------------------------------------------------- FFT plans
 * dsp::fft::MakeFftPlan / IFftPlan (fft_api.h:16-51; kissfft_adapter.cc:11-269)
 * as a device object of its own, both domains.  Semantics per entry point:
 *   forward          real, sanitized input -> nfft/2+1 bins   (adapter :83-122)
 *   inverse          nfft/2+1 bins -> real, *1/nfft, sanitize  (adapter :124-168)
 *   forward_complex  complex -> complex, unnormalised, no sanitize (adapter :171-201)
 *   inverse_complex  complex -> complex, *1/nfft, sanitize     (adapter :204-246)
 * Calling the other domain's entry is CRLOT_ERUNTIME with the reference's
 * message.  Element i of batch b is at [b*ld + i*inc] (ld in floats, inc in
 * elements: floats for real data, float pairs for complex).  Sizes: real nfft
 * even in 2..16384, complex nfft 1..8192 (any factorisation, as kiss_fft);
 * larger sizes are CRLOT_EUNSUPPORTED.  No batch ceiling on the device path;
 * MakeFftPlan's 1..16 rule is applied by the C++ layer (crlot_dsp.hpp). */
#define CRLOT_FFT_REAL 0
#define CRLOT_FFT_COMPLEX 1
typedef struct crlot_fft_plan crlot_fft_plan;
typedef struct crlot_fft_desc {
    int32_t domain; /* CRLOT_FFT_REAL / CRLOT_FFT_COMPLEX (FftPlanDesc::domain) */
    int32_t nfft;   /* FftPlanDesc::nfft */
    int32_t device; /* HIP device ordinal, -1 = current */
} crlot_fft_desc;
int crlot_fft_plan_create(const crlot_fft_desc* desc, crlot_fft_plan** out);
void crlot_fft_plan_destroy(crlot_fft_plan* plan);
int crlot_fft_plan_info(const crlot_fft_plan* plan, int32_t* domain, int32_t* nfft);
int crlot_fft_forward(crlot_fft_plan* plan, const float* d_in, float* d_out_complex, int32_t batch,
                      int64_t ld_in, int64_t inc_in, int64_t ld_out, int64_t inc_out, void* stream);
int crlot_fft_inverse(crlot_fft_plan* plan, const float* d_in_complex, float* d_out, int32_t batch,
                      int64_t ld_in, int64_t inc_in, int64_t ld_out, int64_t inc_out, void* stream);
int crlot_fft_forward_complex(crlot_fft_plan* plan, const float* d_in_complex, float* d_out_complex,
                              int32_t batch, int64_t ld_in, int64_t inc_in, int64_t ld_out,
                              int64_t inc_out, void* stream);
int crlot_fft_inverse_complex(crlot_fft_plan* plan, const float* d_in_complex, float* d_out_complex,
                              int32_t batch, int64_t ld_in, int64_t inc_in, int64_t ld_out,
                              int64_t inc_out, void* stream);

/* Host-pointer forms of the four transforms: the reference's own calling
 * convention (IFftPlan::forward(const float*, complex<float>*, batch) etc.),
 * synchronous, data in host memory, same semantics and layout parameters as
 * the device forms.  Power-of-two plans (real nfft 256..4096, complex
 * 128..2048) run on a resident server kernel owned by the plan (call_rt.hip):
 * no kernel launch and no copy-engine transfer per call, the input written into
 * fine-grained device memory through the BAR, the result written by the kernel
 * into pinned host memory.  After a real forward of batch <= 4 the server also
 * runs the inverse of the spectrum it returned; an inverse called next with
 * exactly those bits (memcmp) is served from that result (bit-identical to
 * running it).  The server exits after 20 ms without a call.  Other sizes stage
 * through device buffers and a launch. */
int crlot_fft_forward_host(crlot_fft_plan* plan, const float* in, float* out_complex, int32_t batch,
                           int64_t ld_in, int64_t inc_in, int64_t ld_out, int64_t inc_out);
int crlot_fft_inverse_host(crlot_fft_plan* plan, const float* in_complex, float* out, int32_t batch,
                           int64_t ld_in, int64_t inc_in, int64_t ld_out, int64_t inc_out);
int crlot_fft_forward_complex_host(crlot_fft_plan* plan, const float* in_complex, float* out_complex,
                                   int32_t batch, int64_t ld_in, int64_t inc_in, int64_t ld_out,
                                   int64_t inc_out);
int crlot_fft_inverse_complex_host(crlot_fft_plan* plan, const float* in_complex, float* out_complex,
                                   int32_t batch, int64_t ld_in, int64_t inc_in, int64_t ld_out,
                                   int64_t inc_out);

/* ---------------------------------------------------------------- streaming
 * Low-latency per-hop path (BASELINE config 4): `channels` independent
 * channels, Framer in DROP mode fed H samples per channel per call
 * (Framer::push of one hop then pop, OLAAccumulator push_frame_AoS + produce(H);
 * framer.cc:37-117, OLAAccumulator.cc:124-221).  Each call consumes d_hop_in
 * and, once N samples per channel have arrived, writes the next H output
 * samples per channel into d_hop_out; *emitted (host) gets 0 or H.  Layout:
 * channel-major [channels][H] by default, or interleaved [H][channels] (the
 * reference's interleaved PCM) after crlot_stream_set_layout(st, 1).  Device
 * state (the recent input samples, the OLA blocks) persists across calls.  Any
 * N / H the plan accepts: H % 128 == 0, N % H == 0, N <= 2048 run the
 * register-resident per-hop kernel, other shapes the mixed-radix one. */
int crlot_stream_create(crlot_plan* plan, int32_t channels, crlot_stream** out);
void crlot_stream_destroy(crlot_stream* st);
int crlot_stream_reset(crlot_stream* st);
int crlot_stream_set_layout(crlot_stream* st, int32_t interleaved);
int crlot_stream_push_hop(crlot_stream* st, const float* d_hop_in, float* d_hop_out,
                          int32_t* emitted, void* stream);

/* ---------------------------------------------------------------- resident streaming
 * The same per-hop contract as crlot_stream_* (DROP Framer fed H samples per
 * channel per hop, push_frame_AoS + produce(H); framer.cc:37-117,
 * OLAAccumulator.cc:124-221; bit-identical outputs) for real-time callers whose
 * hops live in HOST memory (BASELINE config 4, the ring-buffer low-latency path).
 * One kernel stays resident on the device with the tables in LDS and each
 * channel's state in registers; hops travel through pinned host rings of
 * `depth` slots (0 -> 4) with a doorbell, so a hop costs no kernel launch and no
 * copy-engine transfer.  The kernel exits after 20 ms without a hop (or on
 * reset / destroy / a plan table update) and is relaunched by the next hop; a
 * hipDeviceSynchronize elsewhere in the process therefore waits at most that
 * idle time.  N in 256..2048, H % 128 == 0, N % H == 0, channels 1..1024.
 * Every other shape the plan streams (960/480, 882/441 ...) gets the same
 * contract in launch mode: per hop an H2D copy of the slot, the per-launch hop
 * kernel (crlot_stream_push_hop's, bit-identical), a D2H copy and an event; no
 * resident kernel (info reports last_device_ns 0, running 0).
 *   push_hop      copy h_in into the next slot, submit, wait, copy the H output
 *                 samples per channel into h_out (*emitted = 0 or H); h_in /
 *                 h_out are [H][C] interleaved PCM if `interleaved`, else [C][H]
 *   input_slot    zero-copy form: the host slot for the next hop (C*H floats,
 *                 always channel-major [C][H]), then submit -> hop index,
 *                 wait -> pointer to that hop's [C][H] output slot (valid until hop
 *                 index + depth is submitted); up to `depth` hops in flight
 *   info          hops submitted, the device time of the last hop (ns, from the
 *                 kernel's own clock: doorbell seen -> output published), running */
typedef struct crlot_stream_rt crlot_stream_rt;
int crlot_stream_rt_create(crlot_plan* plan, int32_t channels, int32_t interleaved, int32_t depth,
                           crlot_stream_rt** out);
void crlot_stream_rt_destroy(crlot_stream_rt* st);
int crlot_stream_rt_reset(crlot_stream_rt* st);
int crlot_stream_rt_push_hop(crlot_stream_rt* st, const float* h_hop_in, float* h_hop_out,
                             int32_t* emitted);
float* crlot_stream_rt_input_slot(crlot_stream_rt* st);
int crlot_stream_rt_submit(crlot_stream_rt* st, int64_t* hop_index);
int crlot_stream_rt_wait(crlot_stream_rt* st, int64_t hop_index, const float** h_hop_out,
                         int32_t* emitted);
int crlot_stream_rt_info(const crlot_stream_rt* st, int64_t* hops, double* last_device_ns,
                         int32_t* running);
/* diagnostic: workgroup 0's phase times of the last hop (ns after the doorbell
 * was seen: hop read issued, hop staged, transform done, output barrier, output
 * issued, release fence, publish barrier); zeros unless the library was built
 * with -DCRLOT_RT_PHASES */
int crlot_stream_rt_phases(const crlot_stream_rt* st, double* ns8);
/* idle exit after `idle_seconds` without a hop; a wait fails (CRLOT_EHIP) after
 * `hop_timeout_seconds` (defaults 0.02 and 2) */
int crlot_stream_rt_set_idle_timeout(crlot_stream_rt* st, double idle_seconds,
                                     double hop_timeout_seconds);

/* ---------------------------------------------------------------- Framer (host)
 * dsp::Framer (framer.h:26-127, framer.cc:15-181): interleaved PCM of
 * `channels` channels in, frames of frame_size*channels interleaved samples out
 * every hop_size samples per channel; ZERO_PAD pads the last partial frame with
 * zeros, DROP never emits one.  A host object (bookkeeping and copies); the
 * batched crlot_roundtrip frames on the device instead.
 * push / pop return 1 (true) or 0 (false) as the reference's bool, negative on
 * a bad handle; set_params fails with CRLOT_EINVAL and the reference's message
 * (std::invalid_argument) on a zero size. */
typedef struct crlot_framer crlot_framer;
int crlot_framer_create(crlot_framer** out);
void crlot_framer_destroy(crlot_framer* f);
int crlot_framer_set_params(crlot_framer* f, int64_t frame_size, int64_t hop_size, int64_t channels,
                            int32_t boundary_mode);
int crlot_framer_push(crlot_framer* f, const float* interleaved, int64_t frames);
int crlot_framer_pop(crlot_framer* f, float* out_frame);
int64_t crlot_framer_available(const crlot_framer* f);
int crlot_framer_reset(crlot_framer* f);
int crlot_framer_info(const crlot_framer* f, int64_t* frame_size, int64_t* hop_size,
                      int64_t* channels, int32_t* boundary_mode, int64_t* buffer_size);

/* ---------------------------------------------------------------- OLAAccumulator
 * dsp::OLAAccumulator (OLAAccumulator.h:15-217, OLAAccumulator.cc:13-295) with
 * its state on the device: per-channel rings [channels][ring_len] and the COLA
 * divisors in HBM, every add / produce a kernel; the host keeps the reference's
 * counters (produced_samples, read_pos, flush, reset) so any call sequence
 * behaves as the reference's.  Per-sample arithmetic is the reference's scalar
 * kernels (kernels.cc:18-36): fma(fma(x, w, 0), gain, acc) or fma(x, gain, acc);
 * out = acc / (norm > eps ? norm : eps), acc = 0.
 * Two call forms: host pointers (the reference's signatures) run on a resident
 * server kernel owned by the object (call_rt.hip): an add is posted without
 * waiting, produce() returns when the samples are in the caller's buffers; after
 * each add the server also computes the produce(n) block the object predicts
 * (n of the previous produce, H before the first), without clearing, and a
 * produce asking for exactly that block is served from it (the ring is cleared
 * by a request behind it).  _device forms run on caller-owned HBM with a stream
 * (NULL = the object's stream); calls on different streams, and switches between
 * the two forms, are ordered by the object.  Null pointers fail with CRLOT_EINVAL and the reference's
 * messages.  Not thread-safe (as the reference). */
typedef struct crlot_ola crlot_ola;
typedef struct crlot_ola_config { /* dsp::OLAConfig (OLAAccumulator.h:15-29) */
    int32_t sample_rate;
    int64_t frame_size;
    int64_t hop_size;
    int64_t channels;
    float eps;                   /* reference default 1e-8f */
    int32_t apply_window_inside;
    int32_t shadow_ring;         /* accepted; value-neutral (ola_accumulator_test.cc:1079-1120) */
    int32_t device;              /* HIP device ordinal, -1 = current */
} crlot_ola_config;
int crlot_ola_create(const crlot_ola_config* cfg, crlot_ola** out);
void crlot_ola_destroy(crlot_ola* o);
int crlot_ola_set_window(crlot_ola* o, const float* window, int32_t wlen);
/* ch_frames[c] (host), c < channels */
int crlot_ola_add_frame_soa(crlot_ola* o, const float* const* ch_frames, const float* window,
                            int64_t start_sample, int64_t start_off, int64_t size, float gain);
/* interleaved [frame_size][channels] (host) */
int crlot_ola_push_frame_aos(crlot_ola* o, const float* interleaved, const float* window,
                             int64_t start_sample, int64_t start_off, int64_t size, float gain);
/* ch_out[c] (host) receives up to n samples; *n_out = samples provided */
int crlot_ola_produce(crlot_ola* o, float* const* ch_out, int64_t n, int64_t* n_out);
/* device forms: channel c of a frame at d_frames + c*ld_frames; window (when the
 * object does not apply its own) a device array of frame_size floats */
int crlot_ola_add_frame_soa_device(crlot_ola* o, const float* d_frames, int64_t ld_frames,
                                   const float* d_window, int64_t start_sample, int64_t start_off,
                                   int64_t size, float gain, void* stream);
int crlot_ola_push_frame_aos_device(crlot_ola* o, const float* d_interleaved, const float* d_window,
                                    int64_t start_sample, int64_t start_off, int64_t size, float gain,
                                    void* stream);
/* channel c written to d_out + c*ld_out (n floats per channel must be valid) */
int crlot_ola_produce_device(crlot_ola* o, float* d_out, int64_t ld_out, int64_t n, int64_t* n_out,
                             void* stream);
int crlot_ola_flush(crlot_ola* o);
int crlot_ola_reset(crlot_ola* o);
int crlot_ola_info(const crlot_ola* o, int64_t* produced_samples, int64_t* read_pos,
                   int64_t* ring_size, int32_t* has_window);
/* channel-0 peak of every sample produced so far (waits for device produces) */
int crlot_ola_meter_peak(crlot_ola* o, float* peak);
/* the object's COLA norm table (ring_size floats, before the eps guard) */
int crlot_ola_norm_table(const crlot_ola* o, float* out);
/* wait for everything issued on the object */
int crlot_ola_synchronize(crlot_ola* o);

/* ---------------------------------------------------------------- OLA kernels
 * dsp::axpy / axpy_windowed / normalize_and_clear (ola/kernels.h:28-53; scalar
 * forms kernels.cc:18-36, which the Highway forms match) as batched device
 * entries: `batch` rows of n elements, row b of dst / src / out / acc at
 * + b*ld; the window (axpy_windowed) and the norm row (normalize_and_clear) are
 * one row of n shared by every row.  Per element, bit-exact with the reference:
 *   axpy               dst = fma(src, g, dst)
 *   axpy_windowed      dst = fma(fma(src, win, 0), g, dst)
 *   normalize_and_clear out = acc / (norm > eps ? norm : eps), acc = 0
 * batch <= 65535.
 * crlot_call_*: the reference's host-pointer signatures (n elements in host
 * memory, synchronous), run on a per-device resident server kernel
 * (call_rt.hip); normalize_and_clear also zeroes acc, as the reference. */
int crlot_axpy(float* d_dst, const float* d_src, float g, int64_t n, int64_t batch, int64_t ld_dst,
               int64_t ld_src, void* stream);
int crlot_axpy_windowed(float* d_dst, const float* d_src, const float* d_win, float g, int64_t n,
                        int64_t batch, int64_t ld_dst, int64_t ld_src, void* stream);
int crlot_normalize_and_clear(float* d_out, float* d_acc, const float* d_norm, float eps, int64_t n,
                              int64_t batch, int64_t ld_out, int64_t ld_acc, void* stream);
int crlot_call_axpy(float* dst, const float* src, float g, int64_t n);
int crlot_call_axpy_windowed(float* dst, const float* src, const float* win, float g, int64_t n);
int crlot_call_normalize_and_clear(float* out, float* acc, const float* norm, float eps, int64_t n);

/* ---------------------------------------------------------------- FrameQueue
 * dsp::FrameQueue (FrameQueue.h:35-59, FrameQueue.cc:9-115, Indexing.h:18-70):
 * all frames of a whole signal, padded by N/2 on both sides when `center`
 * (CRLOT_PAD_CONSTANT zeros / REFLECT reflect-101 / EDGE), frame k = padded
 * samples [k*H, k*H + N), count floor((len + pad - max(N - H, 0)) / H) on the
 * padded length.  The object builds the frames on the device at construction
 * (device_frames: [num_frames][N] in HBM) and keeps the reference's AoS host
 * copy for frame / copy_frame / all_frames.  Errors: CRLOT_EINVAL with the
 * reference's std::invalid_argument messages, CRLOT_ERANGE for a frame index
 * out of range (std::out_of_range; crlot_framequeue_frame returns NULL).
 * crlot_framequeue_frames is the batched device form: n_streams streams of T
 * samples at d_x + s*ld_x -> d_frames [s][count][frame_size]. */
typedef struct crlot_framequeue crlot_framequeue;
int64_t crlot_framequeue_count(int64_t T, int64_t frame_size, int64_t hop_size, int32_t center);
int crlot_framequeue_frames(const float* d_x, int32_t n_streams, int64_t T, int64_t ld_x, int64_t frame_size,
                            int64_t hop_size, int32_t center, int32_t pad_mode, float* d_frames, void* stream);
int crlot_framequeue_create(const float* in, int64_t len, int64_t frame_size, int64_t hop_size, int32_t center,
                            int32_t pad_mode, int32_t device, crlot_framequeue** out);
void crlot_framequeue_destroy(crlot_framequeue* q);
int crlot_framequeue_info(const crlot_framequeue* q, int64_t* num_frames, int64_t* frame_size,
                          int64_t* hop_size);
const float* crlot_framequeue_frame(const crlot_framequeue* q, int64_t frame_idx);
int crlot_framequeue_copy_frame(const crlot_framequeue* q, int64_t frame_idx, float* out);
const float* crlot_framequeue_all_frames(const crlot_framequeue* q);
const float* crlot_framequeue_device_frames(const crlot_framequeue* q);

/* ---------------------------------------------------------------- WAV I/O
 * io/wav.{h,cc} (WavReader / WavWriter over dr_wav): RIFF WAVE, 1 or 2
 * channels, 16/24/32-bit PCM or 32-bit IEEE float (wav.cc:26-55 guards; a
 * rejected file is CRLOT_ERUNTIME, the reference's `false`).  Samples are
 * interleaved float frames with dr_wav's conversions: s16 * 2^-15,
 * s24 * 2^-23, s32 / 2^31 on read; drwav_f32_to_s16 / the reference's 24-bit
 * packer (wav.cc:233-246) / 2^31 * x (clamped) on write.  Host memory only. */
typedef struct crlot_wav_reader crlot_wav_reader;
typedef struct crlot_wav_writer crlot_wav_writer;
int crlot_wav_reader_open(const char* path, crlot_wav_reader** out);
void crlot_wav_reader_close(crlot_wav_reader* r);
int crlot_wav_reader_info(const crlot_wav_reader* r, uint32_t* channels, uint32_t* sample_rate,
                          uint64_t* total_frames, uint32_t* bits_per_sample, int32_t* is_float);
/* reads up to `frames` frames from the current position; *frames_read < frames at the end */
int crlot_wav_reader_read(crlot_wav_reader* r, float* out, uint64_t frames, uint64_t* frames_read);
int crlot_wav_writer_open(const char* path, uint32_t channels, uint32_t sample_rate,
                          uint32_t bits_per_sample, int32_t float_format, crlot_wav_writer** out);
int crlot_wav_writer_write(crlot_wav_writer* w, const float* in, uint64_t frames, uint64_t* written);
/* patches the RIFF/data sizes and closes the file */
int crlot_wav_writer_close(crlot_wav_writer* w);

/* ---------------------------------------------------------------- host tables
 * The reference's table builders, restated in the product's host code
 * (bit-exact with WindowLUT.cc / norm_builder.cc / OLAAccumulator.cc). */
int crlot_window_table(int32_t type, int64_t n, int32_t periodic, int32_t norm, float* out);
int64_t crlot_ring_len(int64_t frame_size, int64_t hop);
int crlot_norm_table(const float* window, int64_t frame_size, int64_t hop, int64_t ring_len,
                     int32_t apply_window_inside, float eps, float* out);
/* dsp::ola::build_norm_linear (norm_builder.cc:8-52): the raw linear sum of the
 * window over every frame start that reaches the ring (no eps, no H == N case) */
int crlot_build_norm_linear(float* norm, const float* window, int64_t ring_len, int64_t frame_size, int64_t hop);
/* The device the calling thread's HIP context uses, as an ISA name ("gfx950");
 * the target of the dsp::get_current_target() drop-in */
const char* crlot_device_target(void);

#ifdef __cplusplus
}
#endif
#endif /* CRLOT_DSP_H_ */
