/*
 * crlot_oracle.h -- CPU restatement of crlot-dsp's STFT->OLA hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (crlot-dsp_amd/, include/)
 * links, loads or calls this.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may use it, and only as the checker / the timed
 * CPU baseline ("kind": "port").
 *
 * Parity pins (see DESIGN.md "Oracle"):
 *   - window / norm / Framer: bit-exact against oracle/_ref (the reference's
 *     own WindowLUT.cc, norm_builder.cc, framer.cc compiled unchanged) through
 *     the fixtures in tests/golden/.
 *   - kissfft: kissfft 131.1.0 is an absent third-party dependency (empty
 *     submodule third_party/kissfft, /root/reference/Makefile:17).  Its
 *     published algorithm is restated here and pinned by the reference's own
 *     known-answer tests (tests/fft_test.cc) and a float64 DFT.
 *   - OLAAccumulator: OLAAccumulator.cc + kernels.cc scalar FMA semantics.
 *     kernels_hwy.cc needs Highway (absent), so the reference OLA object is not
 *     buildable here; the restatement is pinned by the reference's own tests
 *     (ola_accumulator_test.cc H==N reconstruction etc.).
 */
#ifndef CRLOT_ORACLE_H_
#define CRLOT_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* dsp::WindowType / NormalizationType ordinals (WindowLUT.h:14-31) */
enum { OR_HANN = 0, OR_HAMMING = 1, OR_BLACKMAN = 2, OR_RECT = 3, OR_BLACKMAN_HARRIS = 4 };
enum { OR_NORM_NONE = 0, OR_NORM_SUM_TO_ONE = 1, OR_NORM_L2 = 2, OR_NORM_OLA_UNITY_GAIN = 3,
       OR_NORM_OLA_SUM_WSQ = 4 };
/* dsp::BoundaryMode (framer.h:11-14) */
enum { OR_ZERO_PAD = 0, OR_DROP = 1 };

/* ---- WindowLUT::createWindow (WindowLUT.cc:215-254, 256-388) ----
 * returns 0, -1 for N==0, -2 for BLACKMAN_HARRIS / unknown type. */
int or_window(int type, size_t n, int periodic, int norm, float* out);

/* ---- OLAAccumulator::calculate_ring_size (OLAAccumulator.cc:249-258) ---- */
size_t or_ring_len(size_t frame_size, size_t hop);
/* ---- dsp::ola::build_norm_linear (norm_builder.cc:8-52) ---- */
void or_build_norm_linear(float* norm, const float* window, size_t ring_len, size_t frame_size,
                          size_t hop);
/* ---- OLAAccumulator::initialize_normalization (OLAAccumulator.cc:260-288);
 * window may be NULL (no window set). */
void or_init_normalization(float* norm, const float* window, size_t ring_len, size_t frame_size,
                           size_t hop, int apply_window_inside, float eps);

/* ---- dsp::Framer state machine (framer.cc:15-181) ---- */
typedef struct or_framer or_framer;
or_framer* or_framer_new(size_t frame_size, size_t hop, size_t channels, int mode);
void or_framer_free(or_framer*);
int or_framer_push(or_framer*, const float* interleaved, size_t frames); /* 1 ok, 0 fail */
int or_framer_pop(or_framer*, float* out_frame);                         /* 1 frame, 0 none */
size_t or_framer_available(const or_framer*);
void or_framer_reset(or_framer*);

/* ---- kissfft 131.1.0 restatement (kiss_fft.c / kiss_fftr.c, float) ---- */
typedef struct or_kfft_cfg or_kfft_cfg;
or_kfft_cfg* or_kfft_alloc(int nfft, int inverse);
void or_kfft_free(or_kfft_cfg*);
/* fin/fout: interleaved complex float[2*nfft]; fin may equal fout */
void or_kfft(or_kfft_cfg*, const float* fin, float* fout);
typedef struct or_kfftr_cfg or_kfftr_cfg;
or_kfftr_cfg* or_kfftr_alloc(int nfft, int inverse); /* nfft even */
void or_kfftr_free(or_kfftr_cfg*);
void or_kfftr(or_kfftr_cfg*, const float* timedata, float* freqdata /* complex[nfft/2+1] */);
void or_kfftri(or_kfftr_cfg*, const float* freqdata, float* timedata);

/* ---- KissFftPlan::forward / inverse for one batch element
 * (kissfft_adapter.cc:83-168): sanitize -> kiss_fftr ; kiss_fftri -> *1/N -> sanitize ---- */
void or_adapter_forward(or_kfftr_cfg* fwd, int nfft, const float* in, float* out_complex);
void or_adapter_inverse(or_kfftr_cfg* inv, int nfft, const float* in_complex, float* out);
/* complex domain (kissfft_adapter.cc:171-246) */
void or_adapter_forward_complex(or_kfft_cfg* fwd, int nfft, const float* in, float* out);
void or_adapter_inverse_complex(or_kfft_cfg* inv, int nfft, const float* in, float* out);

/* ---- OLA kernels, scalar FMA semantics (kernels.cc:18-36) ---- */
void or_axpy(float* dst, const float* src, float g, size_t n);
void or_axpy_windowed(float* dst, const float* src, const float* win, float g, size_t n);
void or_normalize_and_clear(float* out, float* acc, const float* norm, float eps, size_t n);
/* RingBuffer::split (ring_buffer.cc:44-85): first span [s1, s1+l1), second [0, l2) */
void or_ring_split(size_t cap, size_t start, size_t len, size_t* s1, size_t* l1, size_t* l2);
/* ola::deinterleave_to_scratch (aos_to_soa.cc:7-18) */
void or_deinterleave(const float* x, size_t n, size_t channels, float* scratch);
void or_bench_kernel(int op, size_t n, int64_t reps, float* dst, const float* src, const float* win,
                     float* out);

/* ---- OLAAccumulator (OLAAccumulator.cc:13-295), channels SoA ---- */
typedef struct or_ola or_ola;
or_ola* or_ola_new(size_t frame_size, size_t hop, size_t channels, float eps,
                   int apply_window_inside);
void or_ola_free(or_ola*);
void or_ola_set_window(or_ola*, const float* w);
void or_ola_add_frame_soa(or_ola*, const float* const* ch_frames, const float* window,
                          size_t start_sample, size_t start_off, size_t size, float gain);
void or_ola_push_frame_aos(or_ola*, const float* interleaved, const float* window,
                           size_t start_sample, size_t start_off, size_t size, float gain);
size_t or_ola_produce(or_ola*, float* const* ch_out, size_t n);
void or_ola_flush(or_ola*);
void or_ola_reset(or_ola*);
size_t or_ola_ring_size(const or_ola*);
const float* or_ola_norm(const or_ola*);
size_t or_ola_produced(const or_ola*);
size_t or_ola_read_pos(const or_ola*);
float or_ola_meter_peak(const or_ola*);

/* ---- the hot path, streaming-interleaved reading of bench/e2e_benchmark.cc:138-186 ----
 * One mono stream x[0..T).  Framer(mode) whole push -> pop -> frame*w ->
 * forward -> (identity) -> inverse -> push_frame_AoS(start=k*H, window inside)
 * -> produce(H).  Writes min(F*H, y_cap) samples of y, returns F (frame count).
 * frames_out (optional, F*N floats) receives the synthesis-stage input of
 * push_frame_AoS (i.e. the sanitized inverse output), spec_out (optional,
 * F*(N/2+1) complex) the forward spectra. */
size_t or_frame_count(size_t T, size_t frame_size, size_t hop, int mode);
long or_roundtrip(const float* x, size_t T, size_t frame_size, size_t hop, int window_type,
                  int periodic, int mode, float* y, size_t y_cap, float* frames_out,
                  float* spec_out);
/* many independent streams (stream s at x + s*ld_x, y + s*ld_y), statically
 * partitioned over nthreads pthreads. Returns frames per stream or <0. */
long or_roundtrip_batch(const float* x, size_t n_streams, size_t T, size_t ld_x, size_t frame_size,
                        size_t hop, int window_type, int periodic, int mode, float* y,
                        size_t ld_y, int nthreads);

/* ---- FrameQueue (dsp/frame/FrameQueue.cc:9-115, Indexing.h:18-70) ----
 * pad_mode: 0 CONSTANT, 1 REFLECT, 2 EDGE (dsp::PadMode ordinals).
 * or_fq_count: frames of a len-T signal; or_fq_frames writes them [F][N]. */
int or_fq_reflect101(int i, int n);
float or_fq_pad_value(const float* data, int len, int idx, int pad_mode);
size_t or_fq_count(size_t T, size_t frame_size, size_t hop, int center);
size_t or_fq_frames(const float* x, size_t T, size_t frame_size, size_t hop, int center,
                    int pad_mode, float* frames);

/* Generalised round trip: framing = 0/1 Framer ZERO_PAD/DROP whole push, 2 =
 * FrameQueue(center, pad_mode); analysis_window = multiply frames by w before
 * forward (e2e harness) or not (performance_benchmark.cc:174-246 pipeline).
 * The OLA side is unchanged: add at k*H with the window inside, produce(H)
 * after each frame.  Returns F. */
long or_roundtrip_ex(const float* x, size_t T, size_t frame_size, size_t hop, int window_type,
                     int periodic, int framing, int center, int pad_mode, int analysis_window,
                     float* y, size_t y_cap, float* frames_out, float* spec_out);
/* or_roundtrip with a per-bin real gain applied to every frame's spectrum
 * between the transforms (the spectral step of e2e_benchmark.cc:161-162). */
long or_roundtrip_gain(const float* x, size_t T, size_t n, size_t h, int window_type, int periodic, int framing,
                       const float* bin_gain, float* y, size_t y_cap);
/* the loop with bin_gain then mask row k scaling frame k's spectrum; raw_spec_out:
 * the forward spectra before the step (rows of n + 2 floats) */
/* e2e_benchmark.cc:152-179's literal order: every push, then the produce loop (ring aliasing) */
long or_roundtrip_harness_order(const float* x, size_t T, size_t n, size_t h, int window_type, int periodic,
                                float* y, size_t y_cap);
long or_roundtrip_mask(const float* x, size_t T, size_t n, size_t h, int window_type, int periodic, int framing,
                       int center, int pad_mode, int analysis_window, const float* bin_gain, const float* mask,
                       size_t mask_ld, float* y, size_t y_cap, float* raw_spec_out);
long or_roundtrip_batch_ex(const float* x, size_t n_streams, size_t T, size_t ld_x,
                           size_t frame_size, size_t hop, int window_type, int periodic,
                           int framing, int center, int pad_mode, int analysis_window, float* y,
                           size_t ld_y, int nthreads);

/* splitmix64-based synthetic input: uniform [-1,1) * 0.5 */
void or_synth_fill(float* x, size_t n, unsigned long long seed);

#ifdef __cplusplus
}
#endif
#endif
