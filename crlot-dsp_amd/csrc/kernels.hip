// kernels.hip -- gfx950 kernels of the STFT -> iSTFT -> OLA round trip.
//
// K_fused  k_stft_ola_fused<E,S,NB>: one wave owns a run of consecutive frames
//          of one stream (plus NB-1 warm-up frames) and walks them in order:
//          the frame's input slides through registers (only H new samples are
//          loaded per frame), the FFT/iFFT run in registers + per-wave LDS, and
//          the overlap-add accumulates in registers, so HBM sees 4 B in and
//          4 B out per sample.  Output block k (H samples) is final once frame k
//          is added, exactly the reference's push(k) -> produce(H) order.
// K_synth  k_synth_frames<E>: one wave per frame, any hop; writes the
//          push_frame_AoS input (sanitized inverse output) per frame.
// K_gather k_ola_gather: one thread per output sample, sums the frames in
//          ascending k (the reference's accumulation order) and divides by
//          max(norm, eps): bit-exact OLAAccumulator.
// K_rfft / K_irfft: batched IFftPlan::forward / inverse (adapter semantics).
//
// Numerics (DESIGN.md "Parity"): the float steps the reference fixes are kept
// operation-for-operation -- frame*w (e2e_benchmark.cc:155, a plain multiply),
// sanitize (kissfft_adapter.cc:102-110,156-163), *1/N then sanitize, the OLA
// update fma(fma(src, w, 0), g, dst) (kernels.cc:24-28) and the IEEE division
// acc / max(norm, eps) (kernels.cc:30-36).  Built with -ffp-contract=off and
// the default correctly-rounded f32 division; subnormals are preserved.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "fft_any.h"
#include "fft_pair.h"
#include "fft_pair4k.h"
#include "fft_pair512.h"
#include "fft_pair2k.h"
#include "fft_wave.h"
#include "fused_common.h"
#include "kernels.h"

namespace crlot {

using dev::cf;

namespace {

using namespace fk;

constexpr int kWaves = 4;  // waves per 256-thread workgroup, each independent
constexpr int kBlock = 64 * kWaves;

template <int P>
__host__ __device__ constexpr int xbuf_elems() {
    return P;
}

// LDS carve shared by the kernels: [tw P cf][st P cf][sth P cf][wa N f][ws N f][bufs]
template <int E>
struct Lds {
    static constexpr int P = 64 * E;
    static constexpr int N = 2 * P;
    static constexpr size_t bytes =
        sizeof(cf) * (3 * P) + sizeof(float) * (2 * N) + sizeof(cf) * kWaves * xbuf_elems<P>();
};

template <int E>
__device__ __forceinline__ void load_tables(const DevTables& t, cf* tw, cf* st, cf* sth, float* wa,
                                            float* ws, bool need_windows, const float* ws_src = nullptr) {
    constexpr int P = 64 * E, N = 2 * P;
    const cf* gtw = reinterpret_cast<const cf*>(t.tw);
    const cf* gst = reinterpret_cast<const cf*>(t.st);
    for (int i = threadIdx.x; i < dev::twiddle_table_size(E); i += kBlock) tw[i] = gtw[i];
    for (int i = threadIdx.x; i < P; i += kBlock) {
        const cf w = gst[i];
        st[i] = w;
        sth[i] = cf{w.r * 0.5f, w.i * 0.5f};  // exact
    }
    if (need_windows) {
        const float* gws = ws_src ? ws_src : t.ws;
        for (int i = threadIdx.x; i < N; i += kBlock) {
            wa[i] = t.wa[i];
            ws[i] = gws[i];
        }
    }
    __syncthreads();
}


// The same through a plain pointer and 64-bit indices (staged path).
__device__ __forceinline__ float fetch_x64(const float* x, int64_t j, int64_t T, int mode) {
    if (mode == 1) {
        if (T <= 1) {
            j = 0;
        } else {
            while (j < 0 || j >= T) j = j < 0 ? -j - 1 : 2 * T - 2 - j;
        }
    } else if (mode == 2) {
        j = j < 0 ? 0 : (j >= T ? T - 1 : j);
    }
    return (j >= 0 && j < T) ? x[j] : 0.0f;
}

// Frame loads: lane owns complex samples z[lane + L m] = (x[o + 2i], x[o + 2i + 1]),
// i = lane + L m, o = the frame's origin in x (k*H - pad).  A frame wholly inside
// the stream takes one dwordx2 per pair; an edge frame maps every sample
// through the padding rule (ZERO_PAD tails, FrameQueue centre padding).
template <int M0, int CNT, int E, int L>
__device__ __forceinline__ void load_pairs_l(float2 (&dst)[E], __amdgpu_buffer_rsrc_t rx, int lane,
                                             int origin, int T, int mode) {
    constexpr int N = 2 * L * E;
    if (origin >= 0 && origin + N <= T) {
#pragma unroll
        for (int m = M0; m < M0 + CNT; ++m) dst[m] = dev::bload2(rx, lane * 8 + m * 8 * L, origin * 4);
    } else {
#pragma unroll
        for (int m = M0; m < M0 + CNT; ++m) {
            const int j = origin + 2 * (lane + L * m);
            dst[m] = make_float2(fetch_x(rx, j, T, mode), fetch_x(rx, j + 1, T, mode));
        }
    }
}

#ifndef CRLOT_FUSED_MIN_WAVES
#define CRLOT_FUSED_MIN_WAVES 1
#endif

template <int E, int S, int NB, bool HAS_GAIN, bool FAST = false>
__global__ __launch_bounds__(kBlock, CRLOT_FUSED_MIN_WAVES) void k_stft_ola_fused(const FusedArgs a) {
    constexpr int P = 64 * E, N = 2 * P, H = 128 * S;
    static_assert(NB * S == E, "N = NB * H");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    cf* st = tw + P;
    cf* sth = st + P;
    float* wa = reinterpret_cast<float*>(sth + P);
    float* ws = wa + N;
    cf* bufs = reinterpret_cast<cf*>(ws + N);
    load_tables<E>(a.t, tw, st, sth, wa, ws, true, FAST ? a.t.wsn : nullptr);

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    cf* buf = bufs + wave * xbuf_elems<P>();
    const int gw = blockIdx.x * kWaves + wave;
    if (gw >= a.n_streams * a.n_chunks) return;
    const int s = gw / a.n_chunks, c = gw - s * a.n_chunks;
    const int f0 = c * a.M;
    const int f1 = min(a.F, f0 + a.M);
    const int fs = max(0, f0 - (NB - 1));
    const __amdgpu_buffer_rsrc_t rx = dev::make_rsrc(a.x + int64_t(s) * a.ld_x, uint32_t(a.T) * 4u);
    const __amdgpu_buffer_rsrc_t ry =
        dev::make_rsrc(a.y + int64_t(s) * a.ld_y, uint32_t(a.out_len) * 4u);
    const __amdgpu_buffer_rsrc_t rd = dev::make_rsrc(a.t.den, uint32_t(a.ring_blocks * H) * 4u);
    const __amdgpu_buffer_rsrc_t rr =
        dev::make_rsrc(FAST ? a.t.rden : a.t.den, uint32_t(a.ring_blocks * H) * 4u);
    const float g = a.gain;

#ifndef CRLOT_TW_REGS
#define CRLOT_TW_REGS 0
#endif
#ifndef CRLOT_WIN_REGS
#define CRLOT_WIN_REGS 0
#endif
#if CRLOT_TW_REGS
    dev::TwChain<E, 1> twc;
    dev::load_chain<E, 1, 0>(twc, tw, lane);
#endif
#if CRLOT_WIN_REGS
    float2 wreg_a[E], wreg_s[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        wreg_a[m] = *reinterpret_cast<const float2*>(wa + 2 * (lane + 64 * m));
        wreg_s[m] = *reinterpret_cast<const float2*>(ws + 2 * (lane + 64 * m));
    }
#endif
    float2 xin[E];
    load_pairs_l<0, E, E, 64>(xin, rx, lane, fs * H - a.pad, a.T, a.pad_mode);
    float2 acc[NB][S];
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int q = 0; q < S; ++q) acc[j][q] = make_float2(0.f, 0.f);

    for (int k = fs; k < f1; ++k) {
        // prefetch: frame k+1's new hop and block k's normaliser, consumed at the
        // end of this iteration, so their latency hides under the transforms
        float2 nxt[E];
        if (k + 1 < f1) load_pairs_l<E - S, S, E, 64>(nxt, rx, lane, (k + 1) * H - a.pad, a.T, a.pad_mode);
        float2 dn[S], rn[S];
        if (k >= f0) {
#pragma unroll
            for (int q = 0; q < S; ++q) {
                dn[q] = dev::bload2(rd, lane * 8 + q * 512, (k % a.ring_blocks) * H * 4);
                if constexpr (FAST) rn[q] = dev::bload2(rr, lane * 8 + q * 512, (k % a.ring_blocks) * H * 4);
            }
        }
        // analysis window (harness: frame[i] * w[i]) + forward sanitize
        cf v[E];
#pragma unroll
        for (int m = 0; m < E; ++m) {
#if CRLOT_WIN_REGS
            const float2 w = wreg_a[m];
#else
            const float2 w = *reinterpret_cast<const float2*>(wa + 2 * (lane + 64 * m));
#endif
            v[m].r = dev::sanit(xin[m].x * w.x);
            v[m].i = dev::sanit(xin[m].y * w.y);
        }
#if CRLOT_TW_REGS
        dev::fft_wave_reg<E, false>(v, buf, twc, lane);
        dev::real_split_hook_merge<E, HAS_GAIN, false>(v, buf, st, sth, a.t.gain, lane);
        dev::fft_wave_reg<E, true>(v, buf, twc, lane);
#else
        dev::fft_wave<E, false>(v, buf, tw, lane);
        dev::real_split_hook_merge<E, HAS_GAIN, false>(v, buf, st, sth, a.t.gain, lane);
        dev::fft_wave<E, true>(v, buf, tw, lane);
#endif
        // *1/N, sanitize, synthesis window, OLA accumulate (ascending k)
#pragma unroll
        for (int m = 0; m < E; ++m) {
#if CRLOT_WIN_REGS
            const float2 w = wreg_s[m];
#else
            const float2 w = *reinterpret_cast<const float2*>(ws + 2 * (lane + 64 * m));
#endif
            // FAST: w = ws / N and the 1/N is folded out of the sanitize (exact)
            const float o0 = FAST ? dev::sanit_scaled<N>(v[m].r) : dev::sanit(v[m].r * a.inv_n);
            const float o1 = FAST ? dev::sanit_scaled<N>(v[m].i) : dev::sanit(v[m].i * a.inv_n);
            float2& r = acc[m / S][m % S];
            r.x = __builtin_fmaf(__builtin_fmaf(o0, w.x, 0.0f), g, r.x);
            r.y = __builtin_fmaf(__builtin_fmaf(o1, w.y, 0.0f), g, r.y);
        }
        // block k is complete: produce(H) = acc / max(norm, eps)
        if (FAST && k >= f0) {
            bool ok = true;
#pragma unroll
            for (int q = 0; q < S; ++q) ok = ok && mk_ok(acc[0][q].x) && mk_ok(acc[0][q].y);
            if (__builtin_amdgcn_ballot_w64(!ok) == 0) {
#pragma unroll
                for (int q = 0; q < S; ++q)
                    dev::bstore2(make_float2(mk_div(acc[0][q].x, dn[q].x, rn[q].x),
                                             mk_div(acc[0][q].y, dn[q].y, rn[q].y)),
                                 ry, lane * 8 + q * 512, k * H * 4);
            } else {
#pragma unroll
                for (int q = 0; q < S; ++q)
                    dev::bstore2(make_float2(acc[0][q].x / dn[q].x, acc[0][q].y / dn[q].y), ry,
                                 lane * 8 + q * 512, k * H * 4);
            }
        } else if (k >= f0) {
#pragma unroll
            for (int q = 0; q < S; ++q)
#ifdef CRLOT_ABL_NODIV  // timing-only ablation
                dev::bstore2(make_float2(acc[0][q].x * dn[q].x, acc[0][q].y * dn[q].y), ry,
                             lane * 8 + q * 512, k * H * 4);
#else
                dev::bstore2(make_float2(acc[0][q].x / dn[q].x, acc[0][q].y / dn[q].y), ry,
                             lane * 8 + q * 512, k * H * 4);
#endif
        }
#pragma unroll
        for (int j = 0; j < NB - 1; ++j)
#pragma unroll
            for (int q = 0; q < S; ++q) acc[j][q] = acc[j + 1][q];
#pragma unroll
        for (int q = 0; q < S; ++q) acc[NB - 1][q] = make_float2(0.f, 0.f);
#pragma unroll
        for (int m = 0; m < E - S; ++m) xin[m] = xin[m + S];
#pragma unroll
        for (int m = E - S; m < E; ++m) xin[m] = nxt[m];
    }
}

// ------------------------------------------------------------------ fused, two frames per wave
// K_fused2 k_stft_ola_fused2<E,S,NB>: K_fused with frames k and k+1 in flight
// per iteration (fft_wave2: shared twiddle/window/super-twiddle reads, one
// fence pair per exchange for both frames).  xin holds hops k..k+NB; the OLA
// adds frame k, emits block k, then adds frame k+1 -- the same ascending-k
// arithmetic, so results equal K_fused bit for bit.  Exact-rewrite numerics only.
template <int S, int E>
__device__ __forceinline__ void load_hop(float2* dst, __amdgpu_buffer_rsrc_t rx, int lane, int origin,
                                         int T, int mode) {
    constexpr int H = 128 * S;
    if (origin >= 0 && origin + H <= T) {
#pragma unroll
        for (int q = 0; q < S; ++q) dst[q] = dev::bload2(rx, lane * 8 + q * 512, origin * 4);
    } else {
#pragma unroll
        for (int q = 0; q < S; ++q) {
            const int j = origin + 2 * (lane + 64 * q);
            dst[q] = make_float2(fetch_x(rx, j, T, mode), fetch_x(rx, j + 1, T, mode));
        }
    }
}

#ifndef CRLOT_FUSED2_MIN_WAVES
#define CRLOT_FUSED2_MIN_WAVES 1
#endif
template <int E, int S, int NB, bool HAS_GAIN>
__global__ __launch_bounds__(kBlock, CRLOT_FUSED2_MIN_WAVES) void k_stft_ola_fused2(const FusedArgs a) {
    constexpr int P = 64 * E, N = 2 * P, H = 128 * S;
    static_assert(NB * S == E, "N = NB * H");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    cf* st = tw + P;
    cf* sth = st + P;
    float* wa = reinterpret_cast<float*>(sth + P);
    float* ws = wa + N;
    cf* bufs = reinterpret_cast<cf*>(ws + N);
    load_tables<E>(a.t, tw, st, sth, wa, ws, true, a.t.wsn);

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    cf* buf0 = bufs + wave * 2 * P;
    cf* buf1 = buf0 + P;
    const int gw = blockIdx.x * kWaves + wave;
    if (gw >= a.n_streams * a.n_chunks) return;
    const int s = gw / a.n_chunks, c = gw - s * a.n_chunks;
    const int f0 = c * a.M;
    const int f1 = min(a.F, f0 + a.M);
    const int fs = max(0, f0 - (NB - 1));
    const __amdgpu_buffer_rsrc_t rx = dev::make_rsrc(a.x + int64_t(s) * a.ld_x, uint32_t(a.T) * 4u);
    const __amdgpu_buffer_rsrc_t ry =
        dev::make_rsrc(a.y + int64_t(s) * a.ld_y, uint32_t(a.out_len) * 4u);
    const __amdgpu_buffer_rsrc_t rd = dev::make_rsrc(a.t.den, uint32_t(a.ring_blocks * H) * 4u);
    const __amdgpu_buffer_rsrc_t rr = dev::make_rsrc(a.t.rden, uint32_t(a.ring_blocks * H) * 4u);
    const float g = a.gain;

    // xin[h*S + q]: hop (k + h), pair q, h = 0..NB
    float2 xin[E + S];
#pragma unroll
    for (int h = 0; h <= NB; ++h) load_hop<S, E>(xin + h * S, rx, lane, (fs + h) * H - a.pad, a.T, a.pad_mode);
    float2 acc[NB][S];
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int q = 0; q < S; ++q) acc[j][q] = make_float2(0.f, 0.f);

    auto windowed = [&](cf (&v)[E], int off) {
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const float2 w = *reinterpret_cast<const float2*>(wa + 2 * (lane + 64 * m));
            v[m].r = dev::sanit(xin[off + m].x * w.x);
            v[m].i = dev::sanit(xin[off + m].y * w.y);
        }
    };
    auto accumulate = [&](const cf (&v)[E]) {
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const float2 w = *reinterpret_cast<const float2*>(ws + 2 * (lane + 64 * m));
            const float o0 = dev::sanit_scaled<N>(v[m].r);
            const float o1 = dev::sanit_scaled<N>(v[m].i);
            float2& r = acc[m / S][m % S];
            r.x = __builtin_fmaf(__builtin_fmaf(o0, w.x, 0.0f), g, r.x);
            r.y = __builtin_fmaf(__builtin_fmaf(o1, w.y, 0.0f), g, r.y);
        }
    };
    auto emit = [&](int k) {  // produce(H) of block k, then shift the accumulators
        if (k >= f0) {
            float2 dn[S], rn[S];
#pragma unroll
            for (int q = 0; q < S; ++q) {
                dn[q] = dev::bload2(rd, lane * 8 + q * 512, (k % a.ring_blocks) * H * 4);
                rn[q] = dev::bload2(rr, lane * 8 + q * 512, (k % a.ring_blocks) * H * 4);
            }
            bool ok = true;
#pragma unroll
            for (int q = 0; q < S; ++q) ok = ok && mk_ok(acc[0][q].x) && mk_ok(acc[0][q].y);
            const bool fast = __builtin_amdgcn_ballot_w64(!ok) == 0;
#pragma unroll
            for (int q = 0; q < S; ++q) {
                const float2 o = fast ? make_float2(mk_div(acc[0][q].x, dn[q].x, rn[q].x),
                                                    mk_div(acc[0][q].y, dn[q].y, rn[q].y))
                                      : make_float2(acc[0][q].x / dn[q].x, acc[0][q].y / dn[q].y);
                dev::bstore2(o, ry, lane * 8 + q * 512, k * H * 4);
            }
        }
#pragma unroll
        for (int j = 0; j < NB - 1; ++j)
#pragma unroll
            for (int q = 0; q < S; ++q) acc[j][q] = acc[j + 1][q];
#pragma unroll
        for (int q = 0; q < S; ++q) acc[NB - 1][q] = make_float2(0.f, 0.f);
    };

    int k = fs;
    for (; k + 1 < f1; k += 2) {
        // prefetch hops k+NB+1, k+NB+2 for the next pair
        float2 nxt[2 * S];
        load_hop<S, E>(nxt, rx, lane, (k + NB + 1) * H - a.pad, a.T, a.pad_mode);
        load_hop<S, E>(nxt + S, rx, lane, (k + NB + 2) * H - a.pad, a.T, a.pad_mode);
        cf v0[E], v1[E];
        windowed(v0, 0);
        windowed(v1, S);
        dev::fft_wave2<E, false>(v0, v1, buf0, buf1, tw, lane);
        dev::real_split_hook_merge2<E, HAS_GAIN>(v0, v1, buf0, buf1, st, sth, a.t.gain, lane);
        dev::fft_wave2<E, true>(v0, v1, buf0, buf1, tw, lane);
        accumulate(v0);
        emit(k);
        accumulate(v1);
        emit(k + 1);
#pragma unroll
        for (int m = 0; m < E - S; ++m) xin[m] = xin[m + 2 * S];
#pragma unroll
        for (int q = 0; q < 2 * S; ++q) xin[E - S + q] = nxt[q];
    }
    if (k < f1) {  // odd count: the last frame alone
        cf v0[E];
        windowed(v0, 0);
        dev::fft_wave<E, false>(v0, buf0, tw, lane);
        dev::real_split_hook_merge<E, HAS_GAIN, false>(v0, buf0, st, sth, a.t.gain, lane);
        dev::fft_wave<E, true>(v0, buf0, tw, lane);
        accumulate(v0);
        emit(k);
    }
}

// ------------------------------------------------------------------ fused, frame pairs (N = 512)
// K_pair512 k_stft_ola_pair512<SH,NB>: K_pair's walk for N = 512 (fft_pair512.h):
// frames 2j and 2j+1 of a stream in one 512-point complex transform per wave,
// lane l holding samples l + 64 m (m < 8); a hop is SH = H/64 floats per lane.
// Same regimes, OLA order, divisions and store rules as K_pair; twiddles and
// both windows in registers; one 4.6 KB LDS buffer per wave.
#ifndef CRLOT_P512_WAVES
#define CRLOT_P512_WAVES 4  // 2 waves: same time; 8 waves: -2 % (A/B at 1024 x 480000, 512/128)
#endif
constexpr int kP512Waves = CRLOT_P512_WAVES;
template <int SH, int NB, bool HAS_GAIN>
__global__ __launch_bounds__(64 * kP512Waves) void k_stft_ola_pair512(const FusedArgs a) {
    constexpr int E = 8, N = 512, H = 64 * SH;
    static_assert(NB * SH == E, "N = NB * H");
    static_assert(SH >= 2, "den rows are read 16 bytes at a time");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    dev::pc* buf = reinterpret_cast<dev::pc*>(smem) + wave * dev::kP512Buf;
    const int gw = blockIdx.x * kP512Waves + wave;
    if (gw >= a.n_streams * a.n_chunks) return;
    if (!a.fix_all && a.t.pflags[gw] == 0u) return;  // fix-up walker: flagged chunks only
    const int s = gw / a.n_chunks, c = gw - s * a.n_chunks;
    const int f0 = c * a.M;
    const int f1 = min(a.F, f0 + a.M);
    const int fs = max(0, f0 - (NB - 1)) & ~1;  // pairs start on even frames
    const __amdgpu_buffer_rsrc_t rx = dev::make_rsrc(a.x + int64_t(s) * a.ld_x, uint32_t(a.T) * 4u);
    const __amdgpu_buffer_rsrc_t ry =
        dev::make_rsrc(a.y + int64_t(s) * a.ld_y, uint32_t(a.out_len) * 4u);
    const __amdgpu_buffer_rsrc_t ry_null = dev::make_rsrc(a.y, 0u);
    const __amdgpu_buffer_rsrc_t rp = dev::make_rsrc(a.t.pden, uint32_t(a.ring_blocks * H) * 8u);
    const float xlo = a.t.px_lo, xhi = a.t.px_hi;

    dev::Pair512TwReg tw;
    dev::pair512_tw_load(tw, reinterpret_cast<const dev::pc*>(a.t.ptw), lane);
    float wa[E], ws[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        wa[m] = a.t.wa[lane + 64 * m];
        ws[m] = a.t.wsn[lane + 64 * m] * a.gain;  // (ws g: ola_pair.h ola_pair_push_w)
    }

    float xin[E + SH];
    uint32_t hopok = 0;
#pragma unroll
    for (int h = 0; h <= NB; ++h) {
        load_hop1<SH>(xin + h * SH, rx, lane, (fs + h) * H - a.pad, a.T, a.pad_mode);
        hopok |= hop_ok<SH>(xin + h * SH, xlo, xhi) << h;
    }
    float acc[NB][SH];
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int q = 0; q < SH; ++q) acc[j][q] = 0.f;

    auto accumulate = [&](const dev::pc (&v)[E], bool imag, bool paired) {
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const float x = imag ? v[m].y : v[m].x;
            const float o = paired ? dev::sanit_scaled_finite<N>(x) : dev::sanit_scaled<N>(x);
            float& r = acc[m / SH][m % SH];
            r = __builtin_fmaf(o, ws[m], r);  // (ws g: the hot walker's ola_pair_push_w)
        }
    };
    auto emit = [&](int k, const float (&dr)[2 * SH]) {  // produce(H) of block k, then shift
        float mx = 0.0f, mn = 0x1p127f;
#pragma unroll
        for (int q = 0; q < SH; ++q) {
            const float u = __builtin_fabsf(acc[0][q]);
            mx = __builtin_fmaxf(mx, u);
            mn = __builtin_fminf(mn, u);
        }
        const bool ok = (mx <= 0x1p64f) & ((mn >= 0x1p-64f) | (mx == 0.0f));
        float o[SH];
#pragma unroll
        for (int q = 0; q < SH; ++q) o[q] = mk_div(acc[0][q], dr[q], dr[SH + q]);
        if (__builtin_amdgcn_ballot_w64(!ok) != 0) {
#pragma unroll
            for (int q = 0; q < SH; ++q) o[q] = acc[0][q] / dr[q];
        }
        const __amdgpu_buffer_rsrc_t rk = k >= f0 ? ry : ry_null;
#pragma unroll
        for (int q = 0; q < SH; ++q)
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o[q]), rk, lane * 4,
                                                  k * (4 * H) + q * 256, 0);
#pragma unroll
        for (int j = 0; j < NB - 1; ++j)
#pragma unroll
            for (int q = 0; q < SH; ++q) acc[j][q] = acc[j + 1][q];
#pragma unroll
        for (int q = 0; q < SH; ++q) acc[NB - 1][q] = 0.f;
    };
    auto transform = [&](dev::pc (&v)[E]) {
        dev::pair512_fwd(v, buf, tw, lane);
        if constexpr (HAS_GAIN) {
#pragma unroll
            for (int d = 0; d < E; ++d) {
                const int kb = dev::pair512_bin(lane, d);
                v[d] = v[d] * a.t.gain[kb <= N / 2 ? kb : N - kb];
            }
        }
        dev::pair512_inv(v, buf, tw, lane);
    };

    constexpr uint32_t kPairHops = (1u << (NB + 1)) - 1;  // hops k .. k+NB
    for (int k = fs; k < f1; k += 2) {
        float nxt[2 * SH];
        load_hop1<SH>(nxt, rx, lane, (k + NB + 1) * H - a.pad, a.T, a.pad_mode);
        load_hop1<SH>(nxt + SH, rx, lane, (k + NB + 2) * H - a.pad, a.T, a.pad_mode);
        const bool paired = (hopok & kPairHops) == kPairHops;
        if (paired) {
            const bool partner = k + 1 < a.F;
            dev::pc v[E];
#pragma unroll
            for (int m = 0; m < E; ++m) v[m] = dev::pc_mk(xin[m] * wa[m], partner ? xin[m + SH] * wa[m] : 0.0f);
            transform(v);
            float dr0[2 * SH], dr1[2 * SH];
            load_den<SH>(dr0, rp, lane, k % a.ring_blocks);
            load_den<SH>(dr1, rp, lane, (k + 1) % a.ring_blocks);
            accumulate(v, false, true);
            emit(k, dr0);
            if (k + 1 < f1) {
                accumulate(v, true, true);
                emit(k + 1, dr1);
            }
        } else {  // unpaired: frames k and k+1 alone, full sanitize
            const int npass = min(2, f1 - k);
            for (int p = 0; p < npass; ++p) {
                dev::pc v[E];
#pragma unroll
                for (int m = 0; m < E; ++m)
                    v[m] = dev::pc_mk(dev::sanit((p ? xin[m + SH] : xin[m]) * wa[m]), 0.0f);
                transform(v);
                float dr[2 * SH];
                load_den<SH>(dr, rp, lane, (k + p) % a.ring_blocks);
                accumulate(v, false, false);
                emit(k + p, dr);
            }
        }
        hopok = (hopok | hop_ok<SH>(nxt, xlo, xhi) << (NB + 1) | hop_ok<SH>(nxt + SH, xlo, xhi) << (NB + 2)) >> 2;
#pragma unroll
        for (int m = 0; m < E + SH - 2 * SH; ++m) xin[m] = xin[m + 2 * SH];
#pragma unroll
        for (int q = 0; q < 2 * SH; ++q) xin[E - SH + q] = nxt[q];
    }
}

// ------------------------------------------------------------------ fused, frame pairs (N = 4096)
// K_pair4k k_stft_ola_pair4k<SH,NB>: K_pair's walk for N = 4096 by a 256-lane
// workgroup (fft_pair4k.h): frames 2j and 2j+1 of a stream in one 4096-point
// complex transform, lane t holding samples t + 256 m; a hop is SH = H/256
// floats per lane.  Same regimes, OLA order, divisions and store rules as
// K_pair; the regime of a pair is agreed by the whole workgroup
// (__syncthreads_or), since its transforms exchange data across the four waves.
template <int SH>
__device__ __forceinline__ void load_hop4k(float* dst, __amdgpu_buffer_rsrc_t rx, int t, int origin, int T,
                                           int mode) {
    constexpr int H = 256 * SH;
    if (origin >= 0 && origin + H <= T) {
#pragma unroll
        for (int q = 0; q < SH; ++q) dst[q] = dev::bload1(rx, t * 4, origin * 4 + q * 1024);
    } else {
#pragma unroll
        for (int q = 0; q < SH; ++q) dst[q] = fetch_x(rx, origin + t + 256 * q, T, mode);
    }
}
template <int SH>
__device__ __forceinline__ bool hop_bad(const float* h, float lo, float hi) {
    bool bad = false;
#pragma unroll
    for (int q = 0; q < SH; ++q) {
        const float a = __builtin_fabsf(h[q]);
        bad |= !((a >= lo) & (a <= hi)) & (a != 0.0f);
    }
    return bad;
}
// den | rden of block b for workgroup lane t (DevTables::pden: [block][256][den SH | rden SH])
template <int SH>
__device__ __forceinline__ void load_den4k(float (&dr)[2 * SH], __amdgpu_buffer_rsrc_t rp, int t, int b) {
#pragma unroll
    for (int j = 0; j < 2 * SH / 4; ++j) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rp, t * (8 * SH), b * (2048 * SH) + 16 * j, 0);
        const unsigned u0 = v[0], u1 = v[1], u2 = v[2], u3 = v[3];  // (see bload2)
        dr[4 * j] = __builtin_bit_cast(float, u0);
        dr[4 * j + 1] = __builtin_bit_cast(float, u1);
        dr[4 * j + 2] = __builtin_bit_cast(float, u2);
        dr[4 * j + 3] = __builtin_bit_cast(float, u3);
    }
}

constexpr size_t kPair4kLds = sizeof(cf) * (dev::kP4Xbuf + 4 * dev::kPairXbuf);

template <int SH, int NB, bool HAS_GAIN>
__global__ __launch_bounds__(256, 2) void k_stft_ola_pair4k(const FusedArgs a) {
    constexpr int E = 16, N = 4096, H = 256 * SH;
    static_assert(NB * SH == E, "N = NB * H");
    static_assert(SH >= 2, "den rows are read 16 bytes at a time");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    dev::pc* xb = reinterpret_cast<dev::pc*>(smem);
    const int t = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    dev::pc* qb = xb + dev::kP4Xbuf + wave * dev::kPairXbuf;

    // as the fix-up walker after k_stft_ola_pair4k_hot (pair_hot.hip): only the
    // chunks it flagged (uniform per workgroup, before any barrier)
    if (!a.fix_all && a.t.pflags[blockIdx.x] == 0u) return;
    const int s = blockIdx.x / a.n_chunks, c = blockIdx.x - s * a.n_chunks;
    const int f0 = c * a.M;
    const int f1 = min(a.F, f0 + a.M);
    const int fs = max(0, f0 - (NB - 1)) & ~1;  // pairs start on even frames
    const __amdgpu_buffer_rsrc_t rx = dev::make_rsrc(a.x + int64_t(s) * a.ld_x, uint32_t(a.T) * 4u);
    const __amdgpu_buffer_rsrc_t ry =
        dev::make_rsrc(a.y + int64_t(s) * a.ld_y, uint32_t(a.out_len) * 4u);
    const __amdgpu_buffer_rsrc_t ry_null = dev::make_rsrc(a.y, 0u);
    const __amdgpu_buffer_rsrc_t rp = dev::make_rsrc(a.t.pden4, uint32_t(a.ring_blocks * H) * 8u);
    const float xlo = a.t.px_lo, xhi = a.t.px_hi;

    dev::Pair4kTwFor<SH, HAS_GAIN> tw;
    dev::pair4k_tw_load(tw, reinterpret_cast<const dev::pc*>(a.t.ptw4), t);
    float wa[E], ws[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        wa[m] = a.t.wa[t + 256 * m];
        ws[m] = a.t.wsn[t + 256 * m] * a.gain;  // (ws g: ola_pair.h ola_pair_push_w)
    }

    // xin[h*SH + q]: hop (k + h), h = 0..NB; bit h of hopok: hop k + h keeps the paired regime
    float xin[E + SH];
    uint32_t hopok = 0;
#pragma unroll
    for (int h = 0; h <= NB; ++h) {
        load_hop4k<SH>(xin + h * SH, rx, t, (fs + h) * H - a.pad, a.T, a.pad_mode);
        hopok |= (__syncthreads_or(hop_bad<SH>(xin + h * SH, xlo, xhi)) ? 0u : 1u) << h;
    }
    float acc[NB][SH];
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int q = 0; q < SH; ++q) acc[j][q] = 0.f;

    auto accumulate = [&](const dev::pc (&v)[E], bool imag, bool paired) {
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const float x = imag ? v[m].y : v[m].x;
            const float o = paired ? dev::sanit_scaled_finite<N>(x) : dev::sanit_scaled<N>(x);
            float& r = acc[m / SH][m % SH];
            r = __builtin_fmaf(o, ws[m], r);  // (ws g: the hot walker's ola_pair_push_w)
        }
    };
    auto emit = [&](int k, const float (&dr)[2 * SH]) {  // produce(H) of block k, then shift
        float mx = 0.0f, mn = 0x1p127f;
#pragma unroll
        for (int q = 0; q < SH; ++q) {
            const float u = __builtin_fabsf(acc[0][q]);
            mx = __builtin_fmaxf(mx, u);
            mn = __builtin_fminf(mn, u);
        }
        const bool ok = (mx <= 0x1p64f) & ((mn >= 0x1p-64f) | (mx == 0.0f));
        float o[SH];
#pragma unroll
        for (int q = 0; q < SH; ++q) o[q] = mk_div(acc[0][q], dr[q], dr[SH + q]);
        if (__builtin_amdgcn_ballot_w64(!ok) != 0) {
#pragma unroll
            for (int q = 0; q < SH; ++q) o[q] = acc[0][q] / dr[q];
        }
        const __amdgpu_buffer_rsrc_t rk = k >= f0 ? ry : ry_null;
#pragma unroll
        for (int q = 0; q < SH; ++q)
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o[q]), rk, t * 4,
                                                  k * (4 * H) + q * 1024, 0);
#pragma unroll
        for (int j = 0; j < NB - 1; ++j)
#pragma unroll
            for (int q = 0; q < SH; ++q) acc[j][q] = acc[j + 1][q];
#pragma unroll
        for (int q = 0; q < SH; ++q) acc[NB - 1][q] = 0.f;
    };
    auto transform = [&](dev::pc (&v)[E]) {
        dev::pair4k_fwd(v, xb, qb, tw, t);
        if constexpr (HAS_GAIN) {
#pragma unroll
            for (int d = 0; d < E; ++d) {
                const int kb = dev::pair4k_bin(t, d);
                v[d] = v[d] * a.t.gain[kb <= N / 2 ? kb : N - kb];
            }
        }
        dev::pair4k_inv(v, xb, qb, tw, t);
    };

    constexpr uint32_t kPairHops = (1u << (NB + 1)) - 1;  // hops k .. k+NB
    for (int k = fs; k < f1; k += 2) {
        float nxt[2 * SH];
        load_hop4k<SH>(nxt, rx, t, (k + NB + 1) * H - a.pad, a.T, a.pad_mode);
        load_hop4k<SH>(nxt + SH, rx, t, (k + NB + 2) * H - a.pad, a.T, a.pad_mode);
        const bool paired = (hopok & kPairHops) == kPairHops;
        if (paired) {
            const bool partner = k + 1 < a.F;
            dev::pc v[E];
#pragma unroll
            for (int m = 0; m < E; ++m) v[m] = dev::pc_mk(xin[m] * wa[m], partner ? xin[m + SH] * wa[m] : 0.0f);
            transform(v);
            float dr0[2 * SH], dr1[2 * SH];
            load_den4k<SH>(dr0, rp, t, k % a.ring_blocks);
            load_den4k<SH>(dr1, rp, t, (k + 1) % a.ring_blocks);
            accumulate(v, false, true);
            emit(k, dr0);
            if (k + 1 < f1) {
                accumulate(v, true, true);
                emit(k + 1, dr1);
            }
        } else {  // unpaired: frames k and k+1 alone, full sanitize
            const int npass = min(2, f1 - k);
            for (int p = 0; p < npass; ++p) {
                dev::pc v[E];
#pragma unroll
                for (int m = 0; m < E; ++m)
                    v[m] = dev::pc_mk(dev::sanit((p ? xin[m + SH] : xin[m]) * wa[m]), 0.0f);
                transform(v);
                float dr[2 * SH];
                load_den4k<SH>(dr, rp, t, (k + p) % a.ring_blocks);
                accumulate(v, false, false);
                emit(k + p, dr);
            }
        }
        const uint32_t ok1 = __syncthreads_or(hop_bad<SH>(nxt, xlo, xhi)) ? 0u : 1u;
        const uint32_t ok2 = __syncthreads_or(hop_bad<SH>(nxt + SH, xlo, xhi)) ? 0u : 1u;
        hopok = (hopok | ok1 << (NB + 1) | ok2 << (NB + 2)) >> 2;
#pragma unroll
        for (int m = 0; m < E + SH - 2 * SH; ++m) xin[m] = xin[m + 2 * SH];
#pragma unroll
        for (int q = 0; q < 2 * SH; ++q) xin[E - SH + q] = nxt[q];
    }
}

// ------------------------------------------------------------------ fused, frame pairs (N = 2048)
// K_pair2k k_stft_ola_pair2k<SH,NB>: K_pair4k's walk for N = 2048 by a 128-lane
// workgroup (fft_pair2k.h), lane t holding samples t + 128 m; a hop is
// SH = H/128 floats per lane; tables in DevTables::ptw4 / pden4 (128 lanes).
template <int SH>
__device__ __forceinline__ void load_hop2k(float* dst, __amdgpu_buffer_rsrc_t rx, int t, int origin, int T,
                                           int mode) {
    constexpr int H = 128 * SH;
    if (origin >= 0 && origin + H <= T) {
#pragma unroll
        for (int q = 0; q < SH; ++q) dst[q] = dev::bload1(rx, t * 4, origin * 4 + q * 512);
    } else {
#pragma unroll
        for (int q = 0; q < SH; ++q) dst[q] = fetch_x(rx, origin + t + 128 * q, T, mode);
    }
}
template <int SH>
__device__ __forceinline__ void load_den2k(float (&dr)[2 * SH], __amdgpu_buffer_rsrc_t rp, int t, int b) {
#pragma unroll
    for (int j = 0; j < 2 * SH / 4; ++j) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rp, t * (8 * SH), b * (1024 * SH) + 16 * j, 0);
        const unsigned u0 = v[0], u1 = v[1], u2 = v[2], u3 = v[3];  // (see bload2)
        dr[4 * j] = __builtin_bit_cast(float, u0);
        dr[4 * j + 1] = __builtin_bit_cast(float, u1);
        dr[4 * j + 2] = __builtin_bit_cast(float, u2);
        dr[4 * j + 3] = __builtin_bit_cast(float, u3);
    }
}

constexpr size_t kPair2kLds = sizeof(cf) * (dev::kP2Xbuf + 2 * dev::kP2Tbuf);

template <int SH, int NB, bool HAS_GAIN>
__global__ __launch_bounds__(128, 2) void k_stft_ola_pair2k(const FusedArgs a) {
    constexpr int E = 16, N = 2048, H = 128 * SH;
    static_assert(NB * SH == E, "N = NB * H");
    static_assert(SH >= 2, "den rows are read 16 bytes at a time");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    dev::pc* xb = reinterpret_cast<dev::pc*>(smem);
    const int t = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    dev::pc* qb = xb + dev::kP2Xbuf + wave * dev::kP2Tbuf;

    // as the fix-up walker after the hot walker (pair_hot.hip): only the chunks it
    // flagged (uniform per workgroup, before any barrier)
    if (!a.fix_all && a.t.pflags[blockIdx.x] == 0u) return;
    const int s = blockIdx.x / a.n_chunks, c = blockIdx.x - s * a.n_chunks;
    const int f0 = c * a.M;
    const int f1 = min(a.F, f0 + a.M);
    const int fs = max(0, f0 - (NB - 1)) & ~1;  // pairs start on even frames
    const __amdgpu_buffer_rsrc_t rx = dev::make_rsrc(a.x + int64_t(s) * a.ld_x, uint32_t(a.T) * 4u);
    const __amdgpu_buffer_rsrc_t ry =
        dev::make_rsrc(a.y + int64_t(s) * a.ld_y, uint32_t(a.out_len) * 4u);
    const __amdgpu_buffer_rsrc_t ry_null = dev::make_rsrc(a.y, 0u);
    const __amdgpu_buffer_rsrc_t rp = dev::make_rsrc(a.t.pden4, uint32_t(a.ring_blocks * H) * 8u);
    const float xlo = a.t.px_lo, xhi = a.t.px_hi;

    dev::Pair2kTwFor<SH, HAS_GAIN> tw;
    dev::pair2k_tw_load(tw, reinterpret_cast<const dev::pc*>(a.t.ptw4), t);
    float wa[E], ws[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        wa[m] = a.t.wa[t + 128 * m];
        ws[m] = a.t.wsn[t + 128 * m] * a.gain;  // (ws g: ola_pair.h ola_pair_push_w)
    }

    // xin[h*SH + q]: hop (k + h), h = 0..NB; bit h of hopok: hop k + h keeps the paired regime
    float xin[E + SH];
    uint32_t hopok = 0;
#pragma unroll
    for (int h = 0; h <= NB; ++h) {
        load_hop2k<SH>(xin + h * SH, rx, t, (fs + h) * H - a.pad, a.T, a.pad_mode);
        hopok |= (__syncthreads_or(hop_bad<SH>(xin + h * SH, xlo, xhi)) ? 0u : 1u) << h;
    }
    float acc[NB][SH];
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int q = 0; q < SH; ++q) acc[j][q] = 0.f;

    auto accumulate = [&](const dev::pc (&v)[E], bool imag, bool paired) {
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const float x = imag ? v[m].y : v[m].x;
            const float o = paired ? dev::sanit_scaled_finite<N>(x) : dev::sanit_scaled<N>(x);
            float& r = acc[m / SH][m % SH];
            r = __builtin_fmaf(o, ws[m], r);  // (ws g: the hot walker's ola_pair_push_w)
        }
    };
    auto emit = [&](int k, const float (&dr)[2 * SH]) {  // produce(H) of block k, then shift
        float mx = 0.0f, mn = 0x1p127f;
#pragma unroll
        for (int q = 0; q < SH; ++q) {
            const float u = __builtin_fabsf(acc[0][q]);
            mx = __builtin_fmaxf(mx, u);
            mn = __builtin_fminf(mn, u);
        }
        const bool ok = (mx <= 0x1p64f) & ((mn >= 0x1p-64f) | (mx == 0.0f));
        float o[SH];
#pragma unroll
        for (int q = 0; q < SH; ++q) o[q] = mk_div(acc[0][q], dr[q], dr[SH + q]);
        if (__builtin_amdgcn_ballot_w64(!ok) != 0) {
#pragma unroll
            for (int q = 0; q < SH; ++q) o[q] = acc[0][q] / dr[q];
        }
        const __amdgpu_buffer_rsrc_t rk = k >= f0 ? ry : ry_null;
#pragma unroll
        for (int q = 0; q < SH; ++q)
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o[q]), rk, t * 4,
                                                  k * (4 * H) + q * 512, 0);
#pragma unroll
        for (int j = 0; j < NB - 1; ++j)
#pragma unroll
            for (int q = 0; q < SH; ++q) acc[j][q] = acc[j + 1][q];
#pragma unroll
        for (int q = 0; q < SH; ++q) acc[NB - 1][q] = 0.f;
    };
    auto transform = [&](dev::pc (&v)[E]) {
        dev::pair2k_fwd(v, xb, qb, tw, t);
        if constexpr (HAS_GAIN) {
#pragma unroll
            for (int d = 0; d < E; ++d) {
                const int kb = dev::pair2k_bin(t, d);
                v[d] = v[d] * a.t.gain[kb <= N / 2 ? kb : N - kb];
            }
        }
        dev::pair2k_inv(v, xb, qb, tw, t);
    };

    constexpr uint32_t kPairHops = (1u << (NB + 1)) - 1;  // hops k .. k+NB
    for (int k = fs; k < f1; k += 2) {
        float nxt[2 * SH];
        load_hop2k<SH>(nxt, rx, t, (k + NB + 1) * H - a.pad, a.T, a.pad_mode);
        load_hop2k<SH>(nxt + SH, rx, t, (k + NB + 2) * H - a.pad, a.T, a.pad_mode);
        const bool paired = (hopok & kPairHops) == kPairHops;
        if (paired) {
            const bool partner = k + 1 < a.F;
            dev::pc v[E];
#pragma unroll
            for (int m = 0; m < E; ++m) v[m] = dev::pc_mk(xin[m] * wa[m], partner ? xin[m + SH] * wa[m] : 0.0f);
            transform(v);
            float dr0[2 * SH], dr1[2 * SH];
            load_den2k<SH>(dr0, rp, t, k % a.ring_blocks);
            load_den2k<SH>(dr1, rp, t, (k + 1) % a.ring_blocks);
            accumulate(v, false, true);
            emit(k, dr0);
            if (k + 1 < f1) {
                accumulate(v, true, true);
                emit(k + 1, dr1);
            }
        } else {  // unpaired: frames k and k+1 alone, full sanitize
            const int npass = min(2, f1 - k);
            for (int p = 0; p < npass; ++p) {
                dev::pc v[E];
#pragma unroll
                for (int m = 0; m < E; ++m)
                    v[m] = dev::pc_mk(dev::sanit((p ? xin[m + SH] : xin[m]) * wa[m]), 0.0f);
                transform(v);
                float dr[2 * SH];
                load_den2k<SH>(dr, rp, t, (k + p) % a.ring_blocks);
                accumulate(v, false, false);
                emit(k + p, dr);
            }
        }
        const uint32_t ok1 = __syncthreads_or(hop_bad<SH>(nxt, xlo, xhi)) ? 0u : 1u;
        const uint32_t ok2 = __syncthreads_or(hop_bad<SH>(nxt + SH, xlo, xhi)) ? 0u : 1u;
        hopok = (hopok | ok1 << (NB + 1) | ok2 << (NB + 2)) >> 2;
#pragma unroll
        for (int m = 0; m < E + SH - 2 * SH; ++m) xin[m] = xin[m + 2 * SH];
#pragma unroll
        for (int q = 0; q < 2 * SH; ++q) xin[E - SH + q] = nxt[q];
    }
}

// ------------------------------------------------------------------ fused, workgroup walker
// K_fused_wg k_stft_ola_wg<L,S,NB>: the fused walk of K_fused for frames too big
// for one wave (N = 16 L, E = 8): a workgroup of L lanes owns a run of frames
// of one stream, lane t holding z[t + L m].  The frame-invariant tables
// (analysis/synthesis window, super-twiddles, pass twiddles) sit in registers,
// so LDS holds only the three exchange buffers (A/B alternate through the FFT
// passes, C for the split); each exchange costs one s_barrier.
template <int L, int S, int NB, bool HAS_GAIN>
__global__ __launch_bounds__(L) void k_stft_ola_wg(const FusedArgs a) {
    constexpr int E = 8, P = L * E, H = 2 * L * S;
    static_assert(NB * S == E, "N = NB * H");
    constexpr int NX = dev::fft_exchanges(P, E);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cf* bufA = reinterpret_cast<cf*>(smem);
    cf* bufB = bufA + P;
    cf* bufC = bufB + P;

    const int t = threadIdx.x;
    const int s = blockIdx.x / a.n_chunks, c = blockIdx.x - s * a.n_chunks;
    const int f0 = c * a.M;
    const int f1 = min(a.F, f0 + a.M);
    const int fs = max(0, f0 - (NB - 1));
    const __amdgpu_buffer_rsrc_t rx = dev::make_rsrc(a.x + int64_t(s) * a.ld_x, uint32_t(a.T) * 4u);
    const __amdgpu_buffer_rsrc_t ry =
        dev::make_rsrc(a.y + int64_t(s) * a.ld_y, uint32_t(a.out_len) * 4u);
    const __amdgpu_buffer_rsrc_t rd = dev::make_rsrc(a.t.den, uint32_t(a.ring_blocks * H) * 4u);
    const float g = a.gain;

    dev::TwChainWg<E, L, 1> twc;
    dev::load_chain_wg<E, L, 1, 0>(twc, reinterpret_cast<const cf*>(a.t.tw), t);
    float2 wa[E], ws[E];
    cf st[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        wa[m] = *reinterpret_cast<const float2*>(a.t.wa + 2 * (t + L * m));
        ws[m] = *reinterpret_cast<const float2*>(a.t.ws + 2 * (t + L * m));
        st[m] = reinterpret_cast<const cf*>(a.t.st)[t + L * m];
    }

    float2 xin[E];
    load_pairs_l<0, E, E, L>(xin, rx, t, fs * H - a.pad, a.T, a.pad_mode);
    float2 acc[NB][S];
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int q = 0; q < S; ++q) acc[j][q] = make_float2(0.f, 0.f);

    for (int k = fs; k < f1; ++k) {
        float2 nxt[E];
        if (k + 1 < f1) load_pairs_l<E - S, S, E, L>(nxt, rx, t, (k + 1) * H - a.pad, a.T, a.pad_mode);
        float2 dn[S];
        if (k >= f0) {
#pragma unroll
            for (int q = 0; q < S; ++q)
                dn[q] = dev::bload2(rd, t * 8 + q * 8 * L, (k % a.ring_blocks) * H * 4);
        }
        cf v[E];
#pragma unroll
        for (int m = 0; m < E; ++m) {
            v[m].r = dev::sanit(xin[m].x * wa[m].x);
            v[m].i = dev::sanit(xin[m].y * wa[m].y);
        }
        dev::fft_passes_wg<E, L, 1, 0, false>(v, bufA, bufB, twc, t);
        dev::real_split_hook_merge_wg<E, L, HAS_GAIN>(v, bufC, st, a.t.gain, t);
        dev::fft_passes_wg<E, L, 1, (NX & 1), true>(v, bufA, bufB, twc, t);
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const float o0 = dev::sanit(v[m].r * a.inv_n);
            const float o1 = dev::sanit(v[m].i * a.inv_n);
            float2& r = acc[m / S][m % S];
            r.x = __builtin_fmaf(__builtin_fmaf(o0, ws[m].x, 0.0f), g, r.x);
            r.y = __builtin_fmaf(__builtin_fmaf(o1, ws[m].y, 0.0f), g, r.y);
        }
        if (k >= f0) {
#pragma unroll
            for (int q = 0; q < S; ++q)
                dev::bstore2(make_float2(acc[0][q].x / dn[q].x, acc[0][q].y / dn[q].y), ry,
                             t * 8 + q * 8 * L, k * H * 4);
        }
#pragma unroll
        for (int j = 0; j < NB - 1; ++j)
#pragma unroll
            for (int q = 0; q < S; ++q) acc[j][q] = acc[j + 1][q];
#pragma unroll
        for (int q = 0; q < S; ++q) acc[NB - 1][q] = make_float2(0.f, 0.f);
#pragma unroll
        for (int m = 0; m < E - S; ++m) xin[m] = xin[m + S];
#pragma unroll
        for (int m = E - S; m < E; ++m) xin[m] = nxt[m];
    }
}

// ------------------------------------------------------------------ staged
struct SynthArgs {
    DevTables t;
    const float* x;
    float* frames;  // [s][k][N]
    float* spec;    // [s][k][P+1] cf, optional
    int64_t ld_x, T, F;
    int h, n_streams, pad, pad_mode;
    float inv_n;
};

template <int E, bool HAS_GAIN, bool SPEC>
__global__ __launch_bounds__(kBlock) void k_synth_frames(const SynthArgs a) {
    constexpr int P = 64 * E, N = 2 * P;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    cf* st = tw + P;
    cf* sth = st + P;
    float* wa = reinterpret_cast<float*>(sth + P);
    float* ws = wa + N;
    cf* bufs = reinterpret_cast<cf*>(ws + N);
    load_tables<E>(a.t, tw, st, sth, wa, ws, true);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    cf* buf = bufs + wave * xbuf_elems<P>();
    const int64_t gw = int64_t(blockIdx.x) * kWaves + wave;
    if (gw >= int64_t(a.n_streams) * a.F) return;
    const int64_t s = gw / a.F, k = gw % a.F;
    const float* x = a.x + s * a.ld_x;
    const int64_t base = k * a.h - a.pad;
    const bool inside = base >= 0 && base + N <= a.T;
    cf v[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const int i0 = 2 * (lane + 64 * m);
        const int64_t t0 = base + i0;
        float x0, x1;
        if (inside) {
            x0 = x[t0];
            x1 = x[t0 + 1];
        } else {
            x0 = fetch_x64(x, t0, a.T, a.pad_mode);
            x1 = fetch_x64(x, t0 + 1, a.T, a.pad_mode);
        }
        v[m].r = dev::sanit(x0 * wa[i0]);
        v[m].i = dev::sanit(x1 * wa[i0 + 1]);
    }
    dev::fft_wave<E, false>(v, buf, tw, lane);
    cf* spec = SPEC ? reinterpret_cast<cf*>(a.spec) + gw * (P + 1) : nullptr;
    dev::real_split_hook_merge<E, HAS_GAIN, SPEC>(v, buf, st, sth, a.t.gain, lane, spec);
    dev::fft_wave<E, true>(v, buf, tw, lane);
    float* out = a.frames + gw * N;
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const int i0 = 2 * (lane + 64 * m);
        *reinterpret_cast<float2*>(out + i0) =
            make_float2(dev::sanit(v[m].r * a.inv_n), dev::sanit(v[m].i * a.inv_n));
    }
}

struct GatherArgs {
    const float* frames;
    const float* ws;
    const float* den;
    float* y;
    int64_t ld_frames, ld_y, F, out_len;
    int n, h, ring_len, n_streams;
    float gain;
};

__global__ __launch_bounds__(256) void k_ola_gather(const GatherArgs a) {
    const int64_t idx = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const int64_t total = int64_t(a.n_streams) * a.out_len;
    if (idx >= total) return;
    const int64_t s = idx / a.out_len, n = idx % a.out_len;
    // frames k with k*H <= n < k*H + N, ascending
    int64_t kmax = n / a.h;
    if (kmax > a.F - 1) kmax = a.F - 1;
    int64_t kmin = n - a.n + 1 <= 0 ? 0 : (n - a.n + a.h) / a.h;
    const float* fr = a.frames + s * a.F * a.ld_frames;
    float acc = 0.0f;
    for (int64_t k = kmin; k <= kmax; ++k) {
        const int64_t off = n - k * a.h;
        const float src = fr[k * a.ld_frames + off];
        acc = __builtin_fmaf(__builtin_fmaf(src, a.ws[off], 0.0f), a.gain, acc);
    }
    const float d = a.den[n % a.ring_len];
    a.y[s * a.ld_y + n] = acc / d;
}

// The ring a push-everything-first loop leaves (bench/performance_benchmark.cc
// :212-231 pushes every frame, then produces): positions n and n + R share ring
// slot n (RingBuffer::split wraps, OLAAccumulator.cc:86-107), and since R > N
// the frames reaching n all precede the ones reaching n + R.  So slot p's sum is
// k_ola_gather's chain over position p continued over p + R, p + 2R, ..., in
// ascending frame order as the adds arrived.  acc[p]: the slot (what the ring
// holds), y[p]: the produce of it (acc / den[p]).  frames: F frames at hops from
// position 0, len = F h + max(0, N - h) positions.
__device__ __forceinline__ float gather_chain(const GatherArgs& a, int64_t n, float acc) {
    int64_t kmax = n / a.h;
    if (kmax > a.F - 1) kmax = a.F - 1;
    const int64_t kmin = n - a.n + 1 <= 0 ? 0 : (n - a.n + a.h) / a.h;
    for (int64_t k = kmin; k <= kmax; ++k) {
        const int64_t off = n - k * a.h;
        acc = __builtin_fmaf(__builtin_fmaf(a.frames[k * a.ld_frames + off], a.ws[off], 0.0f), a.gain, acc);
    }
    return acc;
}

// y_len > 0: threads [0, y_len) first give k_ola_gather's produce blocks into
// a.y (the same chain and division), the next R threads the wrapped slots into
// acc_out / ya -- both overlap-adds of a batch in one launch
__global__ __launch_bounds__(256) void k_ola_gather_wrap(const GatherArgs a, float* __restrict__ acc_out,
                                                         float* ya, int64_t len, int64_t y_len) {
    int64_t p = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (p < y_len) {
        a.y[p] = gather_chain(a, p, 0.0f) / a.den[p % a.ring_len];
        return;
    }
    p -= y_len;
    if (p >= a.ring_len) return;
    float acc = 0.0f;
    for (int64_t n = p; n < len; n += a.ring_len) acc = gather_chain(a, n, acc);
    acc_out[p] = acc;
    ya[p] = acc / a.den[p];
}

// The same arithmetic with a (sample block, stream) grid and no 64-bit
// division: each 256-sample block's first sample n0 is split by h and ring_len
// once (uniform), each thread finishes its quotient in float with one
// correction and counts its frames down; it requests the frame samples,
// windows and divisor of V outputs before summing any (memory-level
// parallelism), then sums the frames in ascending k as above.
template <int V, int SL>  // V outputs per thread, 256 apart, up to SL frames each in registers
__global__ __launch_bounds__(256) void k_ola_gather2(const GatherArgs a) {
    const int64_t s = blockIdx.y;
    const int h = a.h, N = a.n;
    const float* fr = a.frames + s * a.F * a.ld_frames;
    float src[V][SL], w[V][SL], dv[V];
    int cnt[V], nn[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int n0 = (int(blockIdx.x) * V + v) * 256;
        const int n = n0 + int(threadIdx.x);
        nn[v] = n;
        cnt[v] = 0;
        dv[v] = 1.0f;
        if (n >= a.out_len) continue;
        const int q0 = n0 / h, r0 = n0 - q0 * h;
        const int r1 = r0 + int(threadIdx.x);            // < h + 256 < 2^24: exact in float
        int q = int(float(r1) * (1.0f / float(h)));      // within one of r1 / h
        if (q * h > r1) --q;
        else if ((q + 1) * h <= r1) ++q;
        const int kq = q0 + q, r = r1 - q * h;           // n = kq h + r
        int nf = 1;                                      // frames k = kq - j with j h < N - r
        while (nf * h < N - r) ++nf;
        const int kmax = min(kq, int(a.F) - 1);
        const int kmin = max(0, kq - nf + 1);
        cnt[v] = kmax - kmin + 1;
        int d = n0 % a.ring_len + int(threadIdx.x);
        while (d >= a.ring_len) d -= a.ring_len;
        dv[v] = a.den[d];
        if (cnt[v] > SL) continue;  // more frames: the loop below
#pragma unroll
        for (int j = 0; j < SL; ++j) {
            const int k = kmin + j, off = n - k * h;
            src[v][j] = j < cnt[v] ? fr[int64_t(k) * a.ld_frames + off] : 0.0f;
            w[v][j] = j < cnt[v] ? a.ws[off] : 0.0f;
        }
    }
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int n = nn[v];
        if (n >= a.out_len) continue;
        float acc = 0.0f;
        if (cnt[v] <= SL) {
#pragma unroll
            for (int j = 0; j < SL; ++j)
                if (j < cnt[v]) acc = __builtin_fmaf(__builtin_fmaf(src[v][j], w[v][j], 0.0f), a.gain, acc);
        } else {
            const int kmax = min(n / h, int(a.F) - 1);
            for (int k = kmax - cnt[v] + 1; k <= kmax; ++k) {
                const int off = n - k * h;
                acc = __builtin_fmaf(__builtin_fmaf(fr[int64_t(k) * a.ld_frames + off], a.ws[off], 0.0f), a.gain, acc);
            }
        }
        a.y[s * a.ld_y + n] = acc / dv[v];
    }
}

// One workgroup per (output block b of H samples, stream): the block's
// frames are k = b-nb+1 .. b (nb = ceil(N/H)), frame k's samples for it a
// contiguous run at (b-k) H, so a thread's offsets need no division.  Every
// frame sample, window tap and the divisor are requested before the sum, which
// runs in ascending k exactly as k_ola_gather's.
template <int MAXNB>
__global__ __launch_bounds__(256) void k_ola_gather_blk(const GatherArgs a, int bpb) {
    const int64_t s = blockIdx.y;
    const int h = a.h, N = a.n;
    const int nb = (N + h - 1) / h;
    const float* fr = a.frames + s * a.F * a.ld_frames;
    const int b1 = int(min<int64_t>(a.F, int64_t(blockIdx.x + 1) * bpb));
    for (int b = int(blockIdx.x) * bpb; b < b1; ++b) {  // bpb blocks per workgroup (short hops)
    const int kmin = max(0, b - nb + 1), kmax = min(b, int(a.F) - 1);
    const int dbase = int(int64_t(b) * h % a.ring_len);
    float* yo = a.y + s * a.ld_y + int64_t(b) * h;
    for (int j = int(threadIdx.x); j < h; j += int(blockDim.x)) {
        if (int64_t(b) * h + j >= a.out_len) break;
        int d = dbase + j;
        d = d >= a.ring_len ? d - a.ring_len : d;
        const float dv = a.den[d];
        float acc = 0.0f;
        if (kmax - kmin + 1 <= MAXNB) {
            float src[MAXNB], w[MAXNB];
#pragma unroll
            for (int i = 0; i < MAXNB; ++i) {
                const int k = kmin + i, off = (b - k) * h + j;
                const bool in = k <= kmax && off < N;
                src[i] = in ? fr[int64_t(k) * a.ld_frames + off] : 0.0f;
                w[i] = in ? a.ws[off] : 0.0f;
            }
#pragma unroll
            for (int i = 0; i < MAXNB; ++i) {
                const int k = kmin + i, off = (b - k) * h + j;
                if (k <= kmax && off < N) acc = __builtin_fmaf(__builtin_fmaf(src[i], w[i], 0.0f), a.gain, acc);
            }
        } else {
            for (int k = kmin; k <= kmax; ++k) {
                const int off = (b - k) * h + j;
                if (off < N) acc = __builtin_fmaf(__builtin_fmaf(fr[int64_t(k) * a.ld_frames + off], a.ws[off], 0.0f), a.gain, acc);
            }
        }
        yo[j] = acc / dv;
    }
    }
}

// ------------------------------------------------------------------ rfft / irfft
struct FftArgs {
    DevTables t;
    const float* in;
    float* out;
    int64_t ld_in, inc_in, ld_out, inc_out;
    int batch;
    float inv_n;
};

template <int E>
__global__ __launch_bounds__(kBlock) void k_rfft(const FftArgs a) {
    constexpr int P = 64 * E;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    cf* st = tw + P;
    cf* sth = st + P;
    cf* bufs = sth + P;
    load_tables<E>(a.t, tw, st, sth, nullptr, nullptr, false);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    cf* buf = bufs + wave * xbuf_elems<P>();
    const int64_t b = int64_t(blockIdx.x) * kWaves + wave;
    if (b >= a.batch) return;
    const float* in = a.in + b * a.ld_in;
    cf v[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const int64_t i0 = 2 * (lane + 64 * m);
        v[m].r = dev::sanit(in[i0 * a.inc_in]);
        v[m].i = dev::sanit(in[(i0 + 1) * a.inc_in]);
    }
    dev::fft_wave<E, false>(v, buf, tw, lane);
    // split only (kiss_fftr): X[k] for own k, X[P] from k == 0
#pragma unroll
    for (int m = 0; m < E; ++m) buf[lane + 64 * m] = v[m];
    dev::wave_lds_fence();
    float* out = a.out + b * a.ld_out;
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const int k = lane + 64 * m;
        const cf zk = v[m];
        const cf fpnk = dev::conj(buf[(P - k) & (P - 1)]);
        const cf f1 = dev::cadd(zk, fpnk);
        const cf f2 = dev::csub(zk, fpnk);
        const cf t = dev::cmul(f2, sth[k]);
        cf xk = {__builtin_fmaf(f1.r, 0.5f, t.r), __builtin_fmaf(f1.i, 0.5f, t.i)}, xp;
        if (k == 0) dev::dc_split(zk, xk, xp);
        out[int64_t(2 * k) * a.inc_out] = xk.r;
        out[int64_t(2 * k) * a.inc_out + 1] = xk.i;
        if (k == 0) {
            out[int64_t(2 * P) * a.inc_out] = xp.r;
            out[int64_t(2 * P) * a.inc_out + 1] = xp.i;
        }
    }
}

template <int E>
__global__ __launch_bounds__(kBlock) void k_irfft(const FftArgs a) {
    constexpr int P = 64 * E;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    cf* st = tw + P;
    cf* sth = st + P;
    cf* bufs = sth + P;
    load_tables<E>(a.t, tw, st, sth, nullptr, nullptr, false);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    cf* buf = bufs + wave * xbuf_elems<P>();
    const int64_t b = int64_t(blockIdx.x) * kWaves + wave;
    if (b >= a.batch) return;
    const float* in = a.in + b * a.ld_in;
    cf v[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const int k = lane + 64 * m;
        const cf xk = {in[int64_t(2 * k) * a.inc_in], in[int64_t(2 * k) * a.inc_in + 1]};
        const int pk = P - k;
        const cf xpk = {in[int64_t(2 * pk) * a.inc_in], in[int64_t(2 * pk) * a.inc_in + 1]};
        const cf w = st[k];
        const cf fek = {xk.r + xpk.r, xk.i - xpk.i};
        const cf tmp = {xk.r - xpk.r, xk.i + xpk.i};
        v[m].r = __builtin_fmaf(tmp.r, w.r, __builtin_fmaf(tmp.i, w.i, fek.r));
        v[m].i = __builtin_fmaf(tmp.i, w.r, __builtin_fmaf(-tmp.r, w.i, fek.i));
        if (k == 0) v[m] = dev::dc_merge(xk, xpk);
    }
    dev::fft_wave<E, true>(v, buf, tw, lane);
    float* out = a.out + b * a.ld_out;
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const int64_t i0 = 2 * (lane + 64 * m);
        out[i0 * a.inc_out] = dev::sanit(v[m].r * a.inv_n);
        out[(i0 + 1) * a.inc_out] = dev::sanit(v[m].i * a.inv_n);
    }
}

// The batched speculation's forward and inverse in one launch (batch.cpp
// run_chain): K_rfft's arithmetic to the spectrum -- written out, and handed
// through LDS to K_irfft's arithmetic -- so the bits of both kernels with one
// dependent launch less.  r_host (nullable): a second copy of the inverse
// frames, e.g. in host-mapped memory.
template <int E>
__global__ __launch_bounds__(kBlock) void k_rfft_irfft(const FftArgs a, float* __restrict__ r, float* r_host,
                                                       int64_t ld_r) {
    constexpr int P = 64 * E;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    cf* st = tw + P;
    cf* sth = st + P;
    cf* bufs = sth + P;
    load_tables<E>(a.t, tw, st, sth, nullptr, nullptr, false);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    cf* buf = bufs + wave * xbuf_elems<P>();
    cf* xs = bufs + kWaves * xbuf_elems<P>() + wave * (P + 1);  // the spectrum, X[0 .. P]
    const int64_t b = int64_t(blockIdx.x) * kWaves + wave;
    if (b >= a.batch) return;
    const float* in = a.in + b * a.ld_in;
    cf v[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const int64_t i0 = 2 * (lane + 64 * m);
        v[m].r = dev::sanit(in[i0]);
        v[m].i = dev::sanit(in[i0 + 1]);
    }
    dev::fft_wave<E, false>(v, buf, tw, lane);
#pragma unroll
    for (int m = 0; m < E; ++m) buf[lane + 64 * m] = v[m];
    dev::wave_lds_fence();
    float* out = a.out + b * a.ld_out;
#pragma unroll
    for (int m = 0; m < E; ++m) {  // (k_rfft's split)
        const int k = lane + 64 * m;
        const cf zk = v[m];
        const cf fpnk = dev::conj(buf[(P - k) & (P - 1)]);
        const cf f1 = dev::cadd(zk, fpnk);
        const cf f2 = dev::csub(zk, fpnk);
        const cf t = dev::cmul(f2, sth[k]);
        cf xk = {__builtin_fmaf(f1.r, 0.5f, t.r), __builtin_fmaf(f1.i, 0.5f, t.i)}, xp;
        if (k == 0) dev::dc_split(zk, xk, xp);
        out[2 * k] = xk.r;
        out[2 * k + 1] = xk.i;
        xs[k] = xk;
        if (k == 0) {
            out[2 * P] = xp.r;
            out[2 * P + 1] = xp.i;
            xs[P] = xp;
        }
    }
    dev::wave_lds_fence();
#pragma unroll
    for (int m = 0; m < E; ++m) {  // (k_irfft's merge)
        const int k = lane + 64 * m;
        const cf xk = xs[k];
        const cf xpk = xs[P - k];
        const cf w = st[k];
        const cf fek = {xk.r + xpk.r, xk.i - xpk.i};
        const cf tmp = {xk.r - xpk.r, xk.i + xpk.i};
        v[m].r = __builtin_fmaf(tmp.r, w.r, __builtin_fmaf(tmp.i, w.i, fek.r));
        v[m].i = __builtin_fmaf(tmp.i, w.r, __builtin_fmaf(-tmp.r, w.i, fek.i));
        if (k == 0) v[m] = dev::dc_merge(xk, xpk);
    }
    dev::fft_wave<E, true>(v, buf, tw, lane);
    float* ro = r + b * ld_r;
    float* rh = r_host ? r_host + b * ld_r : nullptr;
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const int64_t i0 = 2 * (lane + 64 * m);
        const float2 q = make_float2(dev::sanit(v[m].r * a.inv_n), dev::sanit(v[m].i * a.inv_n));
        *reinterpret_cast<float2*>(ro + i0) = q;
        if (rh) *reinterpret_cast<float2*>(rh + i0) = q;
    }
}

// ------------------------------------------------------------------ complex FFT
// Batched IFftPlan::forward_complex / inverse_complex (kissfft_adapter.cc:171-246)
// of P = 64 E points: forward is the plain unnormalised DFT (no sanitize);
// inverse is the +i DFT, then *1/P and sanitize.  Element i of batch b is the
// float pair at [b*ld + 2*i*inc].
template <int E, bool INV>
__global__ __launch_bounds__(kBlock) void k_cfft(const FftArgs a) {
    constexpr int P = 64 * E;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    cf* st = tw + P;
    cf* sth = st + P;
    cf* bufs = sth + P;
    load_tables<E>(a.t, tw, st, sth, nullptr, nullptr, false);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    cf* buf = bufs + wave * xbuf_elems<P>();
    const int64_t b = int64_t(blockIdx.x) * kWaves + wave;
    if (b >= a.batch) return;
    const float* in = a.in + b * a.ld_in;
    cf v[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const int64_t i = lane + 64 * m;
        v[m] = {in[2 * i * a.inc_in], in[2 * i * a.inc_in + 1]};
    }
    dev::fft_wave<E, INV>(v, buf, tw, lane);
    float* out = a.out + b * a.ld_out;
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const int64_t i = lane + 64 * m;
        if constexpr (INV) {
            out[2 * i * a.inc_out] = dev::sanit(v[m].r * a.inv_n);
            out[2 * i * a.inc_out + 1] = dev::sanit(v[m].i * a.inv_n);
        } else {
            out[2 * i * a.inc_out] = v[m].r;
            out[2 * i * a.inc_out + 1] = v[m].i;
        }
    }
}

// ------------------------------------------------------------------ any size
// General-size path (fft_any.h): one wave per frame / transform, two LDS
// buffers of P elements per wave, tables read from global memory (L1/L2).
struct AnyArgs {
    DevTables t;
    const float* twany;  // W_P^k, k < P
    dev::any::Plan pl;
    const float* in;
    float* out;
    float* spec;
    int64_t ld_in, inc_in, ld_out, inc_out;  // FFT kernels
    int64_t T, F;                            // synth kernel
    int h, n_streams, batch, pad, pad_mode, waves_per_block;
    int tw_len;  // float pairs in twany
    float inv_n;
};

// LDS of the any-size kernels: [tw tw_len cf][st P cf][wa 2P f][per wave: 2 x P cf]
struct AnyLds {
    cf* tw;
    cf* st;
    float* wa;
    cf* A;
    cf* B;
};

template <bool LDS_TABLES>
__device__ __forceinline__ AnyLds any_lds(const AnyArgs& a, bool need_wa) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int p = a.pl.p;
    AnyLds l;
    if constexpr (!LDS_TABLES) {  // large P: tables stay in global memory (L1/L2)
        l.tw = const_cast<cf*>(reinterpret_cast<const cf*>(a.twany));
        l.st = const_cast<cf*>(reinterpret_cast<const cf*>(a.t.st));
        l.wa = const_cast<float*>(a.t.wa);
        l.A = reinterpret_cast<cf*>(smem) + size_t(threadIdx.x >> 6) * 2 * p;
        l.B = l.A + p;
        return l;
    }
    l.tw = reinterpret_cast<cf*>(smem);
    l.st = l.tw + a.tw_len;
    l.wa = reinterpret_cast<float*>(l.st + p);
    l.A = reinterpret_cast<cf*>(l.wa + 2 * p) + size_t(threadIdx.x >> 6) * 2 * p;
    l.B = l.A + p;
    const int nt = blockDim.x;
    const cf* gtw = reinterpret_cast<const cf*>(a.twany);
    const cf* gst = reinterpret_cast<const cf*>(a.t.st);
    for (int i = threadIdx.x; i < a.tw_len; i += nt) l.tw[i] = gtw[i];
    for (int i = threadIdx.x; i < p; i += nt) l.st[i] = gst[i];
    if (need_wa)
        for (int i = threadIdx.x; i < 2 * p; i += nt) l.wa[i] = a.t.wa[i];
    __syncthreads();
    return l;
}

static size_t any_lds_bytes(int p, int tw_len, int waves, bool tables) {
    const size_t bufs = size_t(waves) * 2 * p * sizeof(cf);
    return tables ? sizeof(cf) * (size_t(tw_len) + p) + sizeof(float) * 2 * p + bufs : bufs;
}

// K_synth for any N: the push_frame_AoS input of every frame (and optionally the
// forward spectrum), the same steps as k_synth_frames.
template <bool HAS_GAIN, bool LDS_TABLES>
__global__ __launch_bounds__(512) void k_synth_any(const AnyArgs a) {
    const int p = a.pl.p, n = 2 * p;
    const int lane = threadIdx.x & 63;
    const AnyLds l = any_lds<LDS_TABLES>(a, true);
    cf* A = l.A;
    cf* B = l.B;
    const int64_t gw = int64_t(blockIdx.x) * a.waves_per_block + (threadIdx.x >> 6);
    if (gw >= int64_t(a.n_streams) * a.F) return;
    const int64_t s = gw / a.F, k = gw % a.F;
    const float* x = a.in + s * a.ld_in;
    const int64_t base = k * a.h - a.pad;
    const cf* tw = l.tw;
    const bool inside = base >= 0 && base + n <= a.T;
    for (int i = lane; i < p; i += 64) {
        const int64_t t0 = base + 2 * i;
        float x0, x1;
        if (inside) {
            x0 = x[t0];
            x1 = x[t0 + 1];
        } else {
            x0 = fetch_x64(x, t0, a.T, a.pad_mode);
            x1 = fetch_x64(x, t0 + 1, a.T, a.pad_mode);
        }
        A[i] = {dev::sanit(x0 * l.wa[2 * i]), dev::sanit(x1 * l.wa[2 * i + 1])};
    }
    dev::wave_lds_fence();
    cf* z = dev::any::fft<false>(A, B, a.pl, tw, lane);
    cf* zo = z == A ? B : A;
    cf* spec = a.spec ? reinterpret_cast<cf*>(a.spec) + gw * (p + 1) : nullptr;
    dev::any::split_merge<HAS_GAIN>(z, zo, p, l.st, a.t.gain, spec, lane);
    dev::wave_lds_fence();
    cf* r = dev::any::fft<true>(zo, z, a.pl, tw, lane);
    float* out = a.out + gw * n;
    for (int i = lane; i < p; i += 64) {
        const cf v = r[i];
        out[2 * i] = dev::sanit(v.r * a.inv_n);
        out[2 * i + 1] = dev::sanit(v.i * a.inv_n);
    }
}

// K_fused_any: the fused walk for any N.  A wave owns a run of consecutive frames
// of one stream (+ warm-up frames); the OLA accumulates in a per-wave LDS ring
// of RL = H ceil(N/H) floats in ascending k (k_ola_gather's arithmetic, so the
// result equals the staged path bit for bit); block k is divided by max(norm,
// eps) and stored right after frame k.  Tables are staged once per workgroup.
struct AnyFusedArgs {
    AnyArgs a;        // tables, plan, x (in), y (out), T, pad
    int64_t ld_y;
    int out_len_i, n_chunks, M, F, rl;  // rl = ring floats per wave
    int ring_len;
    float gain;
    const uint32_t* mask;  // K_pair15 flags [stream / mask_div][mask_chunks], or nullptr: every stream
    int mask_chunks, mask_div;
};

template <bool HAS_GAIN>
__global__ __launch_bounds__(1024) void k_stft_ola_any(const AnyFusedArgs f) {
    const AnyArgs& a = f.a;
    const int p = a.pl.p, n = 2 * p, H = a.h;
    const int lane = threadIdx.x & 63;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // [tables (any_lds layout)][per wave: A, B (2P cf)][per wave: ring (rl f)]
    const AnyLds l = any_lds<true>(a, true);
    const int wave = threadIdx.x >> 6;
    float* ws = reinterpret_cast<float*>(l.A - size_t(wave) * 2 * p + size_t(a.waves_per_block) * 2 * p);
    float* ring = ws + 2 * p + size_t(wave) * f.rl;
    if (wave == 0)
        for (int i = lane; i < 2 * p; i += 64) ws[i] = a.t.ws[i];
    __syncthreads();
    const int64_t gw = int64_t(blockIdx.x) * a.waves_per_block + wave;
    if (gw >= int64_t(a.n_streams) * f.n_chunks) return;
    const int64_t s = gw / f.n_chunks, c = gw - s * f.n_chunks;
    if (f.mask) {  // redo only the streams the pair walker flagged
        bool any = false;
        for (int j = 0; j < f.mask_chunks; ++j)
            any |= ((f.mask[(s / f.mask_div) * f.mask_chunks + j] >> (s % f.mask_div)) & 1u) != 0u;
        if (!any) return;
    }
    const int nbr = f.rl / H;
    const int f0 = int(c) * f.M;
    const int f1 = min(f.F, f0 + f.M);
    const int fs = max(0, f0 - (nbr - 1));
    const float* x = a.in + s * a.ld_in;
    float* y = a.out + s * f.ld_y;
    cf* A = l.A;
    cf* B = l.B;
    for (int i = lane; i < f.rl; i += 64) ring[i] = 0.0f;
    for (int k = fs; k < f1; ++k) {
        const int64_t base = int64_t(k) * H - a.pad;
        const bool inside = base >= 0 && base + n <= a.T;
        for (int i = lane; i < p; i += 64) {
            const int64_t t0 = base + 2 * i;
            float x0, x1;
            if (inside) {
                x0 = x[t0];
                x1 = x[t0 + 1];
            } else {
                x0 = fetch_x64(x, t0, a.T, a.pad_mode);
                x1 = fetch_x64(x, t0 + 1, a.T, a.pad_mode);
            }
            A[i] = {dev::sanit(x0 * l.wa[2 * i]), dev::sanit(x1 * l.wa[2 * i + 1])};
        }
        dev::wave_lds_fence();
        cf* z = dev::any::fft<false>(A, B, a.pl, l.tw, lane);
        cf* zo = z == A ? B : A;
        dev::any::split_merge<HAS_GAIN>(z, zo, p, l.st, a.t.gain, nullptr, lane);
        dev::wave_lds_fence();
        const cf* r = dev::any::fft<true>(zo, z, a.pl, l.tw, lane);
        // push_frame_AoS(k*H): ring[(kH + i) mod rl] = fma(fma(src, w, 0), g, ring)
        const int rb = (k % nbr) * H;
        for (int i = lane; i < n; i += 64) {
            const cf v = r[i >> 1];
            const float src = dev::sanit(((i & 1) ? v.i : v.r) * a.inv_n);
            int pos = rb + i;
            if (pos >= f.rl) pos -= f.rl;
            ring[pos] = __builtin_fmaf(__builtin_fmaf(src, ws[i], 0.0f), f.gain, ring[pos]);
        }
        dev::wave_lds_fence();
        // produce(H): block k is complete
        const int64_t ob = int64_t(k) * H;
        int di = int(ob % f.ring_len);
        for (int i = lane; i < H; i += 64) {
            const int pos = rb + i;
            if (k >= f0) {
                int d = di + i;
                if (d >= f.ring_len) d -= f.ring_len;
                y[ob + i] = ring[pos] / a.t.den[d];
            }
            ring[pos] = 0.0f;
        }
        dev::wave_lds_fence();
    }
}

// K_stream_any: one hop of the per-hop streaming path for any N, H (DROP Framer).
// Per channel: `hist` holds the last hl >= N + H samples (hop q at (qH) mod hl),
// `acc` the OLA ring of rl = H ceil(N/H) floats.  When this hop completes frame
// k (host-decided: wave-uniform), the frame runs through the same arithmetic as
// K_fused_any and block k (H samples) is emitted.
struct StreamAnyArgs {
    AnyArgs a;                       // tables, plan, in (hop), out (hop), inv_n, h
    float* hist;
    float* acc;
    int64_t in_ld, in_inc, out_ld, out_inc;
    int64_t q, k;                    // hop index; frame completed by it (-1: none)
    int channels, hl, rl, ring_len;
    float gain;
};

template <bool HAS_GAIN>
__global__ __launch_bounds__(512) void k_stream_any(const StreamAnyArgs f) {
    const AnyArgs& a = f.a;
    const int p = a.pl.p, n = 2 * p, H = a.h;
    const int lane = threadIdx.x & 63;
    const AnyLds l = any_lds<true>(a, true);
    const int wave = threadIdx.x >> 6;
    float* ws = reinterpret_cast<float*>(l.A - size_t(wave) * 2 * p + size_t(a.waves_per_block) * 2 * p);
    if (wave == 0)
        for (int i = lane; i < n; i += 64) ws[i] = a.t.ws[i];
    __syncthreads();
    const int c = blockIdx.x * a.waves_per_block + wave;
    if (c >= f.channels) return;
    float* hist = f.hist + int64_t(c) * f.hl;
    float* acc = f.acc + int64_t(c) * f.rl;
    // store the hop
    const int hb = int((f.q * H) % f.hl);
    for (int i = lane; i < H; i += 64) hist[hb + i] = a.in[c * f.in_ld + i * f.in_inc];
    if (f.k < 0) return;
    __threadfence();  // the hop written by other lanes of this wave is read back below
    const int64_t k = f.k;
    const int fb = int((k * H) % f.hl);
    cf* A = l.A;
    cf* B = l.B;
    for (int i = lane; i < p; i += 64) {
        int j0 = fb + 2 * i, j1 = j0 + 1;
        if (j0 >= f.hl) j0 -= f.hl;
        if (j1 >= f.hl) j1 -= f.hl;
        A[i] = {dev::sanit(hist[j0] * l.wa[2 * i]), dev::sanit(hist[j1] * l.wa[2 * i + 1])};
    }
    dev::wave_lds_fence();
    cf* z = dev::any::fft<false>(A, B, a.pl, l.tw, lane);
    cf* zo = z == A ? B : A;
    dev::any::split_merge<HAS_GAIN>(z, zo, p, l.st, a.t.gain, nullptr, lane);
    dev::wave_lds_fence();
    const cf* r = dev::any::fft<true>(zo, z, a.pl, l.tw, lane);
    const int nbr = f.rl / H;
    const int rb = int(k % nbr) * H;
    for (int i = lane; i < n; i += 64) {
        const cf v = r[i >> 1];
        const float src = dev::sanit(((i & 1) ? v.i : v.r) * a.inv_n);
        int pos = rb + i;
        if (pos >= f.rl) pos -= f.rl;
        acc[pos] = __builtin_fmaf(__builtin_fmaf(src, ws[i], 0.0f), f.gain, acc[pos]);
    }
    __threadfence_block();
    const int di = int((k * H) % f.ring_len);
    for (int i = lane; i < H; i += 64) {
        int d = di + i;
        if (d >= f.ring_len) d -= f.ring_len;
        a.out[c * f.out_ld + i * f.out_inc] = acc[rb + i] / a.t.den[d];
        acc[rb + i] = 0.0f;
    }
}

// batched IFftPlan::forward / inverse / forward_complex / inverse_complex, any size
template <int KIND, bool LDS_TABLES>  // KIND: 0 rfft, 1 irfft, 2 cfft, 3 icfft
__global__ __launch_bounds__(512) void k_fft_any(const AnyArgs a) {
    const int p = a.pl.p;
    const int lane = threadIdx.x & 63;
    const AnyLds l = any_lds<LDS_TABLES>(a, false);
    cf* A = l.A;
    cf* B = l.B;
    const int64_t b = int64_t(blockIdx.x) * a.waves_per_block + (threadIdx.x >> 6);
    if (b >= a.batch) return;
    const float* in = a.in + b * a.ld_in;
    float* out = a.out + b * a.ld_out;
    const cf* tw = l.tw;
    const cf* st = l.st;
    if (KIND == 0) {
        for (int i = lane; i < p; i += 64)
            A[i] = {dev::sanit(in[int64_t(2 * i) * a.inc_in]), dev::sanit(in[int64_t(2 * i + 1) * a.inc_in])};
    } else if (KIND == 1) {
        // kiss_fftri merge of the caller's bins X[0..P]
        for (int k = lane; k < p; k += 64) {
            const cf xk = {in[int64_t(2 * k) * a.inc_in], in[int64_t(2 * k) * a.inc_in + 1]};
            const int pk = p - k;
            const cf xpk = {in[int64_t(2 * pk) * a.inc_in], in[int64_t(2 * pk) * a.inc_in + 1]};
            A[k] = dev::any::rmerge(xk, xpk, st[k], k);
        }
    } else {
        for (int i = lane; i < p; i += 64)
            A[i] = {in[int64_t(2 * i) * a.inc_in], in[int64_t(2 * i) * a.inc_in + 1]};
    }
    dev::wave_lds_fence();
    cf* z = dev::any::fft<(KIND == 1 || KIND == 3)>(A, B, a.pl, tw, lane);
    if (KIND == 0) {  // kiss_fftr split: X[k], k <= P
        for (int k = lane; k < p; k += 64) {
            cf xk, xp;
            dev::any::rsplit(z, p, st, k, xk, xp);
            out[int64_t(2 * k) * a.inc_out] = xk.r;
            out[int64_t(2 * k) * a.inc_out + 1] = xk.i;
            if (k == 0) {
                out[int64_t(2 * p) * a.inc_out] = xp.r;
                out[int64_t(2 * p) * a.inc_out + 1] = xp.i;
            }
        }
    } else if (KIND == 1) {
        for (int i = lane; i < p; i += 64) {
            out[int64_t(2 * i) * a.inc_out] = dev::sanit(z[i].r * a.inv_n);
            out[int64_t(2 * i + 1) * a.inc_out] = dev::sanit(z[i].i * a.inv_n);
        }
    } else if (KIND == 2) {
        for (int i = lane; i < p; i += 64) {
            out[int64_t(2 * i) * a.inc_out] = z[i].r;
            out[int64_t(2 * i) * a.inc_out + 1] = z[i].i;
        }
    } else {
        for (int i = lane; i < p; i += 64) {
            out[int64_t(2 * i) * a.inc_out] = dev::sanit(z[i].r * a.inv_n);
            out[int64_t(2 * i) * a.inc_out + 1] = dev::sanit(z[i].i * a.inv_n);
        }
    }
}

// ------------------------------------------------------------------ streaming
// One hop of the low-latency path (BASELINE config 4): per channel, the last
// NB = N/H hops live in `hist` (slot q mod NB holds hop q) and the OLA
// accumulator blocks in `acc` (slot b mod NB holds output block b).  Call q
// (0-based) brings hop q; once q >= NB-1 the DROP-mode Framer yields frame
// f = q-NB+1 (hops f..q), which goes through the same transform and OLA
// arithmetic as the batched kernels; block f is then complete and emitted.
// The lane that owns frame sample i owns it in every frame (H % 128 == 0), so a
// lane only ever touches its own acc words: no cross-lane hazards.
struct StreamArgs {
    DevTables t;
    const float* in;   // hop input: channel c sample i at in[c*in_ld + i*in_inc]
    float* out;        // hop output, same layout (out_ld, out_inc)
    float* hist;       // [C][N]
    float* acc;        // [C][N]
    int64_t in_ld, in_inc, out_ld, out_inc;
    int64_t q;         // index of the hop being pushed
    int channels, ring_len;
    float inv_n, gain;
};

template <int E, int S, bool HAS_GAIN>
__global__ __launch_bounds__(kBlock) void k_stream_hop(const StreamArgs a) {
    constexpr int P = 64 * E, N = 2 * P, H = 128 * S, NB = E / S;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    cf* st = tw + P;
    cf* sth = st + P;
    float* wa = reinterpret_cast<float*>(sth + P);
    float* ws = wa + N;
    cf* bufs = reinterpret_cast<cf*>(ws + N);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c = blockIdx.x * kWaves + wave;
    const bool live = c < a.channels;
    const int cc = live ? c : 0;
    const float* in = a.in + cc * a.in_ld;
    float* hist = a.hist + int64_t(cc) * N;
    float* acc = a.acc + int64_t(cc) * N;
    const int64_t q = a.q;
    const bool frame = q >= NB - 1;
    const int64_t f = q - (NB - 1);
    // Everything a hop reads from global memory is requested before the table
    // staging barrier, so the two latencies overlap (a hop is latency-bound).
    float2 hop[S];
#pragma unroll
    for (int s2 = 0; s2 < S; ++s2) {
        const int i0 = 2 * (lane + 64 * s2);
        hop[s2] = make_float2(in[i0 * a.in_inc], in[(i0 + 1) * a.in_inc]);
    }
    float2 xv[E];      // frame samples (older hops from their slots, the new hop last)
    float2 cur[E];     // OLA blocks this frame adds to
    float2 dd[S];      // divisors of the block that completes
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const int i0 = 2 * (lane + 64 * m);
        const int slot = int((f + m / S) % NB);
        xv[m] = (frame && m < E - S) ? *reinterpret_cast<const float2*>(hist + slot * H + (i0 % H))
                                     : make_float2(0.f, 0.f);
        cur[m] = frame ? *reinterpret_cast<const float2*>(acc + slot * H + (i0 % H)) : make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int m = 0; m < S; ++m) {
        const int64_t n = f * H + ((2 * (lane + 64 * m)) % H);
        dd[m] = frame ? make_float2(a.t.den[n % a.ring_len], a.t.den[(n + 1) % a.ring_len]) : make_float2(1.f, 1.f);
    }
    load_tables<E>(a.t, tw, st, sth, wa, ws, true);
    cf* buf = bufs + wave * xbuf_elems<P>();
    if (!live) return;
    if (frame) {
        cf v[E];
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int i0 = 2 * (lane + 64 * m);
            const float2 x2 = m >= E - S ? hop[m - (E - S)] : xv[m];
            v[m].r = dev::sanit(x2.x * wa[i0]);
            v[m].i = dev::sanit(x2.y * wa[i0 + 1]);
        }
        dev::fft_wave<E, false>(v, buf, tw, lane);
        dev::real_split_hook_merge<E, HAS_GAIN, false>(v, buf, st, sth, a.t.gain, lane);
        dev::fft_wave<E, true>(v, buf, tw, lane);
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int i0 = 2 * (lane + 64 * m);
            const float o0 = dev::sanit(v[m].r * a.inv_n);
            const float o1 = dev::sanit(v[m].i * a.inv_n);
            const int slot = int((f + m / S) % NB);
            float2* r = reinterpret_cast<float2*>(acc + slot * H + (i0 % H));
            float2 cu = cur[m];
            cu.x = __builtin_fmaf(__builtin_fmaf(o0, ws[i0], 0.0f), a.gain, cu.x);
            cu.y = __builtin_fmaf(__builtin_fmaf(o1, ws[i0 + 1], 0.0f), a.gain, cu.y);
            if (m < S) {  // block f is complete: produce(H) and clear its slot
                const int pos = i0 % H;
                float* o = a.out + c * a.out_ld;
                o[pos * a.out_inc] = cu.x / dd[m].x;
                o[(pos + 1) * a.out_inc] = cu.y / dd[m].y;
                cu = make_float2(0.f, 0.f);
            }
            *r = cu;
        }
    }
    // store the new hop into its slot for later frames
    const int qslot = int(q % NB);
#pragma unroll
    for (int s2 = 0; s2 < S; ++s2)
        *reinterpret_cast<float2*>(hist + qslot * H + 2 * (lane + 64 * s2)) = hop[s2];
}

// ------------------------------------------------------------------ dispatch
template <int E>
inline size_t lds_bytes_full() {
    return Lds<E>::bytes;
}
template <int E>
inline size_t lds_bytes_fft() {
    constexpr int P = 64 * E;
    return sizeof(cf) * (3 * P) + sizeof(cf) * kWaves * xbuf_elems<P>();
}


int e_of(int n) {
    switch (n) {
        case 256: return 2;
        case 512: return 4;
        case 1024: return 8;
        case 2048: return 16;
        case 4096: return 32;
        default: return 0;
    }
}

// K_fused2 (two frames per wave) where its registers keep the occupancy: E = 4
// (97-111 VGPRs, 4 waves/SIMD) and E = 8 with S = 2 (168: 3 waves/SIMD, the
// headline); the other E = 8 hops need 170-197 VGPRs (2 waves/SIMD) and lose.
constexpr bool fused2_used(int e, int s, bool fast) {
#ifdef CRLOT_NO_FUSED2
    return false;
#endif
    return fast && (e == 4 || (e == 8 && s == 2));
}

template <int E, int S>
hipError_t fused_es(const FusedArgs& a, int64_t grid, hipStream_t stream) {
    constexpr int NB = E / S;
#ifdef CRLOT_NO_FAST  // A/B builds
    const bool fast = false;
#else
    const bool fast = a.t.wsn && a.t.rden;
#endif
#ifndef CRLOT_NO_FUSED2  // A/B builds: single-frame K_fused everywhere
    if (fused2_used(E, S, fast)) {
        auto k2 = a.t.gain ? k_stft_ola_fused2<E, S, NB, true> : k_stft_ola_fused2<E, S, NB, false>;
        const size_t lds2 = Lds<E>::bytes + sizeof(cf) * kWaves * 64 * E;
        hipError_t e2 = set_lds(k2, lds2);
        if (e2 != hipSuccess) return e2;
        note_launch(CRLOT_K_FUSED2, grid);
        hipLaunchKernelGGL(k2, dim3(unsigned(grid)), dim3(kBlock), lds2, stream, a);
        return hipGetLastError();
    }
#endif
    auto k = a.t.gain ? (fast ? k_stft_ola_fused<E, S, NB, true, true> : k_stft_ola_fused<E, S, NB, true, false>)
                      : (fast ? k_stft_ola_fused<E, S, NB, false, true> : k_stft_ola_fused<E, S, NB, false, false>);
    const size_t lds = Lds<E>::bytes;
    hipError_t e = set_lds(k, lds);
    if (e != hipSuccess) return e;
    note_launch(CRLOT_K_FUSED, grid);
    hipLaunchKernelGGL(k, dim3(unsigned(grid)), dim3(kBlock), lds, stream, a);
    return hipGetLastError();
}

// CRLOT_PAIR4K_NOHOT=1 (A/B, N = 4096, 2048 and 512): the two-regime walker alone over every chunk.
static bool pair4k_hot_disabled() {
    static const bool v = [] {
        const char* e = ab_env("CRLOT_PAIR4K_NOHOT");
        return e && e[0] == '1';
    }();
    return v;
}
// K_pair4k's / K_pair2k's hot walker at three waves per SIMD (k_pair_wg_hot3,
// measured slower: DESIGN.md section 5) only in -DCRLOT_PAIR_WG_HOT3_EXPERIMENT
// builds with CRLOT_PAIR4K_HOT=3 (A/Bs; bit-identical)
static bool pair4k_hot3() {
#ifdef CRLOT_PAIR_WG_HOT3_EXPERIMENT
    static const bool v = [] {
        const char* e = ab_env("CRLOT_PAIR4K_HOT");
        return e && e[0] == '3';
    }();
    return v;
#else
    return false;
#endif
}

// K_pair512: N = 512, H = 64 SH, 4 independent waves per workgroup.
template <int SH>
hipError_t pair512_sh(const FusedArgs& a, int64_t waves, hipStream_t stream) {
    constexpr int NB = 8 / SH;
    auto k = a.t.gain ? k_stft_ola_pair512<SH, NB, true> : k_stft_ola_pair512<SH, NB, false>;
    const size_t lds = sizeof(cf) * dev::kP512Buf * kP512Waves;
    hipError_t e = set_lds(k, lds);
    if (e != hipSuccess) return e;
    const int64_t grid = (waves + kP512Waves - 1) / kP512Waves;
    if (!a.t.pflags || a.t.pflags_len < waves) return hipErrorInvalidValue;
    FusedArgs b = a;
    // the paired-only hot walker (H = 128, 256), then this two-regime walker over
    // the chunks it flagged; a gain or reflect/edge padding: the latter alone
    if ((SH == 2 || SH == 4) && !a.t.gain && a.pad_mode == 0 && !pair4k_hot_disabled() && a.t.hot) {
        if ((e = launch_pair512_hot(SH, a, waves, kP512Waves, stream)) != hipSuccess) return e;
    } else {
        b.fix_all = 1;
    }
    note_launch(CRLOT_K_PAIR512, grid);
    hipLaunchKernelGGL(k, dim3(unsigned(grid)), dim3(64 * kP512Waves), lds, stream, b);
    return hipGetLastError();
}
hipError_t launch_pair512(int sh, const FusedArgs& a, int64_t waves, hipStream_t stream) {
    switch (sh) {
        case 2: return pair512_sh<2>(a, waves, stream);
        case 4: return pair512_sh<4>(a, waves, stream);
        case 8: return pair512_sh<8>(a, waves, stream);
        default: return hipErrorInvalidValue;
    }
}

// K_pair2k: N = 2048, H = 128 SH, one 128-lane workgroup per chunk, four per CU.
template <int SH>
hipError_t pair2k_sh(const FusedArgs& a, int64_t grid, hipStream_t stream) {
    constexpr int NB = 16 / SH;
    auto k = a.t.gain ? k_stft_ola_pair2k<SH, NB, true> : k_stft_ola_pair2k<SH, NB, false>;
    hipError_t e = set_lds(k, kPair2kLds);
    if (e != hipSuccess) return e;
    note_launch(CRLOT_K_PAIR2K, grid);
    hipLaunchKernelGGL(k, dim3(unsigned(grid)), dim3(128), kPair2kLds, stream, a);
    return hipGetLastError();
}
void choose_chunks_rounds(int64_t F, int n_streams, int halo, int resident, int& n_chunks, int& m);
// The plan's chunk knob (crlot_plan_set_chunks, via the call's LaunchCtl)
// replaces the chooser's chunking: min(knob, F) chunks per stream.
void chunk_override(int64_t F, FusedArgs& a) {
    const int64_t n = chunks_or(0, F);
    if (n <= 0) return;
    a.M = int((F + n - 1) / n);
    a.n_chunks = int((F + a.M - 1) / a.M);
}
int fused_resident_waves();
hipError_t launch_pair2k(const Geometry& g, FusedArgs a, int64_t F, int n_streams, hipStream_t stream) {
    const bool hot = g.h == 512 && !a.t.gain && g.pad_mode == 0 && !pair4k_hot_disabled() && a.t.hot;
    const bool hot3 = hot && pair4k_hot3();  // six two-wave workgroups per CU, else four
    choose_chunks_rounds(F, n_streams, g.n / g.h + 1, fused_resident_waves() / 16 * (hot3 ? 6 : 4), a.n_chunks, a.M);
    chunk_override(F, a);
    note_chunks(a.n_chunks);
    a.ring_blocks = g.ring_len / g.h;
    a.pad = g.pad;
    a.pad_mode = g.pad_mode;
    a.inv_n = g.inv_n;
    a.gain = g.gain;
    const int64_t grid = int64_t(n_streams) * a.n_chunks;
    if (!a.t.pflags || a.t.pflags_len < grid) return hipErrorInvalidValue;
    // the paired-only hot walker where it holds its registers (H = 512), then the
    // two-regime walker over the chunks it flagged; otherwise the latter alone
    if (hot) {
        hipError_t e = hot3 ? launch_pair2k_hot3(4, a, grid, stream) : launch_pair2k_hot(4, a, grid, stream);
        if (e != hipSuccess) return e;
    } else {
        a.fix_all = 1;
    }
    switch (g.h / 128) {
        case 2: return pair2k_sh<2>(a, grid, stream);
        case 4: return pair2k_sh<4>(a, grid, stream);
        case 8: return pair2k_sh<8>(a, grid, stream);
        default: return hipErrorInvalidValue;
    }
}

template <int E>
hipError_t fused_e(int s, const FusedArgs& a, int64_t grid, hipStream_t stream) {
    if constexpr (E >= 1) {
        if (s == 1) return fused_es<E, 1>(a, grid, stream);
    }
    if constexpr (E >= 2) {
        if (s == 2) return fused_es<E, 2>(a, grid, stream);
    }
    if constexpr (E >= 4) {
        if (s == 4) return fused_es<E, 4>(a, grid, stream);
    }
    if constexpr (E >= 8) {
        if (s == 8) return fused_es<E, 8>(a, grid, stream);
    }
    if constexpr (E >= 16) {
        if (s == 16) return fused_es<E, 16>(a, grid, stream);
    }
    return hipErrorInvalidValue;
}

// Waves of K_fused the device holds at once: 4 per SIMD (<= 128 VGPRs), 4 SIMDs
// per CU.
int fused_resident_waves() {
    static const int v = [] {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            cus <= 0)
            cus = 256;
        return 16 * cus;
    }();
    return v;
}

// Split each stream's F frames into n chunks (one wave each; NB-1 halo frames
// recomputed per chunk).  Measured on MI355X (scripts/sweep_chunks.sh): ~128-frame
// chunks are right while the grid is several resident rounds deep (headline:
// flat for 12..24 chunks), but a small batch must still fill the device -- at
// least one resident round of waves, two when chunks stay >= 48 frames (config 2:
// +5 %, config 4 batched: +20 % over fixed 128-frame chunks).
void choose_chunks(int64_t F, int n_streams, int nb, int resident, int& n_chunks, int& m) {
    (void)nb;
    const int64_t S = std::max(1, n_streams);
    int64_t n = (F + 127) / 128;
    n = std::max<int64_t>(n, (resident + S - 1) / S);
    const int64_t two = (2 * resident + S - 1) / S;
    if (two > n && F / two >= 48) n = two;
    n = std::max<int64_t>(1, std::min<int64_t>(n, std::max<int64_t>(1, F / 32)));
    m = int((F + n - 1) / n);
    n_chunks = int((F + m - 1) / m);
}

// K_pair*: whole resident rounds.  A pair kernel's workgroup only frees its
// slots when all of its waves finish, so a grid that ends in a partial round
// idles the device for a whole chunk's time (headline, 16 waves/CU: 15 chunks
// = 3.75 rounds 219k Msamples/s, 8 chunks = 2 rounds 232k).  Among chunk counts
// with chunks of >= 48 frames, the fewest (rounds + 0.1) x (frames + halo + 10)
// per wave: the 0.1 charges a single long round for its tail, the 10 a wave's
// start-up (tables, first hops) (measured: headline 6 chunks = 2 rounds best,
// 9-15 within 1-3 %; config-4 shape 64 chunks = one round best).
void choose_chunks_rounds(int64_t F, int n_streams, int halo, int resident, int& n_chunks, int& m) {
    const int64_t S = std::max(1, n_streams), R = std::max(1, resident);
    const int64_t hi = std::max<int64_t>(1, F / 48);
    const int64_t lo = std::min(hi, (F + 511) / 512);
    int64_t best_n = lo;
    double best_cost = 1e300;
    for (int64_t n = lo; n <= hi; ++n) {
        const int64_t mm = (F + n - 1) / n, nc = (F + mm - 1) / mm;
        const double cost = (double((S * nc + R - 1) / R) + 0.1) * double(mm + halo + 10);
        if (cost < best_cost) best_cost = cost, best_n = n;
    }
    m = int((F + best_n - 1) / best_n);
    n_chunks = int((F + m - 1) / m);
}

// frames per workgroup walk (halo NB-1 frames recomputed); CRLOT_WG_CHUNK overrides
int wg_chunk_target() {
    static const int v = [] {
        const char* e = ab_env("CRLOT_WG_CHUNK");
        const int x = e ? std::atoi(e) : 0;
        return x > 0 ? x : 128;
    }();
    return v;
}

}  // namespace

bool pair_mask_supported(int n, int h) {
    return (n == 1024 && (h == 128 || h == 256 || h == 512)) || (n == 512 && (h == 128 || h == 256)) ||
           fk::pair_wg_supported(n, h);
}
bool pair_spec_supported(int n, int h) { return pair_mask_supported(n, h); }
// the frame-pair kernels' tables (N = 2048 / 4096 keep theirs in ptw4 / pden4)
bool pair_tables(const Geometry& g, const DevTables& t) {
    return (g.n >= 2048 ? (t.ptw4 && t.pden4) : (t.ptw && t.pden)) && t.wa && t.wsn && t.rden;
}

// K_pair_mask: K_pair's chunking (whole resident rounds) over its own residency
hipError_t launch_pair_masked(const Geometry& g, const DevTables& t, const SpecMask& m, const float* x, float* y,
                              int n_streams, int64_t T, int64_t ld_x, int64_t ld_y, int64_t F, int64_t out_len,
                              hipStream_t stream) {
    if (!pair_mask_supported(g.n, g.h) || F <= 0 || n_streams <= 0 || !m.p || !pair_tables(g, t) ||
        g.ring_len % g.h != 0)
        return hipErrorInvalidValue;
    FusedArgs a;
    a.t = t;
    a.x = x;
    a.y = y;
    a.ld_x = ld_x;
    a.ld_y = ld_y;
    a.T = int(T);
    a.out_len = int(out_len);
    a.n_streams = n_streams;
    a.F = int(F);
    const int resident = fused_resident_waves() / 16 * fk::pair_mask_walkers_per_cu(g.n);
    choose_chunks_rounds(F, n_streams, g.n / g.h + 1, resident, a.n_chunks, a.M);
    // a batch below one resident round (one window of a few streams: the per-call
    // latency case) walks chunks of >= 8 frames instead, as many as fit the round
    const int64_t S = std::max(1, n_streams);
    if (S * a.n_chunks < resident) {
        const int64_t n = std::min<int64_t>(F / 8, (resident + S - 1) / S);
        if (n > a.n_chunks) {
            a.M = int((F + n - 1) / n);
            a.n_chunks = int((F + a.M - 1) / a.M);
        }
    }
    chunk_override(F, a);
    note_chunks(a.n_chunks);
    a.ring_blocks = g.ring_len / g.h;
    a.pad = g.pad;
    a.pad_mode = g.pad_mode;
    a.inv_n = g.inv_n;
    a.gain = g.gain;
    return fk::launch_pair_mask(g.n, g.h, a, m, int64_t(n_streams) * a.n_chunks, stream);
}

// K_pair_stft: chunks of an even number of frames (pairs start on even frames), about
// 128 per walk, at least two resident rounds of walks (no warm-up frames to amortise)
hipError_t launch_pair_stft(const Geometry& g, const DevTables& t, const float* x, int n_streams, int64_t T,
                            int64_t ld_x, int64_t F, float* spec, int64_t ld_spec, int64_t ld_frame,
                            hipStream_t stream) {
    if (!pair_spec_supported(g.n, g.h) || F <= 0 || n_streams <= 0 || !pair_tables(g, t)) return hipErrorInvalidValue;
    fk::PairSpecArgs a{};
    a.f.t = t;
    a.f.x = x;
    a.f.ld_x = ld_x;
    a.f.T = int(T);
    a.f.n_streams = n_streams;
    a.f.F = int(F);
    a.f.pad = g.pad;
    a.f.pad_mode = g.pad_mode;
    a.spec = spec;
    a.ld_spec = ld_spec;
    a.ld_frame = ld_frame;
    const int64_t S = std::max(1, n_streams), resident = fused_resident_waves() / 16 * fk::pair_spec_walkers_per_cu(g.n);
    int64_t n = std::max<int64_t>((F + 127) / 128, (2 * resident + S - 1) / S);
    n = std::max<int64_t>(1, std::min<int64_t>(n, (F + 1) / 2));  // (down to one pair per walk: small batches)
    if (const int64_t c = chunks_or(0, F); c > 0) n = std::min(c, F);
    int64_t m = (F + n - 1) / n;
    m += m & 1;
    a.f.M = int(m);
    a.f.n_chunks = int((F + m - 1) / m);
    note_chunks(a.f.n_chunks);
    return fk::launch_pair_stft(g.n, g.h, a, int64_t(n_streams) * a.f.n_chunks, stream);
}

// K_pair_istft: K_pair_mask's chunking (whole resident rounds; small batches in >= 8-frame chunks)
hipError_t launch_pair_istft(const Geometry& g, const DevTables& t, const SpecMask& m, const float* spec,
                             int64_t ld_spec, int64_t ld_frame, float* y, int n_streams, int64_t F, int64_t ld_y,
                             hipStream_t stream) {
    if (!pair_spec_supported(g.n, g.h) || F <= 0 || n_streams <= 0 || !pair_tables(g, t) || g.ring_len % g.h != 0)
        return hipErrorInvalidValue;
    fk::PairSpecArgs a{};
    a.f.t = t;
    a.f.y = y;
    a.f.ld_y = ld_y;
    a.f.out_len = int(F * g.h);
    a.f.n_streams = n_streams;
    a.f.F = int(F);
    a.f.ring_blocks = g.ring_len / g.h;
    a.f.inv_n = g.inv_n;
    a.f.gain = g.gain;
    a.sin = spec;
    a.ld_spec = ld_spec;
    a.ld_frame = ld_frame;
    a.mask = m;
    const int resident = fused_resident_waves() / 16 * fk::pair_spec_walkers_per_cu(g.n);
    choose_chunks_rounds(F, n_streams, g.n / g.h + 1, resident, a.f.n_chunks, a.f.M);
    const int64_t S = std::max(1, n_streams);
    if (S * a.f.n_chunks < resident) {  // (small batches: chunks of >= 8 frames, as the mask walker)
        const int64_t n = std::min<int64_t>(F / 8, (resident + S - 1) / S);
        if (n > a.f.n_chunks) {
            a.f.M = int((F + n - 1) / n);
            a.f.n_chunks = int((F + a.f.M - 1) / a.f.M);
        }
    }
    chunk_override(F, a.f);
    note_chunks(a.f.n_chunks);
    return fk::launch_pair_istft(g.n, g.h, a, int64_t(n_streams) * a.f.n_chunks, stream);
}

std::vector<float> build_pair512_twiddles() {
    std::vector<float> t;
    for (int k1 = 1; k1 < 8; ++k1)
        for (int l = 0; l < 64; ++l) {
            const double ph = -2.0 * M_PI * double(l * k1) / 512.0;
            t.push_back(float(std::cos(ph)));
            t.push_back(float(std::sin(ph)));
        }
    for (int k2 = 1; k2 < 8; ++k2)
        for (int x = 0; x < 8; ++x) {
            const double ph = -2.0 * M_PI * double(x * k2) / 64.0;
            t.push_back(float(std::cos(ph)));
            t.push_back(float(std::sin(ph)));
        }
    return t;
}

std::vector<float> build_pair2k_twiddles() {
    std::vector<float> t;
    for (int k1 = 1; k1 < 16; ++k1)
        for (int l = 0; l < 128; ++l) {
            const double ph = -2.0 * M_PI * double(l * k1) / 2048.0;
            t.push_back(float(std::cos(ph)));
            t.push_back(float(std::sin(ph)));
        }
    for (int k2 = 1; k2 < 16; ++k2)
        for (int x = 0; x < 8; ++x) {
            const double ph = -2.0 * M_PI * double(x * k2) / 128.0;
            t.push_back(float(std::cos(ph)));
            t.push_back(float(std::sin(ph)));
        }
    return t;
}

std::vector<float> build_pair4k_twiddles() {
    std::vector<float> t;
    for (int k1 = 1; k1 < 16; ++k1)
        for (int l = 0; l < 256; ++l) {
            const double ph = -2.0 * M_PI * double(l * k1) / 4096.0;
            t.push_back(float(std::cos(ph)));
            t.push_back(float(std::sin(ph)));
        }
    for (int k2 = 1; k2 < 16; ++k2)
        for (int x = 0; x < 16; ++x) {
            const double ph = -2.0 * M_PI * double(x * k2) / 256.0;
            t.push_back(float(std::cos(ph)));
            t.push_back(float(std::sin(ph)));
        }
    return t;
}

std::vector<float> build_pass_twiddles(int n) {
    const int p = n / 2, e = p / 64;
    std::vector<float> t;
    int ns = 1;
    while (ns < p) {
        const int r = dev::radix_for(p / ns, e);
        if (ns > 1) {
            for (int q = 1; q < r; ++q)
                for (int jm = 0; jm < ns; ++jm) {
                    const double ph = -2.0 * M_PI * double(q) * double(jm) / double(ns * r);
                    t.push_back(float(std::cos(ph)));
                    t.push_back(float(std::sin(ph)));
                }
        }
        ns *= r;
    }
    return t;
}

bool fused_supported(int n, int h) {
    const int e = e_of(n);
    if (e == 0 || e > 16) return false;
    if (h % 128 != 0 || n % h != 0) return false;
    const int s = h / 128;
    return s == 1 || s == 2 || s == 4 || s == 8 || s == 16;
}

hipError_t launch_fused(const Geometry& g, const DevTables& t, const float* x, float* y,
                        int n_streams, int64_t T, int64_t ld_x, int64_t ld_y, int64_t F,
                        int64_t out_len, hipStream_t stream) {
    if (!fused_supported(g.n, g.h) || F <= 0 || n_streams <= 0) return hipErrorInvalidValue;
    FusedArgs a;
    a.t = t;
    a.x = x;
    a.y = y;
    a.ld_x = ld_x;
    a.ld_y = ld_y;
    a.T = int(T);
    a.out_len = int(out_len);
    a.n_streams = n_streams;
    a.F = int(F);
    const int e = e_of(g.n);
    const bool fast = t.wsn && t.rden;
#ifdef CRLOT_NO_PAIR  // A/B builds: per-frame kernels only
    const bool use_pair = false;
#else
    const bool use_pair = g.n == 1024 && t.ptw && t.pden && t.pflags && fast;
#endif
    const bool use_pair512 = g.n == 512 && t.ptw && t.pden && fast && g.h >= 128;
    if (g.n == 2048 && t.ptw4 && t.pden4 && fast && (g.h == 256 || g.h == 512 || g.h == 1024))
        return launch_pair2k(g, a, F, n_streams, stream);
#ifdef CRLOT_OLD_CHUNKS  // A/B builds: fixed ~128-frame chunks
    const int target = 128;
    a.n_chunks = int((F + target - 1) / target);
    a.M = int((F + a.n_chunks - 1) / a.n_chunks);
    a.n_chunks = int((F + a.M - 1) / a.M);
#else
    // K_fused and K_pair keep 4 waves/SIMD resident, K_fused2 3
    const bool pair = !use_pair && fused2_used(e, g.h / 128, fast);
    const int resident = use_pair ? fused_resident_waves() * pair_waves_per_cu() / 16
                         : pair && e == 8 ? fused_resident_waves() * 3 / 4 : fused_resident_waves();
    if (use_pair || use_pair512)
        choose_chunks_rounds(F, n_streams, g.n / g.h + 1, use_pair512 ? fused_resident_waves() : resident,
                             a.n_chunks, a.M);
    else
        choose_chunks(F, n_streams, g.n / g.h, resident, a.n_chunks, a.M);
    chunk_override(F, a);
#endif
    note_chunks(a.n_chunks);
    a.ring_blocks = g.ring_len / g.h;
    a.pad = g.pad;
    a.pad_mode = g.pad_mode;
    a.inv_n = g.inv_n;
    a.gain = g.gain;
    const int64_t waves = int64_t(n_streams) * a.n_chunks;
    if (use_pair) return launch_pair(g.h / 64, a, waves, stream);
    if (use_pair512) return launch_pair512(g.h / 64, a, waves, stream);
    const int64_t grid = (waves + kWaves - 1) / kWaves;
    const int s = g.h / 128;
    switch (e) {
        case 2: return fused_e<2>(s, a, grid, stream);
        case 4: return fused_e<4>(s, a, grid, stream);
        case 8: return fused_e<8>(s, a, grid, stream);
        case 16: return fused_e<16>(s, a, grid, stream);
        default: return hipErrorInvalidValue;
    }
}

// K_pair straight on interleaved groups (N = 1024, zero padding): n_groups x
// channels streams, sample i of channel c of group g at x[g*ld_x + i*channels + c]
// (outputs likewise), chunked exactly as launch_fused chunks the same number of
// planar streams.  hipErrorNotSupported when the plan is not on K_pair.
hipError_t launch_pair_interleaved(const Geometry& g, const DevTables& t, const float* x, float* y, int n_groups,
                                   int channels, int64_t T, int64_t ld_x, int64_t ld_y, int64_t F,
                                   int64_t out_len, hipStream_t stream) {
    const bool fast = t.wsn && t.rden;
    if (!(g.n == 1024 && t.ptw && t.pden && t.pflags && fast && g.pad_mode == 0 && fused_supported(g.n, g.h) &&
          g.h <= 512))
        return hipErrorNotSupported;
    const int64_t S = int64_t(n_groups) * channels;
    if (F <= 0 || n_groups <= 0 || channels < 1 || S > INT32_MAX || (T + 2 * g.n) * channels >= (int64_t(1) << 29) ||
        (out_len + 2 * g.n) * channels >= (int64_t(1) << 29))
        return hipErrorInvalidValue;
    FusedArgs a;
    a.t = t;
    a.x = x;
    a.y = y;
    a.ld_x = ld_x;
    a.ld_y = ld_y;
    a.T = int(T);
    a.out_len = int(out_len);
    a.n_streams = int(S);
    a.F = int(F);
    a.cs = channels;
    choose_chunks_rounds(F, a.n_streams, g.n / g.h + 1, fused_resident_waves() * pair_waves_per_cu() / 16,
                         a.n_chunks, a.M);
    chunk_override(F, a);
    note_chunks(a.n_chunks);
    a.ring_blocks = g.ring_len / g.h;
    a.pad = g.pad;
    a.pad_mode = g.pad_mode;
    a.inv_n = g.inv_n;
    a.gain = g.gain;
    return launch_pair(g.h / 64, a, S * a.n_chunks, stream);
}

// K_pair4k: N = 4096, H = 256 SH, one 256-lane workgroup per chunk, two per CU.
template <int SH>
static hipError_t pair4k_sh(const FusedArgs& a, int64_t grid, hipStream_t stream) {
    constexpr int NB = 16 / SH;
    auto k = a.t.gain ? k_stft_ola_pair4k<SH, NB, true> : k_stft_ola_pair4k<SH, NB, false>;
    hipError_t e = set_lds(k, kPair4kLds);
    if (e != hipSuccess) return e;
    note_launch(CRLOT_K_PAIR4K, grid);
    hipLaunchKernelGGL(k, dim3(unsigned(grid)), dim3(256), kPair4kLds, stream, a);
    return hipGetLastError();
}

// Workgroup walker: N = 16 L (E = 8), H = 2 L S.
template <int L, int S>
static hipError_t fused_wg_ls(const FusedArgs& a, int64_t grid, hipStream_t stream) {
    constexpr int NB = 8 / S;
    auto k = a.t.gain ? k_stft_ola_wg<L, S, NB, true> : k_stft_ola_wg<L, S, NB, false>;
    const size_t lds = sizeof(cf) * 3 * 8 * L;
    hipError_t e = set_lds(k, lds);
    if (e != hipSuccess) return e;
    note_launch(CRLOT_K_FUSED_WG, grid);
    hipLaunchKernelGGL(k, dim3(unsigned(grid)), dim3(L), lds, stream, a);
    return hipGetLastError();
}

template <int L>
static hipError_t fused_wg_l(int s, const FusedArgs& a, int64_t grid, hipStream_t stream) {
    switch (s) {
        case 1: return fused_wg_ls<L, 1>(a, grid, stream);
        case 2: return fused_wg_ls<L, 2>(a, grid, stream);
        case 4: return fused_wg_ls<L, 4>(a, grid, stream);
        case 8: return fused_wg_ls<L, 8>(a, grid, stream);
        default: return hipErrorInvalidValue;
    }
}

// N = 4096 always; N = 2048 (L = 128) only when CRLOT_WG_2048=1 (A/B against the
// per-wave E = 16 kernel, which is the default there).
bool fused_wg_supported(int n, int h) {
    static const bool wg2048 = [] {
        const char* e = ab_env("CRLOT_WG_2048");
        return e && e[0] == '1';
    }();
    if (n != 4096 && !(n == 2048 && wg2048)) return false;
    const int L = n / 16;
    if (h % (2 * L) != 0 || n % h != 0) return false;
    const int s = h / (2 * L);
    return s == 1 || s == 2 || s == 4 || s == 8;
}

hipError_t launch_fused_wg(const Geometry& g, const DevTables& t, const float* x, float* y,
                           int n_streams, int64_t T, int64_t ld_x, int64_t ld_y, int64_t F,
                           int64_t out_len, hipStream_t stream) {
    if (!fused_wg_supported(g.n, g.h) || F <= 0 || n_streams <= 0) return hipErrorInvalidValue;
    FusedArgs a;
    a.t = t;
    a.x = x;
    a.y = y;
    a.ld_x = ld_x;
    a.ld_y = ld_y;
    a.T = int(T);
    a.out_len = int(out_len);
    a.n_streams = n_streams;
    a.F = int(F);
    const int target = wg_chunk_target();
    a.n_chunks = int((F + target - 1) / target);
    a.M = int((F + a.n_chunks - 1) / a.n_chunks);
    a.n_chunks = int((F + a.M - 1) / a.M);
    chunk_override(F, a);
    note_chunks(a.n_chunks);
    a.ring_blocks = g.ring_len / g.h;
    a.pad = g.pad;
    a.pad_mode = g.pad_mode;
    a.inv_n = g.inv_n;
    a.gain = g.gain;
    if (g.n == 4096 && t.ptw4 && t.pden4 && t.wsn && t.rden && (g.h == 512 || g.h == 1024 || g.h == 2048)) {
        // K_pair4k: whole resident rounds of workgroups (three per CU with the
        // three-workgroup hot walker, else two)
        const bool hot = (!t.gain || g.h == 1024) && a.pad_mode == 0 && !pair4k_hot_disabled() && a.t.hot;
        const bool hot3 = hot && !t.gain && g.h == 1024 && pair4k_hot3();
        choose_chunks_rounds(F, n_streams, g.n / g.h + 1, fused_resident_waves() / 16 * (hot3 ? 3 : 2), a.n_chunks,
                             a.M);
        chunk_override(F, a);
        note_chunks(a.n_chunks);
        const int64_t grid4 = int64_t(n_streams) * a.n_chunks;
        if (!t.pflags || t.pflags_len < grid4) return hipErrorInvalidValue;
        // the paired-only hot walker, then the two-regime walker over the chunks it
        // flagged; reflect/edge padding, or a spectral gain at H != 1024: the
        // two-regime walker alone
        if (hot) {
            hipError_t e = hot3 ? launch_pair4k_hot3(g.h / 256, a, grid4, stream)
                                : launch_pair4k_hot(g.h / 256, a, grid4, stream);
            if (e != hipSuccess) return e;
        } else {
            a.fix_all = 1;
        }
        switch (g.h / 256) {
            case 2: return pair4k_sh<2>(a, grid4, stream);
            case 4: return pair4k_sh<4>(a, grid4, stream);
            case 8: return pair4k_sh<8>(a, grid4, stream);
            default: return hipErrorInvalidValue;
        }
    }
    const int64_t grid = int64_t(n_streams) * a.n_chunks;
    const int L = g.n / 16, s = g.h / (2 * L);
    switch (L) {
        case 128: return fused_wg_l<128>(s, a, grid, stream);
        case 256: return fused_wg_l<256>(s, a, grid, stream);
        default: return hipErrorInvalidValue;
    }
}

bool synth_supported(int n) { return e_of(n) != 0; }

// ---- any-size path
int stream_any_hist_len(int n, int h) { return h * ((n + h + h - 1) / h); }  // >= N + H, H multiple
int stream_any_ring_len(int n, int h) { return h * ((n + h - 1) / h); }
// kf_factor order: 4s, then 2s, then odd primes; per-pass twiddle tables laid out
// as fft_any.h PassDesc describes (the device table = build_any_twiddles(p)).
static std::vector<int> any_factors(int p) {
    std::vector<int> f;
    int n = p;
    while (n % 4 == 0 && n > 1) {
        f.push_back(4);
        n /= 4;
    }
    while (n % 2 == 0 && n > 1) {
        f.push_back(2);
        n /= 2;
    }
    for (int d = 3; n > 1;) {
        if (d * d > n) d = n;
        if (n % d == 0) {
            f.push_back(d);
            n /= d;
        } else {
            d += 2;
        }
    }
    return f;
}

dev::any::Plan make_any_plan(int p) {
    dev::any::Plan pl{};
    pl.p = p;
    const std::vector<int> f = any_factors(p);
    int ns = 1, off = 0;
    for (size_t i = 0; i < f.size() && int(i) < dev::any::kMaxPasses; ++i) {
        dev::any::PassDesc& d = pl.pass[pl.n_pass++];
        d.r = f[i];
        d.ns = ns;
        d.off = off;
        d.rcp_ns = 1.0f / float(ns);
        off += (d.r - 1) * ns;
        const bool special = d.r == 2 || d.r == 3 || d.r == 4 || d.r == 5 || d.r == 7;
        d.woff = special ? 0 : off;
        if (!special) off += d.r;
        ns *= d.r;
    }
    return pl;
}

// the plan as the call server reads it from device memory (call_rt.hip)
std::vector<uint8_t> build_any_plan_blob(int p) {
    const dev::any::Plan pl = make_any_plan(p);
    std::vector<uint8_t> b(sizeof(pl));
    std::memcpy(b.data(), &pl, sizeof(pl));
    return b;
}

bool any_supported(int p) {
    return p >= 1 && p <= 8192 && any_factors(p).size() <= size_t(dev::any::kMaxPasses);
}

std::vector<float> build_any_twiddles(int p) {
    std::vector<float> t;
    const std::vector<int> f = any_factors(p);
    int ns = 1;
    auto push = [&](double ph) {
        t.push_back(float(std::cos(ph)));
        t.push_back(float(std::sin(ph)));
    };
    for (int r : f) {
        for (int q = 1; q < r; ++q)
            for (int jm = 0; jm < ns; ++jm) push(-2.0 * M_PI * double(q) * double(jm) / double(ns * r));
        if (!(r == 2 || r == 3 || r == 4 || r == 5 || r == 7))
            for (int e = 0; e < r; ++e) push(-2.0 * M_PI * double(e) / double(r));
        ns *= r;
    }
    if (t.empty()) push(0.0);  // P = 1: no passes
    return t;
}

// Waves per workgroup: up to 8 sharing one copy of the LDS tables, sized so two
// workgroups fit a CU's 160 KB when the tables are in LDS (P <= ~1000).
static int any_waves_per_block(int p) {
    const int per = 16 * p;               // two buffers of P float pairs per wave
    const int tables = 24 * p + 8 * 64;   // twiddles ~P, st P, wa 2P (float pairs / floats)
    const int budget = p <= 1024 ? 78 * 1024 - tables : 96 * 1024;
    return std::max(1, std::min(8, budget / per));
}

// tables in LDS when they fit beside the wave buffers (P <= 2048 or so)
static bool any_lds_tables(int p, int tw_len) {
    return any_lds_bytes(p, tw_len, any_waves_per_block(p), true) <= 150 * 1024;
}

template <typename K>
static hipError_t launch_any(K kernel, AnyArgs& a, int64_t items, hipStream_t stream, bool tables,
                             int32_t id = CRLOT_K_FFT_ANY) {
    a.waves_per_block = any_waves_per_block(a.pl.p);
    const size_t lds = any_lds_bytes(a.pl.p, a.tw_len, a.waves_per_block, tables);
    hipError_t e = set_lds(kernel, lds);
    if (e != hipSuccess) return e;
    const int64_t grid = (items + a.waves_per_block - 1) / a.waves_per_block;
    note_launch(id, grid);
    hipLaunchKernelGGL(kernel, dim3(unsigned(grid)), dim3(64 * a.waves_per_block), lds, stream, a);
    return hipGetLastError();
}

hipError_t launch_synth_any(const Geometry& g, const DevTables& t, const float* twany,
                            const float* x, int n_streams, int64_t T, int64_t ld_x, int64_t F,
                            float* frames, float* spec, hipStream_t stream) {
    if (F <= 0 || n_streams <= 0 || !any_supported(g.n / 2)) return hipErrorInvalidValue;
    AnyArgs a{};
    a.t = t;
    a.twany = twany;
    a.pl = make_any_plan(g.n / 2);
    a.in = x;
    a.out = frames;
    a.spec = spec;
    a.ld_in = ld_x;
    a.T = T;
    a.F = F;
    a.h = g.h;
    a.n_streams = n_streams;
    a.pad = g.pad;
    a.pad_mode = g.pad_mode;
    a.inv_n = g.inv_n;
    const int64_t items = int64_t(n_streams) * F;
    a.tw_len = int(build_any_twiddles(a.pl.p).size() / 2);
    const bool tb = any_lds_tables(a.pl.p, a.tw_len);
    if (tb)
        return t.gain ? launch_any(k_synth_any<true, true>, a, items, stream, true, CRLOT_K_SYNTH_ANY)
                      : launch_any(k_synth_any<false, true>, a, items, stream, true, CRLOT_K_SYNTH_ANY);
    return t.gain ? launch_any(k_synth_any<true, false>, a, items, stream, false, CRLOT_K_SYNTH_ANY)
                  : launch_any(k_synth_any<false, false>, a, items, stream, false, CRLOT_K_SYNTH_ANY);
}

hipError_t launch_fused_any(const Geometry& g, const DevTables& t, const float* twany,
                            const float* x, float* y, int n_streams, int64_t T, int64_t ld_x,
                            int64_t ld_y, int64_t F, hipStream_t stream, const uint32_t* mask,
                            int mask_chunks, int mask_div) {
    const int p = g.n / 2;
    if (F <= 0 || n_streams <= 0 || !any_supported(p)) return hipErrorInvalidValue;
    AnyFusedArgs f{};
    AnyArgs& a = f.a;
    a.t = t;
    a.twany = twany;
    a.pl = make_any_plan(p);
    a.in = x;
    a.out = y;
    a.ld_in = ld_x;
    a.T = T;
    a.h = g.h;
    a.n_streams = n_streams;
    a.pad = g.pad;
    a.pad_mode = g.pad_mode;
    a.inv_n = g.inv_n;
    a.tw_len = int(build_any_twiddles(p).size() / 2);
    f.ld_y = ld_y;
    f.F = int(F);
    f.rl = g.h * ((g.n + g.h - 1) / g.h);
    f.ring_len = g.ring_len;
    f.gain = g.gain;
    f.mask = mask;
    f.mask_chunks = mask_chunks;
    f.mask_div = mask_div > 0 ? mask_div : 1;
    const size_t tables = sizeof(cf) * (size_t(a.tw_len) + p) + sizeof(float) * 4 * p;  // + ws
    const size_t per_wave = sizeof(cf) * 2 * p + sizeof(float) * f.rl;
    // two workgroups per CU when each still holds >= 3 walkers (their tails overlap),
    // else one workgroup with as many walkers as the LDS takes (tables shared)
    int per_cu = 2;
    int w = int(std::min<size_t>(8, (75 * 1024 - std::min<size_t>(tables, 75 * 1024)) / per_wave));
    if (w < 3) {
        per_cu = 1;
        w = int(std::min<size_t>(16, (150 * 1024 - std::min<size_t>(tables, 150 * 1024)) / per_wave));
    }
    if (w < 1) return hipErrorInvalidValue;  // too large for one CU: staged path
    a.waves_per_block = w;
    const int nb = (g.n + g.h - 1) / g.h;
    const int resident = fused_resident_waves() / 16 * per_cu * w;  // CUs x walkers per CU
    choose_chunks(F, n_streams, nb, resident, f.n_chunks, f.M);
    if (const int64_t c = chunks_or(0, F); c > 0) {  // the plan's chunk knob
        f.M = int((F + c - 1) / c);
        f.n_chunks = int((F + f.M - 1) / f.M);
    }
    if (!mask) note_chunks(f.n_chunks);  // (a redo walk keeps the pair walker's record)
    const size_t lds = tables + size_t(w) * per_wave;
    const int64_t waves = int64_t(n_streams) * f.n_chunks;
    const int64_t grid = (waves + w - 1) / w;
    auto k = t.gain ? k_stft_ola_any<true> : k_stft_ola_any<false>;
    hipError_t e = set_lds(k, lds);
    if (e != hipSuccess) return e;
    note_launch(CRLOT_K_FUSED_ANY, grid);
    hipLaunchKernelGGL(k, dim3(unsigned(grid)), dim3(64 * w), lds, stream, f);
    return hipGetLastError();
}

hipError_t launch_stream_any(const Geometry& g, const DevTables& t, const float* twany,
                             const float* in, int64_t in_ld, int64_t in_inc, float* out,
                             int64_t out_ld, int64_t out_inc, float* hist, float* acc, int channels,
                             int64_t q, int64_t k, hipStream_t stream) {
    const int p = g.n / 2;
    if (channels <= 0 || !any_supported(p)) return hipErrorInvalidValue;
    StreamAnyArgs f{};
    AnyArgs& a = f.a;
    a.t = t;
    a.twany = twany;
    a.pl = make_any_plan(p);
    a.in = in;
    a.out = out;
    a.h = g.h;
    a.inv_n = g.inv_n;
    a.tw_len = int(build_any_twiddles(p).size() / 2);
    f.hist = hist;
    f.acc = acc;
    f.in_ld = in_ld;
    f.in_inc = in_inc;
    f.out_ld = out_ld;
    f.out_inc = out_inc;
    f.q = q;
    f.k = k;
    f.channels = channels;
    f.hl = stream_any_hist_len(g.n, g.h);
    f.rl = stream_any_ring_len(g.n, g.h);
    f.ring_len = g.ring_len;
    f.gain = g.gain;
    const size_t tables = sizeof(cf) * (size_t(a.tw_len) + p) + sizeof(float) * 4 * p;
    const size_t per_wave = sizeof(cf) * 2 * p;
    int w = int(std::min<size_t>(8, (150 * 1024 - std::min<size_t>(tables, 150 * 1024)) / per_wave));
    if (w < 1) return hipErrorInvalidValue;
    a.waves_per_block = w;
    const size_t lds = tables + size_t(w) * per_wave;
    auto kern = t.gain ? k_stream_any<true> : k_stream_any<false>;
    hipError_t e = set_lds(kern, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(unsigned((channels + w - 1) / w)), dim3(64 * w), lds, stream, f);
    return hipGetLastError();
}

bool fused_any_fits(int n, int h) {
    const int p = n / 2;
    if (!any_supported(p) || h <= 0) return false;
    const size_t tw_len = build_any_twiddles(p).size() / 2;
    const size_t tables = sizeof(cf) * (tw_len + p) + sizeof(float) * 4 * p;
    const size_t per_wave = sizeof(cf) * 2 * p + sizeof(float) * (h * ((n + h - 1) / h));
    return tables + per_wave <= 150 * 1024;
}

hipError_t launch_fft_any(int kind, int p, float inv_scale, const DevTables& t, const float* twany,
                          const float* in, float* out, int batch, int64_t ld_in, int64_t inc_in,
                          int64_t ld_out, int64_t inc_out, hipStream_t stream) {
    if (batch <= 0 || !any_supported(p)) return hipErrorInvalidValue;
    AnyArgs a{};
    a.t = t;
    a.twany = twany;
    a.pl = make_any_plan(p);
    a.in = in;
    a.out = out;
    a.ld_in = ld_in;
    a.inc_in = inc_in;
    a.ld_out = ld_out;
    a.inc_out = inc_out;
    a.batch = batch;
    a.inv_n = inv_scale;
    a.tw_len = int(build_any_twiddles(p).size() / 2);
    const bool tb = any_lds_tables(p, a.tw_len);
    switch (kind * 2 + (tb ? 1 : 0)) {
        case 0: return launch_any(k_fft_any<0, false>, a, batch, stream, false);
        case 1: return launch_any(k_fft_any<0, true>, a, batch, stream, true);
        case 2: return launch_any(k_fft_any<1, false>, a, batch, stream, false);
        case 3: return launch_any(k_fft_any<1, true>, a, batch, stream, true);
        case 4: return launch_any(k_fft_any<2, false>, a, batch, stream, false);
        case 5: return launch_any(k_fft_any<2, true>, a, batch, stream, true);
        case 6: return launch_any(k_fft_any<3, false>, a, batch, stream, false);
        case 7: return launch_any(k_fft_any<3, true>, a, batch, stream, true);
        default: return hipErrorInvalidValue;
    }
}

template <int E>
static hipError_t synth_e(const SynthArgs& a, int64_t grid, hipStream_t stream) {
    const size_t lds = Lds<E>::bytes;
    if (a.spec) {
        auto k = a.t.gain ? k_synth_frames<E, true, true> : k_synth_frames<E, false, true>;
        hipError_t e = set_lds(k, lds);
        if (e != hipSuccess) return e;
        note_launch(CRLOT_K_SYNTH, grid);
        hipLaunchKernelGGL(k, dim3(unsigned(grid)), dim3(kBlock), lds, stream, a);
    } else {
        auto k = a.t.gain ? k_synth_frames<E, true, false> : k_synth_frames<E, false, false>;
        hipError_t e = set_lds(k, lds);
        if (e != hipSuccess) return e;
        note_launch(CRLOT_K_SYNTH, grid);
        hipLaunchKernelGGL(k, dim3(unsigned(grid)), dim3(kBlock), lds, stream, a);
    }
    return hipGetLastError();
}

hipError_t launch_synth_frames(const Geometry& g, const DevTables& t, const float* x,
                               int n_streams, int64_t T, int64_t ld_x, int64_t F, float* frames,
                               float* spec, hipStream_t stream) {
    if (!synth_supported(g.n) || F <= 0 || n_streams <= 0) return hipErrorInvalidValue;
    SynthArgs a;
    a.t = t;
    a.x = x;
    a.frames = frames;
    a.spec = spec;
    a.ld_x = ld_x;
    a.T = T;
    a.F = F;
    a.h = g.h;
    a.n_streams = n_streams;
    a.pad = g.pad;
    a.pad_mode = g.pad_mode;
    a.inv_n = g.inv_n;
    const int64_t waves = int64_t(n_streams) * F;
    const int64_t grid = (waves + kWaves - 1) / kWaves;
    switch (e_of(g.n)) {
        case 2: return synth_e<2>(a, grid, stream);
        case 4: return synth_e<4>(a, grid, stream);
        case 8: return synth_e<8>(a, grid, stream);
        case 16: return synth_e<16>(a, grid, stream);
        case 32: return synth_e<32>(a, grid, stream);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_ola_gather(const Geometry& g, const DevTables& t, const float* frames,
                             int64_t ld_frames, float* y, int n_streams, int64_t F,
                             int64_t ld_y, int64_t out_len, hipStream_t stream) {
    if (F <= 0 || n_streams <= 0 || out_len <= 0) return hipErrorInvalidValue;
    GatherArgs a;
    a.frames = frames;
    a.ws = t.ws;
    a.den = t.den;
    a.y = y;
    a.ld_frames = ld_frames;
    a.ld_y = ld_y;
    a.F = F;
    a.out_len = out_len;
    a.n = g.n;
    a.h = g.h;
    a.ring_len = g.ring_len;
    a.n_streams = n_streams;
    a.gain = g.gain;
    static const int gv = [] {  // A/B: CRLOT_GATHER=2 the per-sample-grid kernel
        const char* e = ab_env("CRLOT_GATHER");
        return e ? std::atoi(e) : 3;
    }();
    if (gv == 3 && n_streams <= 65535 && F < (int64_t(1) << 31) && out_len <= F * g.h &&
        out_len < (int64_t(1) << 31) - int64_t(g.h)) {
        const int nb = (g.n + g.h - 1) / g.h;
        auto kg = nb <= 4 ? k_ola_gather_blk<4> : k_ola_gather_blk<8>;
        const int threads = g.h >= 256 ? 256 : (g.h + 63) / 64 * 64;
        static const int bpb_env = [] {
            const char* e = ab_env("CRLOT_GATHER_BPB");
            return e ? std::atoi(e) : 0;
        }();
        const int bpb = bpb_env > 0 ? bpb_env : std::max(1, 1024 / g.h);  // >= 1024 outputs per workgroup
        note_launch(CRLOT_K_GATHER, (F + bpb - 1) / bpb * n_streams);
        hipLaunchKernelGGL(kg, dim3(unsigned((F + bpb - 1) / bpb), unsigned(n_streams)), dim3(threads), 0, stream,
                           a, bpb);
        return hipGetLastError();
    }
    if (n_streams <= 65535 && out_len < (int64_t(1) << 31) - 256 && int64_t(g.h) + 256 < (1 << 24)) {
        // one sample per thread (two per thread measured 5-15 % slower: occupancy)
        auto kg = (g.n + g.h - 1) / g.h <= 4 ? k_ola_gather2<1, 4> : k_ola_gather2<1, 8>;
        const int64_t per_block = 256;
        note_launch(CRLOT_K_GATHER, (out_len + per_block - 1) / per_block * n_streams);
        hipLaunchKernelGGL(kg, dim3(unsigned((out_len + per_block - 1) / per_block), unsigned(n_streams)),
                           dim3(256), 0, stream, a);
        return hipGetLastError();
    }
    const int64_t total = int64_t(n_streams) * out_len;
    const int64_t grid = (total + 255) / 256;
    note_launch(CRLOT_K_GATHER, grid);
    hipLaunchKernelGGL(k_ola_gather, dim3(unsigned(grid)), dim3(256), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_ola_gather_wrap(const Geometry& g, const DevTables& t, const float* frames, int64_t ld_frames,
                                  int64_t F, int64_t len, float* acc, float* y, hipStream_t stream, float* y_blocks) {
    if (F <= 0 || len <= 0 || g.ring_len <= 0 || g.n > g.ring_len) return hipErrorInvalidValue;
    GatherArgs a{};
    a.frames = frames;
    a.ws = t.ws;
    a.den = t.den;
    a.y = y_blocks;
    a.ld_frames = ld_frames;
    a.F = F;
    a.n = g.n;
    a.h = g.h;
    a.ring_len = g.ring_len;
    a.n_streams = 1;
    a.gain = g.gain;
    const int64_t y_len = y_blocks ? len : 0;
    const int64_t grid = (y_len + int64_t(g.ring_len) + 255) / 256;
    note_launch(CRLOT_K_GATHER, grid);
    hipLaunchKernelGGL(k_ola_gather_wrap, dim3(unsigned(grid)), dim3(256), 0, stream, a, acc, y, len, y_len);
    return hipGetLastError();
}

template <int E>
static hipError_t rfft_irfft_e(const FftArgs& a, float* r, float* r_host, int64_t ld_r, hipStream_t stream) {
    constexpr int P = 64 * E;
    const size_t lds = lds_bytes_fft<E>() + sizeof(cf) * kWaves * (P + 1);
    const int64_t grid = (int64_t(a.batch) + kWaves - 1) / kWaves;
    hipError_t e = set_lds(k_rfft_irfft<E>, lds);
    if (e != hipSuccess) return e;
    note_launch(CRLOT_K_FFT, grid);
    hipLaunchKernelGGL(k_rfft_irfft<E>, dim3(unsigned(grid)), dim3(kBlock), lds, stream, a, r, r_host, ld_r);
    return hipGetLastError();
}

hipError_t launch_rfft_irfft(const Geometry& g, const DevTables& t, const float* in, int64_t ld_in, float* spec,
                             int64_t ld_spec, float* r, float* r_host, int64_t ld_r, int batch, hipStream_t stream) {
    if (batch <= 0) return hipErrorInvalidValue;
    FftArgs a;
    a.t = t;
    a.in = in;
    a.out = spec;
    a.ld_in = ld_in;
    a.inc_in = 1;
    a.ld_out = ld_spec;
    a.inc_out = 1;
    a.batch = batch;
    a.inv_n = g.inv_n;
    switch (e_of(g.n)) {
        case 2: return rfft_irfft_e<2>(a, r, r_host, ld_r, stream);
        case 4: return rfft_irfft_e<4>(a, r, r_host, ld_r, stream);
        case 8: return rfft_irfft_e<8>(a, r, r_host, ld_r, stream);
        case 16: return rfft_irfft_e<16>(a, r, r_host, ld_r, stream);
        default: return hipErrorInvalidValue;  // (4096: the spectra would not fit LDS beside the tables)
    }
}

template <int E, bool INV, bool CPLX = false>
static hipError_t fft_e(const FftArgs& a, hipStream_t stream) {
    const size_t lds = lds_bytes_fft<E>();
    const int64_t grid = (int64_t(a.batch) + kWaves - 1) / kWaves;
    auto k = CPLX ? k_cfft<E, INV> : INV ? k_irfft<E> : k_rfft<E>;
    hipError_t e = set_lds(k, lds);
    if (e != hipSuccess) return e;
    note_launch(CRLOT_K_FFT, grid);
    hipLaunchKernelGGL(k, dim3(unsigned(grid)), dim3(kBlock), lds, stream, a);
    return hipGetLastError();
}

template <bool INV, bool CPLX = false>
static hipError_t fft_dispatch(const Geometry& g, const DevTables& t, const float* in, float* out,
                               int batch, int64_t ld_in, int64_t inc_in, int64_t ld_out,
                               int64_t inc_out, hipStream_t stream) {
    if (batch <= 0) return hipErrorInvalidValue;
    FftArgs a;
    a.t = t;
    a.in = in;
    a.out = out;
    a.ld_in = ld_in;
    a.inc_in = inc_in;
    a.ld_out = ld_out;
    a.inc_out = inc_out;
    a.batch = batch;
    a.inv_n = CPLX ? 2.0f * g.inv_n : g.inv_n;  // 1/P for a P = N/2 point complex plan
    switch (e_of(g.n)) {
        case 2: return fft_e<2, INV, CPLX>(a, stream);
        case 4: return fft_e<4, INV, CPLX>(a, stream);
        case 8: return fft_e<8, INV, CPLX>(a, stream);
        case 16: return fft_e<16, INV, CPLX>(a, stream);
        case 32: return fft_e<32, INV, CPLX>(a, stream);
        default: return hipErrorInvalidValue;
    }
}

template <int E, int S>
static hipError_t stream_es(const StreamArgs& a, hipStream_t stream) {
    auto k = a.t.gain ? k_stream_hop<E, S, true> : k_stream_hop<E, S, false>;
    const size_t lds = Lds<E>::bytes;
    hipError_t e = set_lds(k, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3(unsigned((a.channels + kWaves - 1) / kWaves)), dim3(kBlock), lds,
                       stream, a);
    return hipGetLastError();
}

template <int E>
static hipError_t stream_e(int s, const StreamArgs& a, hipStream_t stream) {
    if constexpr (E >= 1) {
        if (s == 1) return stream_es<E, 1>(a, stream);
    }
    if constexpr (E >= 2) {
        if (s == 2) return stream_es<E, 2>(a, stream);
    }
    if constexpr (E >= 4) {
        if (s == 4) return stream_es<E, 4>(a, stream);
    }
    if constexpr (E >= 8) {
        if (s == 8) return stream_es<E, 8>(a, stream);
    }
    if constexpr (E >= 16) {
        if (s == 16) return stream_es<E, 16>(a, stream);
    }
    return hipErrorInvalidValue;
}

hipError_t launch_stream_hop(const Geometry& g, const DevTables& t, const float* in, int64_t in_ld,
                             int64_t in_inc, float* out, int64_t out_ld, int64_t out_inc,
                             float* hist, float* acc, int channels, int64_t q,
                             hipStream_t stream) {
    if (!fused_supported(g.n, g.h) || channels <= 0) return hipErrorInvalidValue;
    StreamArgs a;
    a.t = t;
    a.in = in;
    a.out = out;
    a.hist = hist;
    a.acc = acc;
    a.in_ld = in_ld;
    a.in_inc = in_inc;
    a.out_ld = out_ld;
    a.out_inc = out_inc;
    a.q = q;
    a.channels = channels;
    a.ring_len = g.ring_len;
    a.inv_n = g.inv_n;
    a.gain = g.gain;
    const int s = g.h / 128;
    switch (e_of(g.n)) {
        case 2: return stream_e<2>(s, a, stream);
        case 4: return stream_e<4>(s, a, stream);
        case 8: return stream_e<8>(s, a, stream);
        case 16: return stream_e<16>(s, a, stream);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_rfft(const Geometry& g, const DevTables& t, const float* in, float* out,
                       int batch, int64_t ld_in, int64_t inc_in, int64_t ld_out, int64_t inc_out,
                       hipStream_t stream) {
    return fft_dispatch<false>(g, t, in, out, batch, ld_in, inc_in, ld_out, inc_out, stream);
}

hipError_t launch_cfft(const Geometry& g, const DevTables& t, const float* in, float* out, int batch,
                       int64_t ld_in, int64_t inc_in, int64_t ld_out, int64_t inc_out, bool inverse,
                       hipStream_t stream) {
    return inverse ? fft_dispatch<true, true>(g, t, in, out, batch, ld_in, inc_in, ld_out, inc_out, stream)
                   : fft_dispatch<false, true>(g, t, in, out, batch, ld_in, inc_in, ld_out, inc_out, stream);
}

hipError_t launch_irfft(const Geometry& g, const DevTables& t, const float* in, float* out,
                        int batch, int64_t ld_in, int64_t inc_in, int64_t ld_out, int64_t inc_out,
                        hipStream_t stream) {
    return fft_dispatch<true>(g, t, in, out, batch, ld_in, inc_in, ld_out, inc_out, stream);
}

}  // namespace crlot

