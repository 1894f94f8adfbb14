// pair1k.hip -- K_pair, the N = 1024 frame-pair walker (the headline kernel).
// Numerics as kernels.hip (header comment there); the transform is fft_pair.h.
#include <algorithm>
#include <cmath>

#include "fft_pair.h"
#include "fused_common.h"

namespace crlot {

using dev::cf;

namespace fk {

// ------------------------------------------------------------------ fused, frame pairs (N = 1024)
// K_pair k_stft_ola_pair<SH,NB,W>: the fused walk with frames 2j and 2j+1 of a
// stream packed into ONE 1024-point complex transform (fft_pair.h):
// z = x_2j * w + i x_2j+1 * w; the round trip's real part is frame 2j's
// push_frame_AoS input and the imaginary part frame 2j+1's.  Pairs are aligned
// to even frame indices whatever the chunking (a chunk's warm-up starts on an
// even frame and a pair straddling its end still transforms the real partner),
// so every frame's bits depend only on the stream.  Lane l holds samples
// l + 64 m of the frame; a hop is SH = H/64 floats per lane.
//
// Two regimes per pair, chosen from the pair's own hops (k .. k+NB), so again
// independent of the chunking:
//  * paired: every sample is 0 or px_lo <= |x| <= px_hi (DevTables, set on the
//    host from the window and the spectral gain).  Then sanitize(x*w) == x*w up
//    to the sign of a zero, which no output bit can see (a nonzero value plus a
//    zero of either sign is exact, and the output sanitize maps both zeros to
//    +0); no transform can overflow; and the output sanitize reduces to its
//    threshold test.
//  * unpaired (a NaN, Inf, huge or tiny sample): each frame gets a transform of
//    its own (imaginary part zero) with the full sanitize on both sides, so a
//    frame whose spectrum overflows cannot leak into its neighbour -- the
//    reference transforms every frame alone (kissfft_adapter.cc:83-168).
// Everything after the inverse is K_fused2's: folded 1/N, OLA in ascending k,
// Markstein division with a per-wave IEEE fallback.
// LDS: t1 [15*64 cf] | t2 [3*16 cf] | wa4 [1024 f] | ws4 [1024 f] | per-wave
// transpose buffers.  Windows are stored [m/4][lane][m%4] so one ds_read_b128
// gives a lane 4 taps.
template <int W>
struct PairLds {
    static constexpr size_t t1 = 0;
    static constexpr size_t t2 = t1 + sizeof(cf) * 15 * 64;
    static constexpr size_t wa = t2 + sizeof(cf) * 3 * 16;
    static constexpr size_t ws = wa + sizeof(float) * 1024;
    static constexpr size_t bufs = ws + sizeof(float) * 1024;
    static constexpr size_t bytes = bufs + sizeof(cf) * dev::kPairXbuf * W;
};

#ifdef CRLOT_PAIR_TRACE
__device__ uint32_t g_pair_trace[4 << 16];
#endif
#ifdef CRLOT_PAIR_PHASES  // debug builds: per-wave cycles by loop phase (s_memtime)
__device__ uint32_t g_pair_phase[8 << 16];
#define PHASE(i)                                              \
    do {                                                      \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();     \
        ph[i] += uint32_t(t_ - ph_last);                      \
        ph_last = t_;                                         \
    } while (0)
#else
#define PHASE(i) \
    do {         \
    } while (0)
#endif
#ifndef CRLOT_PAIR_REG_TW
#define CRLOT_PAIR_REG_TW 1  // measured: same cycles as LDS twiddles at 4 waves/SIMD, +0.2..5.6 % on the clock
#endif
#ifndef CRLOT_PAIR_MIN_WAVES
#define CRLOT_PAIR_MIN_WAVES (CRLOT_PAIR_REG_TW ? 3 : 4)
#endif
template <int SH, int NB, int W, bool HAS_GAIN>
__global__ __launch_bounds__(64 * W, CRLOT_PAIR_MIN_WAVES) void k_stft_ola_pair(const FusedArgs a) {
    constexpr int E = 16, N = 1024, H = 64 * SH;
    static_assert(NB * SH == E, "N = NB * H");
    static_assert(SH >= 2, "den rows are read 16 bytes at a time");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    dev::pc* t1 = reinterpret_cast<dev::pc*>(smem + PairLds<W>::t1);
    dev::pc* t2s = reinterpret_cast<dev::pc*>(smem + PairLds<W>::t2);
    float* wa4 = reinterpret_cast<float*>(smem + PairLds<W>::wa);
    float* ws4 = reinterpret_cast<float*>(smem + PairLds<W>::ws);
    {
        const dev::pc* g1 = reinterpret_cast<const dev::pc*>(a.t.ptw);
        for (int i = threadIdx.x; i < 15 * 64 + 3 * 16; i += 64 * W) t1[i] = g1[i];  // t1 | t2
        for (int i = threadIdx.x; i < N; i += 64 * W) {
            const int l = i & 63, m = i >> 6;  // tap n = l + 64 m
            const int d = (m >> 2) * 256 + l * 4 + (m & 3);
            wa4[d] = a.t.wa[i];
            ws4[d] = a.t.wsn[i];
        }
        __syncthreads();
    }
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    dev::pc* buf = reinterpret_cast<dev::pc*>(smem + PairLds<W>::bufs) + wave * dev::kPairXbuf;
    const dev::pc* t2 = t2s + (lane & 15);  // t2[16 (c-1)] = W64^{(lane & 15) c}
    const int gw = blockIdx.x * W + wave;
    if (gw >= a.n_streams * a.n_chunks) return;
#ifdef CRLOT_PAIR_TRACE  // debug builds: per-wave start/end (100 MHz clock) and hardware ids
    const uint32_t trace_t0 = uint32_t(__builtin_amdgcn_s_memrealtime());
#endif
    const int s = gw / a.n_chunks, c = gw - s * a.n_chunks;
    const int f0 = c * a.M;
    const int f1 = min(a.F, f0 + a.M);
    const int fs = max(0, f0 - (NB - 1)) & ~1;  // pairs start on even frames
    const __amdgpu_buffer_rsrc_t rx = dev::make_rsrc(a.x + int64_t(s) * a.ld_x, uint32_t(a.T) * 4u);
    const __amdgpu_buffer_rsrc_t ry =
        dev::make_rsrc(a.y + int64_t(s) * a.ld_y, uint32_t(a.out_len) * 4u);
    const __amdgpu_buffer_rsrc_t rp = dev::make_rsrc(a.t.pden, uint32_t(a.ring_blocks * H) * 8u);
    const __amdgpu_buffer_rsrc_t ry_null = dev::make_rsrc(a.y, 0u);
    const float g = a.gain;
    const float xlo = a.t.px_lo, xhi = a.t.px_hi;

    // xin[h*SH + q]: hop (k + h), h = 0..NB, sample lane + 64 q of the hop;
    // bit h of hopok: hop k + h keeps the paired regime
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

    // push_frame_AoS of one frame: (sanitized) inverse output, folded 1/N, window, gain
    auto accumulate = [&](const dev::pc (&v)[E], bool imag, bool paired) {
#pragma unroll
        for (int m4 = 0; m4 < E / 4; ++m4) {
#ifdef CRLOT_ABL_NOWIN  // timing-only ablation: no window reads, wrong results
            const float4 w = make_float4(1e-3f, 2e-3f, 1e-3f, 2e-3f);
#else
            const float4 w = *reinterpret_cast<const float4*>(ws4 + m4 * 256 + lane * 4);
#endif
            const float wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int m = 4 * m4 + u;
                const float x = imag ? v[m].y : v[m].x;
                const float o = paired ? dev::sanit_scaled_finite<N>(x) : dev::sanit_scaled<N>(x);
                float& r = acc[m / SH][m % SH];
                r = __builtin_fmaf(__builtin_fmaf(o, wv[u], 0.0f), g, r);
            }
        }
    };
    // produce(H) of block k, then shift.  The divisions run for warm-up blocks
    // too (only the stores are skipped), so the divisor loads are used
    // unconditionally and stay where they are issued, ahead of the stores.
    auto emit = [&](int k, const float (&dr)[2 * SH]) {
        float mx = 0.0f, mn = 0x1p127f;
#pragma unroll
        for (int q = 0; q < SH; ++q) {
            const float t = __builtin_fabsf(acc[0][q]);
            mx = __builtin_fmaxf(mx, t);
            mn = __builtin_fminf(mn, t);
        }
        const bool ok = (mx <= 0x1p64f) & ((mn >= 0x1p-64f) | (mx == 0.0f));
        float o[SH];
#pragma unroll
        for (int q = 0; q < SH; ++q) o[q] = mk_div(acc[0][q], dr[q], dr[SH + q]);
        if (__builtin_amdgcn_ballot_w64(!ok) != 0) {  // outside Markstein's exact range: IEEE
#pragma unroll
            for (int q = 0; q < SH; ++q) o[q] = acc[0][q] / dr[q];
        }
#ifdef CRLOT_ABL_NODIV  // timing-only ablation
#pragma unroll
        for (int q = 0; q < SH; ++q) o[q] = acc[0][q] * dr[SH + q];
#endif
        // warm-up blocks (k < f0) store through a zero-size descriptor: every
        // lane is out of range and the store is dropped.  No branch around the
        // stores, so vmcnt bookkeeping stays exact at the next divisor wait.
#ifdef CRLOT_ABL_NOSTORE  // timing-only ablation: every store dropped
        const __amdgpu_buffer_rsrc_t rk = ry_null;
#else
        const __amdgpu_buffer_rsrc_t rk = k >= f0 ? ry : ry_null;
#endif
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

#ifdef CRLOT_PAIR_PHASES
    uint32_t ph[6] = {0, 0, 0, 0, 0, 0};
    uint64_t ph_last = __builtin_amdgcn_s_memtime();
#endif
#if CRLOT_PAIR_REG_TW  // twiddles held in registers (3 waves per SIMD)
    dev::PairTw tw;
    dev::pair_tw_load(tw, t1, t2, lane);
    const dev::PairTw& tw1 = tw;
    const dev::PairTw& tw2 = tw;
#else
    const dev::pc* const tw1 = t1;
    const dev::pc* const tw2 = t2;
#endif
    auto transform = [&](dev::pc (&v)[E]) {  // forward, spectral gain, inverse (unnormalised)
#ifdef CRLOT_ABL_NOFFT  // timing-only ablation: the memory stream alone
        return;
#endif
        dev::pair_fft_fwd(v, buf, tw1, tw2, lane);
        PHASE(2);
        if constexpr (HAS_GAIN) {  // real gain, symmetric over the N bins
            const int gbase = dev::pair_bin_lane(lane);
#pragma unroll
            for (int d = 0; d < E; ++d) {
                const int kb = gbase + 64 * d;
                const float gk = a.t.gain[kb <= N / 2 ? kb : N - kb];
                v[d] = v[d] * gk;
            }
        }
        dev::pair_fft_inv(v, buf, tw1, tw2, lane);
#ifdef CRLOT_ABL_DUMMY  // timing-only: CRLOT_ABL_DUMMY extra independent VALU ops per transform
        {
            float d[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) d[i] = v[i].x;
#pragma unroll
            for (int i = 0; i < CRLOT_ABL_DUMMY; ++i) {
#if defined(CRLOT_ABL_DUMMY_PERM)
                if ((i & 1) == 0) {
                    const unsigned a0 = __builtin_bit_cast(unsigned, d[i & 7]);
                    const unsigned b0 = __builtin_bit_cast(unsigned, d[(i + 1) & 7]);
                    const auto r = __builtin_amdgcn_permlane16_swap(a0, b0, false, false);
                    const unsigned r0 = r[0], r1 = r[1];
                    d[i & 7] = __builtin_bit_cast(float, r0);
                    d[(i + 1) & 7] = __builtin_bit_cast(float, r1);
                }
#else
                asm volatile("v_add_f32 %0, %0, %0" : "+v"(d[i & 7]));
#endif
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i].x = d[i];
        }
#endif
    };
    constexpr uint32_t kPairHops = (1u << (NB + 1)) - 1;  // hops k .. k+NB
    for (int k = fs; k < f1; k += 2) {
        // prefetch hops k+NB+1, k+NB+2 for the next pair
        float nxt[2 * SH];
        load_hop1<SH>(nxt, rx, lane, (k + NB + 1) * H - a.pad, a.T, a.pad_mode);
        load_hop1<SH>(nxt + SH, rx, lane, (k + NB + 2) * H - a.pad, a.T, a.pad_mode);
        const bool paired = (hopok & kPairHops) == kPairHops;
        PHASE(0);
        if (paired) {
            const bool partner = k + 1 < a.F;  // frame k+1 exists (even past this chunk)
            dev::pc v[E];
#pragma unroll
            for (int m4 = 0; m4 < E / 4; ++m4) {
#ifdef CRLOT_ABL_NOWIN
                const float4 w = make_float4(0.5f, 0.25f, 0.5f, 0.25f);
#else
                const float4 w = *reinterpret_cast<const float4*>(wa4 + m4 * 256 + lane * 4);
#endif
                const float wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int m = 4 * m4 + u;
                    v[m] = dev::pc_mk(xin[m] * wv[u], partner ? xin[m + SH] * wv[u] : 0.0f);
                }
            }
            PHASE(1);
            transform(v);
            PHASE(3);
            // both blocks' divisors before this pair's stores: vmcnt retires in
            // order, so a load issued after a store also waits for that store
            float dr0[2 * SH], dr1[2 * SH];
            load_den<SH>(dr0, rp, lane, k % a.ring_blocks);
            load_den<SH>(dr1, rp, lane, (k + 1) % a.ring_blocks);
            accumulate(v, false, true);
            emit(k, dr0);
            if (k + 1 < f1) {
                accumulate(v, true, true);
                emit(k + 1, dr1);
            }
            PHASE(4);
        } else {  // unpaired: frames k and k+1 alone, full sanitize (never taken on finite audio)
            const int npass = min(2, f1 - k);
            for (int p = 0; p < npass; ++p) {
                dev::pc v[E];
#pragma unroll
                for (int m4 = 0; m4 < E / 4; ++m4) {
                    const float4 w = *reinterpret_cast<const float4*>(wa4 + m4 * 256 + lane * 4);
                    const float wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int m = 4 * m4 + u;
                        v[m] = dev::pc_mk(dev::sanit((p ? xin[m + SH] : xin[m]) * wv[u]), 0.0f);
                    }
                }
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
#ifdef CRLOT_PAIR_PHASES
    PHASE(5);
    if (lane == 0 && gw < (1 << 16)) {
#pragma unroll
        for (int i = 0; i < 6; ++i) g_pair_phase[8 * gw + i] = ph[i];
        g_pair_phase[8 * gw + 6] = uint32_t((f1 - fs + 1) / 2);
        g_pair_phase[8 * gw + 7] = 1;
    }
#endif
#ifdef CRLOT_PAIR_TRACE
    if (lane == 0 && gw < (1 << 16)) {
        const uint32_t t1e = uint32_t(__builtin_amdgcn_s_memrealtime());
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // HW_REG_HW_ID
        const uint32_t xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20); // HW_REG_XCC_ID
        uint4* tr = reinterpret_cast<uint4*>(g_pair_trace);
        tr[gw] = make_uint4(trace_t0, t1e, hw, xcc);
    }
#endif
}


// K_pair: N = 1024, H = 64 * SH.  W waves per workgroup: with register twiddles
// (default) 4, three 53 KB workgroups per CU at <= 168 VGPRs (3 waves/SIMD);
// with LDS twiddles 16, one 160 KB workgroup per CU at <= 128 VGPRs.
#ifndef CRLOT_PAIR_WAVES
#define CRLOT_PAIR_WAVES (CRLOT_PAIR_REG_TW ? 4 : 16)  // 3 workgroups of 4 waves per CU; one of 12 is within +-1.5 % (slot-controlled A/B), 2 or 6 waves lose 7-25 %
#endif
constexpr int kPairWaves = CRLOT_PAIR_WAVES;

// Waves of K_pair a CU holds: whole workgroups within 160 KiB of LDS, at most
// CRLOT_PAIR_MIN_WAVES per SIMD.
int pair_waves_per_cu() {
    return std::min(int(163840 / PairLds<kPairWaves>::bytes) * kPairWaves, 4 * CRLOT_PAIR_MIN_WAVES);
}

template <int SH>
hipError_t pair_sh(const FusedArgs& a, int64_t waves, hipStream_t stream) {
    constexpr int NB = 16 / SH, W = kPairWaves;
    auto k = a.t.gain ? k_stft_ola_pair<SH, NB, W, true> : k_stft_ola_pair<SH, NB, W, false>;
    const size_t lds = PairLds<W>::bytes;
    hipError_t e = set_lds(k, lds);
    if (e != hipSuccess) return e;
    const int64_t grid = (waves + W - 1) / W;
    hipLaunchKernelGGL(k, dim3(unsigned(grid)), dim3(64 * W), lds, stream, a);
    return hipGetLastError();
}

hipError_t launch_pair(int sh, const FusedArgs& a, int64_t waves, hipStream_t stream) {
    switch (sh) {
        case 2: return pair_sh<2>(a, waves, stream);
        case 4: return pair_sh<4>(a, waves, stream);
        case 8: return pair_sh<8>(a, waves, stream);
        case 16: return pair_sh<16>(a, waves, stream);
        default: return hipErrorInvalidValue;
    }
}


}  // namespace fk

std::vector<float> build_pair_twiddles() {
    std::vector<float> t(2 * dev::kPairT1);
    for (int k1 = 1; k1 < 16; ++k1)
        for (int l = 0; l < 64; ++l) {
            const double ph = -2.0 * M_PI * double(l * k1) / 1024.0;
            const int i = dev::pair_t1_index(k1, l);
            t[2 * i] = float(std::cos(ph));
            t[2 * i + 1] = float(std::sin(ph));
        }
    for (int c = 1; c < 4; ++c)
        for (int b = 0; b < 16; ++b) {
            const double ph = -2.0 * M_PI * double(b * c) / 64.0;
            t.push_back(float(std::cos(ph)));
            t.push_back(float(std::sin(ph)));
        }
    return t;
}


}  // namespace crlot

#ifdef CRLOT_PAIR_TRACE
extern "C" int crlot_debug_pair_trace(void* host, int64_t bytes) {
    return int(hipMemcpyFromSymbol(host, HIP_SYMBOL(crlot::fk::g_pair_trace),
                                   size_t(std::min<int64_t>(bytes, sizeof(crlot::fk::g_pair_trace)))));
}
#endif

#ifdef CRLOT_PAIR_PHASES
extern "C" int crlot_debug_pair_phases(void* host, int64_t bytes) {
    return int(hipMemcpyFromSymbol(host, HIP_SYMBOL(crlot::fk::g_pair_phase),
                                   size_t(std::min<int64_t>(bytes, sizeof(crlot::fk::g_pair_phase)))));
}
#endif
