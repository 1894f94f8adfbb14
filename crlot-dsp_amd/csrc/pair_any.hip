// pair_any.hip -- K_pair15: the frame-pair round trip at N = 960 (20 ms at
// 48 kHz, one transform per wave) and N = 480 (10 ms, one per 32-lane half),
// any hop H whose ring the plan allows.
//
// Frames 2j and 2j+1 of a stream travel as one N-point complex transform,
// z = x_2j w + i x_2j+1 w, as the power-of-two pair kernels do (fft_pair15.h:
// a Good-Thomas 15-point DFT over 15 registers, then a batch of 64- or 32-point
// DFTs over the lanes).  H is in general not a multiple of the lanes, so a
// sample does not stay in its lane from frame to frame: every pair loads its two
// frames whole (15 dwords per lane each, mostly L2 hits -- each sample is read
// N/H times) and the overlap-add runs in an LDS ring of H ceil(N/H) floats per
// walk: push frame k (fma(o * ws, g, ring) in ascending k), produce block k (ring
// / den, IEEE division, then clear), push frame k+1, produce block k+1 -- the
// reference's streaming-interleaved order.  o = v * (1/N) after the inverse, as
// kissfft_adapter.cc:154 scales.
//
// At N = 480 the two halves of a wave walk two streams (2p, 2p+1) over the same
// chunk, so every branch is uniform; addresses carry the half's stream offset
// and edge frames select zero padding per sample.
//
// Paired regime only (like the hot walkers of pair_hot.hip): a sample outside
// [px_lo, px_hi] (or NaN / Inf), or an output below the sanitize threshold,
// flags the walk; a stream with any flagged walk is then recomputed whole by
// the per-frame mixed-radix walker (k_stft_ola_any, kissfft's algorithm with the
// full sanitize), so a stream's bits depend only on its own samples.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "fft_pair15.h"
#include "fused_common.h"

namespace crlot {
namespace fk {

namespace {

constexpr int kE = 15;  // registers per lane

template <int L>
struct P15 {
    static constexpr int N = 15 * L;
    using Tw = std::conditional_t<L == 64, dev::Pair15Tw, dev::Pair15hTw>;
    static __device__ __forceinline__ void tw_load(Tw& tw, const float* g, int hl) {
        if constexpr (L == 64)
            dev::pair15_tw_load(tw, reinterpret_cast<const dev::pc*>(g), hl);
        else
            dev::pair15h_tw_load(tw, reinterpret_cast<const dev::pc*>(g), hl);
    }
    static __device__ __forceinline__ void fwd(dev::pc (&v)[16], dev::pc* buf, const Tw& tw, int lane) {
        if constexpr (L == 64)
            dev::pair15_fwd(v, buf, tw, lane);
        else
            dev::pair15h_fwd(v, buf, tw, lane);
    }
    static __device__ __forceinline__ void inv(dev::pc (&v)[16], dev::pc* buf, const Tw& tw, int lane) {
        if constexpr (L == 64)
            dev::pair15_inv(v, buf, tw, lane);
        else
            dev::pair15h_inv(v, buf, tw, lane);
    }
};

// OLA ring of a walk: the live span is at most H ceil(N/H) floats; the ring is
// the next power of two, so a position wraps with one AND.
__host__ __device__ inline int p15_ring(int n, int h) {
    const int span = h * ((n + h - 1) / h);
    int r = 1;
    while (r < span) r <<= 1;
    return r;
}
// LDS: per wave [transpose 1152 cf][ring(s) 64 / L x RL f], then the windows
// [2][4][L][4] f shared by the workgroup.
template <int L>
size_t p15_lds(int h, int w, bool wreg = false) {
    return size_t(w) * (sizeof(dev::pc) * dev::kPairXbuf + sizeof(float) * (64 / L) * p15_ring(15 * L, h)) +
           (wreg ? 0 : sizeof(float) * 2 * 16 * L);
}

// Launch shapes (CRLOT_P15_VARIANT overrides, A/B): 0 = 5 walks per workgroup,
// windows in LDS, 3 waves/SIMD budget; 1 = 2 walks, windows in registers,
// 2 waves/SIMD; 2 = 4 walks, LDS windows; 3 = 2 walks, LDS windows; 4 = 4 walks,
// windows in registers, 3 waves/SIMD (13 KB of LDS per walk: 12 waves per CU).
struct P15Shape {
    int w;
    bool wreg;
    int wpe;  // register budget: waves per SIMD
};
constexpr P15Shape kP15Shapes[5] = {{5, false, 3}, {2, true, 2}, {4, false, 3}, {2, false, 3}, {4, true, 3}};
constexpr int kP15Waves = 5;  // the widest shape (support check)

}  // namespace

// WREG: windows in registers (else LDS); DPRE: H <= 4 L and the plan has the
// {den, 1/den} table (host-checked), divisors fetched ahead of the pushes
template <int L, int W, bool WREG, int WPE, bool HAS_GAIN = false, bool DPRE = false>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(WPE)))
void k_pair15_hot(const FusedArgs a) {
    constexpr int E = kE, N = P15<L>::N, HALVES = 64 / L;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, hl = lane % L, half = lane / L;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int H = a.hop;
    const int RL = p15_ring(N, H), RM = RL - 1;  // ring >= H ceil(N/H): no live position aliases
    const int NB = (N + H - 1) / H;
    dev::pc* buf = reinterpret_cast<dev::pc*>(smem) + wave * dev::kPairXbuf;
    float* rings = reinterpret_cast<float*>(reinterpret_cast<dev::pc*>(smem) + W * dev::kPairXbuf);
    float* wa4 = rings + W * HALVES * RL;  // tap n = hl + L m at (m / 4) 4 L + 4 hl + m % 4
    float* ws4 = wa4 + 16 * L;
    for (int i = threadIdx.x; i < (WREG ? 0 : 16 * L); i += 64 * W) {
        const int l = i % L, m = i / L;
        const int d = (m >> 2) * (4 * L) + l * 4 + (m & 3);
        wa4[d] = m < E ? a.t.wa[i] : 0.0f;
        ws4[d] = m < E ? a.t.ws[i] * a.inv_n * a.gain : 0.0f;  // (1/N, ws and g folded: push)
    }
    __syncthreads();
    float* ring = rings + (wave * HALVES + half) * RL;
    const int gw = blockIdx.x * W + wave;
    const int n_units = (a.n_streams + HALVES - 1) / HALVES;  // streams (960) or stream pairs (480)
    if (gw >= n_units * a.n_chunks) return;
    const int u = gw / a.n_chunks, c = gw - u * a.n_chunks;
    const int s0 = u * HALVES;  // this wave's first stream
    const bool pair_full = s0 + HALVES <= a.n_streams;
    const int f0 = c * a.M;
    const int f1 = min(a.F, f0 + a.M);
    const int fs = max(0, f0 - (NB - 1)) & ~1;  // pairs start on even frames
    // one descriptor over the wave's streams: the half's stream is an offset (a
    // missing second stream falls outside the range: reads 0, stores dropped)
    const uint32_t span_x = uint32_t((HALVES == 2 && pair_full ? a.ld_x + a.T : a.T) * 4);
    const uint32_t span_y = uint32_t((HALVES == 2 && pair_full ? a.ld_y + a.out_len : a.out_len) * 4);
    const __amdgpu_buffer_rsrc_t rx = dev::make_rsrc(a.x + int64_t(s0) * a.ld_x, span_x);
    const __amdgpu_buffer_rsrc_t ry = dev::make_rsrc(a.y + int64_t(s0) * a.ld_y, span_y);
    const __amdgpu_buffer_rsrc_t ry_null = dev::make_rsrc(a.y, 0u);
    const int xo = half * int(a.ld_x), yo = half * int(a.ld_y);  // < 2^27 (host-checked)
    const int ring_blocks = a.ring_blocks;  // ring_len / H (the den table's blocks)
    const uint32_t xlo_b = __builtin_bit_cast(uint32_t, a.t.px_lo), xhi_b = __builtin_bit_cast(uint32_t, a.t.px_hi);

    typename P15<L>::Tw tw;
    P15<L>::tw_load(tw, a.t.ptw, hl);
    float war[WREG ? E : 1], wsr[WREG ? E : 1];
    if constexpr (WREG) {
#pragma unroll
        for (int m = 0; m < E; ++m) {
            war[m] = a.t.wa[hl + L * m];
            wsr[m] = a.t.ws[hl + L * m] * a.inv_n * a.gain;
        }
    }
    auto win4 = [&](const float* w4, const float* wr, int m4, float (&wv)[4]) {
        if constexpr (WREG) {
#pragma unroll
            for (int q = 0; q < 4; ++q) wv[q] = 4 * m4 + q < E ? wr[4 * m4 + q] : 0.0f;
        } else {
            const float4 w = *reinterpret_cast<const float4*>(w4 + m4 * (4 * L) + hl * 4);
            wv[0] = w.x;
            wv[1] = w.y;
            wv[2] = w.z;
            wv[3] = w.w;
        }
    };
    for (int i = hl; i < RL; i += L) ring[i] = 0.0f;
    dev::wave_lds_fence();

    // frame k: 15 samples per lane, x[origin + hl + L m] of the half's stream;
    // samples outside [0, T) read 0 (zero padding)
    auto load_frame = [&](float (&f)[E], int origin) {
        if (HALVES == 1 || (origin >= 0 && origin + N <= a.T)) {  // uniform: both halves share k and T
            const int v = (xo + origin + hl) * 4;  // at N = 960 the range check does the padding
#pragma unroll
            for (int m = 0; m < E; ++m) f[m] = dev::bload1(rx, v + m * (4 * L), 0);
        } else {
#pragma unroll
            for (int m = 0; m < E; ++m) {
                const int t = origin + hl + L * m;
                const int v = (t >= 0 && t < a.T) ? (xo + t) * 4 : 0x7ffffff0;
                f[m] = dev::bload1(rx, v, 0);
            }
        }
    };
    bool bad = false;
    auto check = [&](const float (&f)[E]) {
        uint32_t mx = 0u, mn = ~0u;
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const uint32_t w = __builtin_bit_cast(uint32_t, f[m]) & 0x7fffffffu;
            mx = max(mx, w);
            mn = min(mn, w - 1u);
        }
        bad |= (mx > xhi_b) | (mn < xlo_b - 1u);
    };
    // push one frame's inverse output into the ring at block k's position: the
    // 1/N scale, the synthesis window and the gain folded into one factor per tap,
    // fma(v, ws / N g, ring) (one rounding where the staged path's o = v / N,
    // fma(fma(o, w, 0), g, acc) has three: inside the FFT tolerance; a flagged
    // stream is redone whole by the per-frame walker, so no walker has to agree)
    auto push = [&](const float (&p)[E], const float (&wg)[E], int k) {
        const int base = k * H + hl;  // k H < 2^27 (host-checked)
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int pos = (base + L * m) & RM;
            ring[pos] = __builtin_fmaf(p[m], wg[m], ring[pos]);
        }
        dev::wave_lds_fence();
    };
    // produce(H) of block k: ring / den, clear; stored when k >= f0.  The quotient
    // is IEEE's: Markstein's correction with RN(1/den) when the plan's divisors
    // allow it (den in [2^-40, 2^40]) and the sums are 0 or in [2^-64, 2^64]
    // (frexp exponents in [-63, 65]; a walk with any other sum is flagged and its
    // stream redone by the per-frame walker), else the division itself.
    const float2* const dr2 = reinterpret_cast<const float2*>(a.t.den_rden);
    // buffer loads of the {den, 1/den} pairs: the block's base in the scalar
    // offset, rows as immediate offsets (no per-row 64-bit addresses); rows past
    // the table read 0, unused
    const __amdgpu_buffer_rsrc_t rden = dev::make_rsrc(dr2, uint32_t(ring_blocks * H) * 8u);
    auto produce = [&](int k) {
        const int base = k * H;
        const int dbase = (k % ring_blocks) * H;
        const __amdgpu_buffer_rsrc_t rk = k >= f0 ? ry : ry_null;
        if (dr2) {
            // groups of 4 rows whose divisor loads issue together: a divisor load
            // waits on every earlier store too (one vmcnt counter), so a block pays
            // ceil(H / 4L) such waits instead of one per row
            for (int j0 = hl; j0 < H; j0 += 4 * L) {
                float2 d[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) d[i] = dev::bload2(rden, (j0 + L * i) * 8, dbase * 8);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int j = j0 + L * i;
                    if (j < H) {
                        const int pos = (base + j) & RM;
                        const float v = ring[pos];
                        ring[pos] = 0.0f;
                        const float o = mk_div(v, d[i].x, d[i].y);
                        bad |= uint32_t(__builtin_amdgcn_frexp_expf(v) + 63) > 128u;  // exponent outside [-63, 65]
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o), rk,
                                                              (yo + base + j) * 4, 0, 0);
                    }
                }
            }
        } else {
            for (int j = hl; j < H; j += L) {
                const int pos = (base + j) & RM;
                const float v = ring[pos];
                ring[pos] = 0.0f;
                const float o = v / a.t.den[dbase + j];
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o), rk, (yo + base + j) * 4, 0, 0);
            }
        }
        dev::wave_lds_fence();
    };
    // H <= 4 L (960/240, 480/120, every hop up to N/4): a block is at most 4 rows
    // of the walk, so both blocks' {den, 1/den} pairs are fetched before the pushes.
    // The row loop this replaces waited on vmcnt(0) at every row's divisor load,
    // which on gfx950 also drains the earlier rows' stores: one store round trip
    // per row (produce above still pays one per group of 4 rows).
    // At L = 32 the halves need the same divisors: half h fetches rows h and 2 + h
    // (JF = 2 pairs per block), a permlane32 swap hands each half the other's rows.
    constexpr int JD = 4, JF = L == 64 ? 4 : 2;
    auto den_fetch = [&](int k, float2 (&d)[JF]) {
        const int dbase = (k % ring_blocks) * H;
#pragma unroll
        for (int q = 0; q < JF; ++q)
            d[q] = dev::bload2(rden, (hl + L * (L == 64 ? q : 2 * q + half)) * 8, dbase * 8);
    };
    auto produce_pre = [&](int k, const float2 (&d)[JF]) {
        const int base = k * H;
        const __amdgpu_buffer_rsrc_t rk = k >= f0 ? ry : ry_null;
        float2 dd[JD];
        if constexpr (L == 64) {
#pragma unroll
            for (int i = 0; i < JD; ++i) dd[i] = d[i];
        } else {
#pragma unroll
            for (int q = 0; q < JF; ++q) {  // lower half: row 2q -> a, upper half: row 2q+1 -> b
                float ax = d[q].x, bx = d[q].x, ay = d[q].y, by = d[q].y;
                dev::swap_f(ax, bx, true);
                dev::swap_f(ay, by, true);
                dd[2 * q] = float2{ax, ay};
                dd[2 * q + 1] = float2{bx, by};
            }
        }
#pragma unroll
        for (int i = 0; i < JD; ++i) {
            const int j = hl + L * i;
            if (j < H) {
                const int pos = (base + j) & RM;
                const float v = ring[pos];
                ring[pos] = 0.0f;
                const float o = mk_div(v, dd[i].x, dd[i].y);
                bad |= uint32_t(__builtin_amdgcn_frexp_expf(v) + 63) > 128u;  // exponent outside [-63, 65]
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o), rk, (yo + base + j) * 4, 0, 0);
            }
        }
        dev::wave_lds_fence();
    };

    float fa[E], fb[E];
    load_frame(fa, fs * H - a.pad);
    load_frame(fb, (fs + 1) * H - a.pad);
    for (int k = fs; k < f1; k += 2) {
        check(fa);
        check(fb);
        const bool partner = k + 1 < a.F;  // frame k+1 past the last: imaginary part 0
        dev::pc v[16];
#pragma unroll
        for (int m4 = 0; m4 < 4; ++m4) {
            float wv[4];
            win4(wa4, war, m4, wv);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int m = 4 * m4 + q;
                if (m < E) v[m] = dev::pc_mk(fa[m] * wv[q], partner ? fb[m] * wv[q] : 0.0f);
            }
        }
        v[15] = dev::pc_mk(0.0f, 0.0f);
        // the next pair's frames, in flight during this pair's transforms
        load_frame(fa, (k + 2) * H - a.pad);
        load_frame(fb, (k + 3) * H - a.pad);
        P15<L>::fwd(v, buf, tw, lane);
        if constexpr (HAS_GAIN) {  // real gain, symmetric over the N bins (L2-resident table)
#pragma unroll
            for (int d = 0; d < 16; ++d) {
                const int kb = L == 64 ? dev::pair15_bin(lane, d) : dev::pair15h_bin(lane, d);  // <= N
                v[d] = v[d] * a.t.gain[kb <= N / 2 ? kb : N - kb];
            }
        }
        P15<L>::inv(v, buf, tw, lane);
        // the output sanitize acts on o = v / N below 1e-30, i.e. on |v| < 1e-30 N =
        // 2^-89.75 (N = 960) / 2^-90.75 (480): frexp exponents <= -89 / -90 (|v| <
        // 2^-89 / 2^-90) flag the walk -- every such v and a few harmless others.
        // (screened: fft_pair.h out_min_exp_screened; the window-edge taps n < L and
        // n >= N - L sit in registers 0 and E-1)
        static_assert(N == 960 || N == 480, "threshold exponent");
        constexpr int kSanExp = N == 960 ? -89 : -90;
        bad |= dev::out_min_exp_screened<E>(v, N == 960 ? 0x1p-89f : 0x1p-90f) <= kSanExp;
        float p[E], wg[E];
#pragma unroll
        for (int m4 = 0; m4 < 4; ++m4) {
            float wv[4];
            win4(ws4, wsr, m4, wv);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int m = 4 * m4 + q;
                if (m < E) {
                    wg[m] = wv[q];
                    p[m] = v[m].x;
                }
            }
        }
        if constexpr (DPRE) {
            // block k's divisors in flight during its push, block k+1's issued before
            // block k's stores (waiting for them does not drain the stores); the sched
            // barrier keeps d1's loads below the push (register pressure: 166-168
            // VGPRs at L = 64, no spill)
            float2 d0[JF], d1[JF];
            if constexpr (L == 64) den_fetch(k, d0);
            push(p, wg, k);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (L != 64) den_fetch(k, d0);  // L = 32: after the push (167 VGPRs before)
            den_fetch(k + 1, d1);
            produce_pre(k, d0);
#pragma unroll
            for (int m = 0; m < E; ++m) p[m] = v[m].y;
            push(p, wg, k + 1);
            if (k + 1 < f1) produce_pre(k + 1, d1);
        } else {
            push(p, wg, k);
            produce(k);
#pragma unroll
            for (int m = 0; m < E; ++m) p[m] = v[m].y;
            push(p, wg, k + 1);
            if (k + 1 < f1) produce(k + 1);
        }
    }
    // flag bit h: the stream of half h redoes (a stream's bits depend on its samples only)
    const uint64_t bal = __builtin_amdgcn_ballot_w64(bad);
    const uint32_t fl = HALVES == 1 ? (bal != 0 ? 1u : 0u)
                                    : ((bal & 0xffffffffull) != 0 ? 1u : 0u) | ((bal >> 32) != 0 ? 2u : 0u);
    if (lane == 0) a.t.pflags[gw] = fl;
}

}  // namespace fk

bool pair15_supported(int n, int h, int ring_len) {
    if (n != 960 && n != 480) return false;
    if (h < 32 || h > n || ring_len % h != 0) return false;
    const size_t lds = n == 960 ? fk::p15_lds<64>(h, fk::kP15Waves) : fk::p15_lds<32>(h, fk::kP15Waves);
    return lds <= 80 * 1024;
}

hipError_t launch_pair15(const Geometry& g, const DevTables& t, const float* x, float* y, int n_streams,
                         int64_t T, int64_t ld_x, int64_t ld_y, int64_t F, int64_t out_len, int* n_chunks,
                         int* streams_per_walk, hipStream_t stream) {
    using namespace fk;
    static const int venv = [] {
        const char* e = ab_env("CRLOT_P15_VARIANT");
        const int v = e ? std::atoi(e) : -1;
        return v >= 0 && v < 5 ? v : -1;
    }();
    // measured (960/240, 480/120 x 1024 streams): 4 walks with the windows in
    // registers, 12 waves per CU (174k / 173.5k Msamples/s) vs 4 walks with LDS
    // windows, 8 waves per CU (148k / 140.5k) and 2 walks (117k / 148.5k)
    const int v = venv >= 0 && !t.gain ? venv : 4;
    const bool wreg = kP15Shapes[v].wreg && !t.gain;  // the gain walker keeps the windows in LDS
    const int W = kP15Shapes[v].w;
    if (!pair15_supported(g.n, g.h, g.ring_len) || !t.ptw || !t.pflags || F <= 0 || n_streams <= 0 ||
        T >= (int64_t(1) << 27) || out_len >= (int64_t(1) << 27) || ld_x >= (int64_t(1) << 27) ||
        ld_y >= (int64_t(1) << 27))
        return hipErrorInvalidValue;
    const int halves = g.n == 480 ? 2 : 1;
    // H <= 4 L: a block is at most 4 rows of the walk, its divisors are fetched
    // ahead (CRLOT_P15_DPRE=0 keeps the row loop, A/B)
    static const bool dpre_env = [] {
        const char* e = ab_env("CRLOT_P15_DPRE");
        return !(e && e[0] == '0');
    }();
    const bool dpre = dpre_env && t.den_rden != nullptr && g.h <= 4 * (g.n / 15);
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
    a.hop = g.h;
    a.ring_blocks = g.ring_len / g.h;
    a.pad = g.pad;
    a.pad_mode = g.pad_mode;
    a.inv_n = g.inv_n;
    a.gain = g.gain;
    // chunks: about two resident rounds of walkers, each >= 48 frames
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    const size_t lds = g.n == 960 ? p15_lds<64>(g.h, W, wreg) : p15_lds<32>(g.h, W, wreg);
    const int64_t wpc = std::min<int64_t>(W * int64_t(160 * 1024 / lds), 4 * kP15Shapes[v].wpe);  // waves per CU
    const int64_t resident = int64_t(cus) * std::max<int64_t>(W, wpc);
    const int64_t units = (n_streams + halves - 1) / halves;
    const int64_t n = chunks_or(std::max<int64_t>(1, std::min<int64_t>(F / 48, (2 * resident + units - 1) / units)), F);
    a.M = int((F + n - 1) / n);
    a.n_chunks = int((F + a.M - 1) / a.M);
    const int64_t waves = units * a.n_chunks;
    if (t.pflags_len < waves) return hipErrorInvalidValue;
    *n_chunks = a.n_chunks;
    *streams_per_walk = halves;
    note_chunks(a.n_chunks);
    hipError_t e = hipSuccess;
    auto go = [&](auto k, int w) {
        if ((e = set_lds(k, lds)) != hipSuccess) return;
        note_launch(CRLOT_K_PAIR15, (waves + w - 1) / w);
        hipLaunchKernelGGL(k, dim3(unsigned((waves + w - 1) / w)), dim3(64 * w), lds, stream, a);
        e = hipGetLastError();
    };
    switch (v) {
        case 1: g.n == 960 ? go(k_pair15_hot<64, 2, true, 2>, 2) : go(k_pair15_hot<32, 2, true, 2>, 2); break;
        case 2: g.n == 960 ? go(k_pair15_hot<64, 4, false, 3>, 4) : go(k_pair15_hot<32, 4, false, 3>, 4); break;
        case 3: g.n == 960 ? go(k_pair15_hot<64, 2, false, 3>, 2) : go(k_pair15_hot<32, 2, false, 3>, 2); break;
        case 4:
            if (t.gain && dpre)  // the spectral hook: 4 walks, the windows in LDS (the gain loads need the registers)
                g.n == 960 ? go(k_pair15_hot<64, 4, false, 3, true, true>, 4)
                           : go(k_pair15_hot<32, 4, false, 3, true, true>, 4);
            else if (t.gain)
                g.n == 960 ? go(k_pair15_hot<64, 4, false, 3, true>, 4) : go(k_pair15_hot<32, 4, false, 3, true>, 4);
            else if (dpre)
                g.n == 960 ? go(k_pair15_hot<64, 4, true, 3, false, true>, 4)
                           : go(k_pair15_hot<32, 4, true, 3, false, true>, 4);
            else
                g.n == 960 ? go(k_pair15_hot<64, 4, true, 3>, 4) : go(k_pair15_hot<32, 4, true, 3>, 4);
            break;
        default: g.n == 960 ? go(k_pair15_hot<64, 5, false, 3>, 5) : go(k_pair15_hot<32, 5, false, 3>, 5); break;
    }
    return e;
}

// [14][L] of W_N^{l k1} (N = 15 L), then at L = 64 [3][16] of W64^{b c}, at
// L = 32 [16] of W32^{b}
std::vector<float> build_pair15_twiddles(int n) {
    const int L = n / 15;
    std::vector<float> t;
    auto put = [&](double ph) {
        t.push_back(float(std::cos(ph)));
        t.push_back(float(std::sin(ph)));
    };
    for (int k1 = 1; k1 < 15; ++k1)
        for (int l = 0; l < L; ++l) put(-2.0 * M_PI * double(l * k1) / double(n));
    if (L == 64) {
        for (int c = 1; c < 4; ++c)
            for (int b = 0; b < 16; ++b) put(-2.0 * M_PI * double(b * c) / 64.0);
    } else {
        for (int b = 0; b < 16; ++b) put(-2.0 * M_PI * double(b) / 32.0);
    }
    return t;
}

}  // namespace crlot
