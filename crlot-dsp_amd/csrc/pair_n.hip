// pair_n.hip -- K_pairN: the frame-pair round trip for frame sizes with small
// prime factors outside the register-resident kernels: 882 and 1764 (20 / 40 ms
// at 44.1 kHz), 1920 (40 ms at 48 kHz), 1000, 640, 400, 320.  One transform per
// wave, or per two waves at 1764 and 1920.
//
// Frames 2j and 2j+1 of a stream travel as one N-point complex transform,
// z = x_2j w + i x_2j+1 w (as K_pair15 and the power-of-two pair kernels do:
// for a real, bin-symmetric gain the round trip's real and imaginary parts are
// the two frames' round trips), through fft_pairn.h's compile-time Stockham
// passes in one LDS buffer per wave.  The walk is K_pair15's (pair_any.hip):
// each pair loads its two frames whole (ceil(N/64) dwords per lane each,
// issued during the previous pair's transforms), the overlap-add runs in an
// LDS ring of the power of two >= H ceil(N/H) floats -- push frame k, produce
// block k, push frame k+1, produce block k+1, the reference's streaming-
// interleaved order -- and o = v (1/N) after the inverse (kissfft_adapter.cc:154).
//
// Paired regime only: a sample outside [px_lo, px_hi] (or NaN / Inf), an
// output below the sanitize threshold or a sum outside Markstein's range flags
// the walk; a stream with any flagged walk is recomputed whole by the per-frame
// walker (k_stft_ola_any), so a stream's bits depend only on its own samples.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "fft_pairn.h"
#include "fused_common.h"

namespace crlot {
namespace fk {

namespace {

// OLA ring floats of a walk: the live span H ceil(N/H), rounded up to a power of
// two (a position wraps with one AND) unless lean (one compare and subtract)
__host__ __device__ inline int pn_ring(int n, int h, bool lean) {
    const int span = h * ((n + h - 1) / h);
    if (lean) return span;
    int r = 1;
    while (r < span) r <<= 1;
    return r;
}

// LDS: [twiddles tw_len cf][wa N f][ws N f] | per wave [buffer N cf][ring RL f]
// CRLOT_PN_PLAN=V (A/B): the alternative radix list V of fft_pairn.h for 882 / 1764
int pn_variant(int n) {
    static const int v = [] {
        const char* e = ab_env("CRLOT_PN_PLAN");
        const int x = e ? std::atoi(e) : 0;
        return x >= 0 && x < 4 ? x : 0;
    }();
    return (n == 882 || n == 1764 || n == 960 || n == 480 || n == 1920) ? v : 0;
}
// CRLOT_PN_WIDE=0/1 (A/B): one or two waves per transform at 882 / 1764 (default
// below: two at 1764)
int pn_halves(int n) {
    static const int w = [] {
        const char* e = ab_env("CRLOT_PN_WIDE");
        return e ? (e[0] == '1' ? 2 : 1) : 0;
    }();
    if (n != 882 && n != 1764 && n != 960 && n != 1920) return 1;
    return w ? w : (n >= 1500 ? 2 : 1);
}
// CRLOT_PN_LEAN=0/1 (A/B): the two-wave walk's LDS without the windows and with an
// exact-size ring (one more walk per CU at 1764)
bool pn_lean(int n) {
    static const int l = [] {
        const char* e = ab_env("CRLOT_PN_LEAN");
        return e ? (e[0] == '1' ? 1 : 0) : -1;
    }();
    if (pn_halves(n) != 2) return false;
    return l == 1;  // measured at 1764/441: 62.7k lean vs 98.0k (the windows and the prefetch matter more)
}
int pn_key(int n) {
    return n + 100000 * pn_variant(n) + 1000000 * (pn_halves(n) - 1) + 10000000 * (pn_lean(n) ? 1 : 0);
}
// N = 1764 as two 882-point halves on two waves (tools/experiments/pairn_dit.inc,
// -DCRLOT_PN_DIT_EXPERIMENT builds only: measured 14 % slower than the two-wave
// 1764-point transform)
constexpr int kDitHalf = 882;  // the half transform's plan key (one wave, fft_pairn.h)
bool pn_dit(int n) {
#ifdef CRLOT_PN_DIT_EXPERIMENT
    return n == 2 * kDitHalf && pn_halves(n) == 2 && !pn_lean(n) && pn_variant(n) == 0;
#else
    (void)n;
    return false;
#endif
}
size_t pn_tables(int n) {
    if (pn_dit(n))  // half-plan twiddles | W1764^k (k < 882) | windows
        return sizeof(dev::pc) * size_t(dev::pn_factor(kDitHalf).tw_len + kDitHalf) + sizeof(float) * 2 * size_t(n);
    return sizeof(dev::pc) * size_t(dev::pn_factor(pn_key(n)).tw_len) + (pn_lean(n) ? 0 : sizeof(float) * 2 * size_t(n));
}
size_t pn_per_walk(int n, int h) {
    return sizeof(dev::pc) * size_t(n) + sizeof(float) * size_t(pn_ring(n, h, pn_lean(n)));
}

// walks per workgroup (one workgroup per CU): as many as the LDS holds, <= 16 waves
int pn_walks(int n, int h) {
    const size_t budget = 160 * 1024;
    const size_t t = pn_tables(n), w = pn_per_walk(n, h);
    if (t + w > budget) return 0;
    return int(std::min<size_t>(16 / pn_halves(n), (budget - t) / w));
}

}  // namespace

// register budget per size: waves per SIMD (the launch puts at most 4 x WPE waves
// in its one workgroup per CU)
constexpr int pn_wpe(int key) {
    const int n = key % 100000, halves = 1 + (key % 10000000) / 1000000;
    if (key >= 10000000) return 4;  // lean: 7 walks (14 waves) per CU at 1764
    return n <= 400 * halves ? 4 : n <= 1000 * halves ? 3 : 2;
}

// The frexp exponent bound of the output sanitize on an unscaled inverse output v
// of an N-point transform: |v| < 2^e for every v with |v / N| < 1e-30 (the
// reference's threshold), e = floor(log2(1e-30 N)) + 1, with room for the
// roundings of v / N (a few more values flag a walk, harmlessly)
constexpr int pn_san_exp(int n) {
    double t = 1e-30 * n;
    int e = 0;
    while (t < 1.0) {
        t *= 2.0;
        --e;
    }
    return t * (1.0 + 0x1p-20) < 2.0 ? e + 1 : e + 2;
}
static_assert(pn_san_exp(1024) == -89 && pn_san_exp(960) == -89 && pn_san_exp(480) == -90, "san exp");

template <int K, bool HAS_GAIN>  // K: plan key (fft_pairn.h pn_factor), N = K % 100000
__global__ __launch_bounds__(256 * pn_wpe(K)) __attribute__((amdgpu_waves_per_eu(pn_wpe(K))))
void k_pairn(const FusedArgs a) {
    constexpr int N = K % 100000;
    constexpr int L = dev::pn_lanes(K), HALVES = L / 64;  // lanes (waves) per transform
    constexpr int E = (N + L - 1) / L;      // natural-order rows per lane (the last partial)
    constexpr int LAST = N - L * (E - 1);   // lanes of the last row
    constexpr bool LEAN = K >= 10000000;
    constexpr dev::PnFac FAC = dev::pn_factor(K);
    static_assert(FAC.rest == 1, "N must factor into 2, 3, 5, 7");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int t = threadIdx.x % L, pw = __builtin_amdgcn_readfirstlane(threadIdx.x / L);  // lane / walk in the workgroup
    const int half = __builtin_amdgcn_readfirstlane((threadIdx.x >> 6) % HALVES);
    const int PPW = int(blockDim.x) / L;  // walks per workgroup
    const int H = a.hop;
    const int RL = pn_ring(N, H, LEAN), RM = RL - 1;
    // ring position of block offset o (< N + H) past frame k's start kb = (k H) mod RL
    auto rpos = [&](int kb, int o) {
        if constexpr (LEAN) {
            int p = kb + o;
            p -= p >= RL ? RL : 0;
            return p >= RL ? p - RL : p;
        } else {
            return (kb + o) & RM;
        }
    };
    auto rbase = [&](int k) { return LEAN ? (k * H) % RL : k * H; };
    const int NB = (N + H - 1) / H;
    dev::pc* tw = reinterpret_cast<dev::pc*>(smem);
    float* wl = reinterpret_cast<float*>(tw + FAC.tw_len);  // LDS windows (not lean)
    float* wend = LEAN ? wl : wl + 2 * N;
    const float* wa = LEAN ? a.t.wa : wl;
    const float* ws = LEAN ? a.t.ws : wl + N;
    dev::pc* buf = reinterpret_cast<dev::pc*>(wend) + size_t(pw) * N;
    float* ring = reinterpret_cast<float*>(reinterpret_cast<dev::pc*>(wend) + size_t(PPW) * N) + size_t(pw) * RL;
    {
        const dev::pc* g = reinterpret_cast<const dev::pc*>(a.t.ptw);
        for (int i = threadIdx.x; i < FAC.tw_len; i += blockDim.x) tw[i] = g[i];
        if constexpr (!LEAN)
            for (int i = threadIdx.x; i < N; i += blockDim.x) {
                wl[i] = a.t.wa[i];
                wl[N + i] = a.t.ws[i] * a.inv_n * a.gain;  // (1/N, ws and g folded: the pushes below)
            }
    }
    __syncthreads();
    const int gw = blockIdx.x * PPW + pw;  // this walk
    if (gw >= a.n_streams * a.n_chunks) return;  // (both waves of a walk together)
    const int s = gw / a.n_chunks, c = gw - s * a.n_chunks;
    const int f0 = c * a.M;
    const int f1 = min(a.F, f0 + a.M);
    const int fs = max(0, f0 - (NB - 1)) & ~1;  // pairs start on even frames
    const __amdgpu_buffer_rsrc_t rx = dev::make_rsrc(a.x + int64_t(s) * a.ld_x, uint32_t(a.T) * 4u);
    const __amdgpu_buffer_rsrc_t ry = dev::make_rsrc(a.y + int64_t(s) * a.ld_y, uint32_t(a.out_len) * 4u);
    const __amdgpu_buffer_rsrc_t ry_null = dev::make_rsrc(a.y, 0u);
    const float g = a.gain, inv_n = a.inv_n;
    const int ring_blocks = a.ring_blocks;
    const uint32_t xlo_b = __builtin_bit_cast(uint32_t, a.t.px_lo), xhi_b = __builtin_bit_cast(uint32_t, a.t.px_hi);
    auto valid = [&](int m) { return m + 1 < E || t < LAST; };

    for (int i = t; i < RL; i += L) ring[i] = 0.0f;
    dev::pn_fence<K>();

    using P0 = dev::PnPass<K, 0>;
    using PL = dev::PnPass<K, FAC.n - 1>;
    // frame k as the first pass reads it: register [it][q] of lane t holds sample
    // j + q M0 (j = t + L it); samples outside [0, T) read 0 (the descriptor's
    // range check; a negative offset wraps past it)
    auto load_frame = [&](float (&f)[P0::ITS][P0::R], int origin) {
#pragma unroll
        for (int it = 0; it < P0::ITS; ++it) {
            const int j = t + L * it;
#pragma unroll
            for (int q = 0; q < P0::R; ++q) {
                const int v = P0::live(it, j) ? (origin + j + q * P0::M) * 4 : 0x7ffffff0;
                f[it][q] = dev::bload1(rx, v, 0);
            }
        }
    };
    bool bad = false;
    auto check = [&](const float (&f)[P0::ITS][P0::R]) {
        uint32_t mx = 0u, mn = ~0u;
#pragma unroll
        for (int it = 0; it < P0::ITS; ++it)
#pragma unroll
            for (int q = 0; q < P0::R; ++q) {
                const uint32_t w = __builtin_bit_cast(uint32_t, f[it][q]) & 0x7fffffffu;
                mx = max(mx, w);
                mn = min(mn, w - 1u);
            }
        bad |= (mx > xhi_b) | (mn < xlo_b - 1u);
    };
    // produce(H) of block k: ring / den (Markstein with {den, 1/den} when the plan
    // allows it, sums outside [2^-64, 2^64] flag the walk; else IEEE), clear
    const float2* const dr2 = reinterpret_cast<const float2*>(a.t.den_rden);
    const __amdgpu_buffer_rsrc_t rden = dev::make_rsrc(dr2, uint32_t(ring_blocks * H) * 8u);
    auto produce = [&](int k) {
        const int base = k * H, kb = rbase(k);
        const int dbase = (k % ring_blocks) * H;
        const __amdgpu_buffer_rsrc_t rk = k >= f0 ? ry : ry_null;
        if (dr2) {
            for (int j0 = t; j0 < H; j0 += 4 * L) {
                float2 d[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) d[i] = dev::bload2(rden, (j0 + L * i) * 8, dbase * 8);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int j = j0 + L * i;
                    if (j < H) {
                        const int pos = rpos(kb, j);
                        const float v = ring[pos];
                        ring[pos] = 0.0f;
                        const float o = mk_div(v, d[i].x, d[i].y);
                        bad |= uint32_t(__builtin_amdgcn_frexp_expf(v) + 63) > 128u;
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o), rk, (base + j) * 4, 0, 0);
                    }
                }
            }
        } else {
            for (int j = t; j < H; j += L) {
                const int pos = rpos(kb, j);
                const float v = ring[pos];
                ring[pos] = 0.0f;
                const float o = v / a.t.den[dbase + j];
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o), rk, (base + j) * 4, 0, 0);
            }
        }
        // no fence: the next push (frame k+1) adds only to blocks after k, and the
        // clears are ordered before any later reuse of their positions by the
        // fences of the next pair's transforms
    };

    // the next pair's frames load during this pair's transforms, except at 1764
    // points: 56 more VGPRs than the walk has (measured: the compiler spills them)
    constexpr bool PF = N < 1500 || (L == 128 && !LEAN);
    float fa[P0::ITS][P0::R], fb[P0::ITS][P0::R];
    if constexpr (PF) {
        load_frame(fa, fs * H - a.pad);
        load_frame(fb, (fs + 1) * H - a.pad);
    }
    for (int k = fs; k < f1; k += 2) {
        if constexpr (!PF) {
            load_frame(fa, k * H - a.pad);
            load_frame(fb, (k + 1) * H - a.pad);
        }
        check(fa);
        check(fb);
        const bool partner = k + 1 < a.F;  // frame k+1 past the last: imaginary part 0
        const int ln = dev::pn_opaque(t);
        {
            // the first forward pass straight from the frame registers
            dev::pc x[P0::ITS][P0::R];
#pragma unroll
            for (int it = 0; it < P0::ITS; ++it) {
                const int j = P0::bf(ln, it);
#pragma unroll
                for (int q = 0; q < P0::R; ++q) {
                    const float w = wa[j + q * P0::M];
                    x[it][q] = dev::pc_mk(fa[it][q] * w, partner ? fb[it][q] * w : 0.0f);
                }
                dev::pn_bfly<false, K, 0>(x[it], tw, j);
            }
            if constexpr (PF) {  // the next pair's frames, in flight during this pair's transforms
                load_frame(fa, (k + 2) * H - a.pad);
                load_frame(fb, (k + 3) * H - a.pad);
            }
            dev::pn_pass_store<K, 0>(buf, ln, x);
            dev::pn_fence<K>();
        }
        dev::pn_passes<false, K, 1, FAC.n>(buf, tw, ln);
        if constexpr (HAS_GAIN) {  // real gain, symmetric over the N bins (L2-resident table)
#pragma unroll
            for (int m = 0; m < E; ++m) {
                if (valid(m)) {
                    const int n = ln + L * m;
                    buf[n] = buf[n] * a.t.gain[n <= N / 2 ? n : N - n];
                }
            }
            dev::pn_fence<K>();
        }
        dev::pn_passes<true, K, 0, FAC.n - 1>(buf, tw, ln);
        // the last inverse pass into registers, pushed from there: frame k the real
        // part, frame k+1 the imaginary part.  Lean walks: o = v (1/N), then o * ws,
        // fma(., g, ring); the output sanitize threshold 1e-30 = 2^-99.66: exponents
        // <= -99 flag the walk.  Otherwise 1/N, ws and g are one staged factor,
        // fma(v, ws / N g, ring) (one rounding for three: inside the FFT tolerance; a
        // flagged stream is redone whole by the per-frame walker), and the threshold
        // test acts on v: |v| < 2^kSanExp covers every |v / N| < 1e-30 (pn_san_exp)
        dev::pc y[PL::ITS][PL::R];
        dev::pn_pass_compute<true, K, FAC.n - 1>(buf, tw, ln, y);
        const int kb0 = rbase(k), kb1 = rbase(k + 1);
        constexpr int kSanExp = LEAN ? -99 : pn_san_exp(N);
        {
            int e = 0;
#pragma unroll
            for (int it = 0; it < PL::ITS; ++it) {
                const int j = ln + L * it;
                if (PL::live(it, j)) {
#pragma unroll
                    for (int q = 0; q < PL::R; ++q) {
                        if constexpr (LEAN) y[it][q] = y[it][q] * dev::pc{inv_n, inv_n};
                        e = min(e, min(__builtin_amdgcn_frexp_expf(y[it][q].x),
                                       __builtin_amdgcn_frexp_expf(y[it][q].y)));
                        const int n = PL::out(j, q);
                        const int pos = rpos(kb0, n);
                        ring[pos] = LEAN ? __builtin_fmaf(y[it][q].x * ws[n], g, ring[pos])
                                         : __builtin_fmaf(y[it][q].x, ws[n], ring[pos]);
                    }
                }
            }
            bad |= e <= kSanExp;
        }
        dev::pn_fence<K>();
        produce(k);
#pragma unroll
        for (int it = 0; it < PL::ITS; ++it) {
            const int j = ln + L * it;
            if (PL::live(it, j)) {
#pragma unroll
                for (int q = 0; q < PL::R; ++q) {
                    const int n = PL::out(j, q);
                    const int pos = rpos(kb1, n);
                    ring[pos] = LEAN ? __builtin_fmaf(y[it][q].y * ws[n], g, ring[pos])
                                     : __builtin_fmaf(y[it][q].y, ws[n], ring[pos]);
                }
            }
        }
        dev::pn_fence<K>();
        if (k + 1 < f1) produce(k + 1);
    }
    // one flag per wave: [stream][chunk][half] (the redo ORs a stream's flags)
    const uint64_t bal = __builtin_amdgcn_ballot_w64(bad);
    if (lane == 0) a.t.pflags[gw * HALVES + half] = bal != 0 ? 1u : 0u;
}

#ifdef CRLOT_PN_DIT_EXPERIMENT
#include "pairn_dit.inc"  // tools/experiments (`make experiments`)
#endif

namespace {
// the instantiated sizes
template <typename F>
bool pn_dispatch(int key, F&& f) {
    switch (key) {
        case 320: f(std::integral_constant<int, 320>{}); return true;
        case 400: f(std::integral_constant<int, 400>{}); return true;
        case 640: f(std::integral_constant<int, 640>{}); return true;
        case 882: f(std::integral_constant<int, 882>{}); return true;
        case 1000: f(std::integral_constant<int, 1000>{}); return true;
        case 1764: f(std::integral_constant<int, 1764>{}); return true;
        case 1000882: f(std::integral_constant<int, 1000882>{}); return true;
        case 1001764: f(std::integral_constant<int, 1001764>{}); return true;
        case 11001764: f(std::integral_constant<int, 11001764>{}); return true;
        case 1001920: f(std::integral_constant<int, 1001920>{}); return true;
#ifdef CRLOT_PN_15
        case 960: f(std::integral_constant<int, 960>{}); return true;
        case 480: f(std::integral_constant<int, 480>{}); return true;
        case 100960: f(std::integral_constant<int, 100960>{}); return true;
        case 200960: f(std::integral_constant<int, 200960>{}); return true;
        case 300960: f(std::integral_constant<int, 300960>{}); return true;
        case 100480: f(std::integral_constant<int, 100480>{}); return true;
        case 200480: f(std::integral_constant<int, 200480>{}); return true;
        case 300480: f(std::integral_constant<int, 300480>{}); return true;
        case 1101920: f(std::integral_constant<int, 1101920>{}); return true;
        case 1201920: f(std::integral_constant<int, 1201920>{}); return true;
#endif
#ifdef CRLOT_PN_VARIANTS
        case 100882: f(std::integral_constant<int, 100882>{}); return true;
        case 200882: f(std::integral_constant<int, 200882>{}); return true;
        case 300882: f(std::integral_constant<int, 300882>{}); return true;
        case 101764: f(std::integral_constant<int, 101764>{}); return true;
        case 201764: f(std::integral_constant<int, 201764>{}); return true;
        case 301764: f(std::integral_constant<int, 301764>{}); return true;
#endif
        default: return false;
    }
}
}  // namespace

}  // namespace fk

bool pairn_size(int n) {
    return fk::pn_dispatch(fk::pn_key(n), [](auto) {});
}

// K_pairN in place of K_pair15 at N = 960 / 480 (CRLOT_PN_OVER15=1, A/B builds
// with -DCRLOT_PN_15)
bool pairn_over_pair15(int n) {
    static const bool v = [] {
        const char* e = ab_env("CRLOT_PN_OVER15");
        return e && e[0] == '1';
    }();
    return v && (n == 960 || n == 480) && pairn_size(n);
}

bool pairn_supported(int n, int h, int ring_len) {
    if (!pairn_size(n)) return false;
    if (h < 32 || h > n || ring_len % h != 0) return false;
    return fk::pn_walks(n, h) >= 1;
}

hipError_t launch_pairn(const Geometry& g, const DevTables& t, const float* x, float* y, int n_streams, int64_t T,
                        int64_t ld_x, int64_t ld_y, int64_t F, int64_t out_len, int* n_chunks, hipStream_t stream) {
    using namespace fk;
    if (!pairn_supported(g.n, g.h, g.ring_len) || !t.ptw || !t.pflags || F <= 0 || n_streams <= 0 ||
        T >= (int64_t(1) << 27) || out_len >= (int64_t(1) << 27))
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
    a.hop = g.h;
    a.ring_blocks = g.ring_len / g.h;
    a.pad = g.pad;
    a.pad_mode = g.pad_mode;
    a.inv_n = g.inv_n;
    a.gain = g.gain;
    const int halves = pn_halves(g.n);
    const int walks = std::min(pn_walks(g.n, g.h), 4 * pn_wpe(pn_key(g.n)) / halves);  // per workgroup
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    // chunks: about two resident rounds of walkers, each >= 48 frames
    const int64_t resident = int64_t(cus) * walks;
    // (a forced chunking keeps a flag per wave within the F-per-stream flag rows)
    const int64_t n = chunks_or(std::max<int64_t>(1, std::min<int64_t>(F / 48, (2 * resident + n_streams - 1) / n_streams)),
                                std::max<int64_t>(1, F / halves));
    a.M = int((F + n - 1) / n);
    a.n_chunks = int((F + a.M - 1) / a.M);
    const int64_t total = int64_t(n_streams) * a.n_chunks;  // walks
    if (t.pflags_len < total * halves) return hipErrorInvalidValue;
    *n_chunks = a.n_chunks * halves;  // flags per stream (one per wave)
    note_chunks(a.n_chunks);
    const size_t lds = pn_tables(g.n) + size_t(walks) * pn_per_walk(g.n, g.h);
    hipError_t e = hipSuccess;
#ifdef CRLOT_PN_DIT_EXPERIMENT
    if (pn_dit(g.n)) {  // 1764 = 2 x 882 on two waves (k_pairn_dit)
        auto k = t.gain ? k_pairn_dit<true> : k_pairn_dit<false>;
        if ((e = set_lds(k, lds)) != hipSuccess) return e;
        note_launch(CRLOT_K_PAIRN, (total + walks - 1) / walks);
        hipLaunchKernelGGL(k, dim3(unsigned((total + walks - 1) / walks)), dim3(128 * walks), lds, stream, a);
        return hipGetLastError();
    }
#endif
    pn_dispatch(pn_key(g.n), [&](auto nc) {
        constexpr int NN = decltype(nc)::value;
        auto k = t.gain ? k_pairn<NN, true> : k_pairn<NN, false>;
        if ((e = set_lds(k, lds)) != hipSuccess) return;
        note_launch(CRLOT_K_PAIRN, (total + walks - 1) / walks);
        hipLaunchKernelGGL(k, dim3(unsigned((total + walks - 1) / walks)), dim3(64 * halves * walks), lds, stream, a);
        e = hipGetLastError();
    });
    return e;
}

// W_{ns r}^{q jm} per pass of fft_pairn.h's factorisation, float pairs
// (1764 by decimation in time: the 882-point plan's, then W1764^k for k < 882)
std::vector<float> build_pairn_twiddles(int n) {
    const bool dit = fk::pn_dit(n);
    const dev::PnFac f = dev::pn_factor(dit ? fk::kDitHalf : fk::pn_key(n));
    std::vector<float> t(2 * size_t(f.tw_len));
    if (dit)
        for (int k = 0; k < n / 2; ++k) {
            const double ph = -2.0 * M_PI * double(k) / double(n);
            t.push_back(float(std::cos(ph)));
            t.push_back(float(std::sin(ph)));
        }
    for (int i = 0; i < f.n; ++i)
        for (int q = 1; q < f.r[i]; ++q)
            for (int jm = 0; jm < f.ns[i]; ++jm) {
                const double ph = -2.0 * M_PI * double(q) * double(jm) / double(f.ns[i] * f.r[i]);
                const size_t at = 2 * size_t(f.off[i] + (q - 1) * f.ns[i] + jm);
                t[at] = float(std::cos(ph));
                t[at + 1] = float(std::sin(ph));
            }
    return t;
}

}  // namespace crlot
