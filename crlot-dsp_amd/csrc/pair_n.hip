// pair_n.hip -- K_pairN: the frame-pair round trip for frame sizes with small
// prime factors outside the register-resident kernels: 882 and 1764 (20 / 40 ms
// at 44.1 kHz), 1000, 640, 400, 320.  One transform per wave.
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

__host__ __device__ inline int pn_ring(int n, int h) {
    const int span = h * ((n + h - 1) / h);
    int r = 1;
    while (r < span) r <<= 1;
    return r;
}

// LDS: [twiddles tw_len cf][wa N f][ws N f] | per wave [buffer N cf][ring RL f]
size_t pn_tables(int n) { return sizeof(dev::pc) * size_t(dev::pn_factor(n).tw_len) + sizeof(float) * 2 * size_t(n); }
size_t pn_per_wave(int n, int h) { return sizeof(dev::pc) * size_t(n) + sizeof(float) * size_t(pn_ring(n, h)); }

// waves per workgroup (one workgroup per CU): as many walks as the LDS holds, <= 16
int pn_waves(int n, int h) {
    const size_t budget = 160 * 1024;
    const size_t t = pn_tables(n), w = pn_per_wave(n, h);
    if (t + w > budget) return 0;
    return int(std::min<size_t>(16, (budget - t) / w));
}

}  // namespace

// register budget per size: waves per SIMD (the launch puts at most 4 x WPE waves
// in its one workgroup per CU)
constexpr int pn_wpe(int n) { return n <= 640 ? 4 : n <= 1000 ? 3 : 2; }

template <int N, bool HAS_GAIN>
__global__ __launch_bounds__(256 * pn_wpe(N)) __attribute__((amdgpu_waves_per_eu(pn_wpe(N))))
void k_pairn(const FusedArgs a) {
    constexpr int E = (N + 63) / 64;  // rows per lane (the last one partial when N % 64 != 0)
    constexpr int LAST = N - 64 * (E - 1);  // lanes of the last row
    constexpr dev::PnFac FAC = dev::pn_factor(N);
    static_assert(FAC.rest == 1, "N must factor into 2, 3, 5, 7");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int W = blockDim.x >> 6;
    const int H = a.hop;
    const int RL = pn_ring(N, H), RM = RL - 1;
    const int NB = (N + H - 1) / H;
    dev::pc* tw = reinterpret_cast<dev::pc*>(smem);
    float* wa = reinterpret_cast<float*>(tw + FAC.tw_len);
    float* ws = wa + N;
    dev::pc* buf = reinterpret_cast<dev::pc*>(ws + N) + size_t(wave) * N;
    float* ring = reinterpret_cast<float*>(reinterpret_cast<dev::pc*>(ws + N) + size_t(W) * N) + size_t(wave) * RL;
    {
        const dev::pc* g = reinterpret_cast<const dev::pc*>(a.t.ptw);
        for (int i = threadIdx.x; i < FAC.tw_len; i += blockDim.x) tw[i] = g[i];
        for (int i = threadIdx.x; i < N; i += blockDim.x) {
            wa[i] = a.t.wa[i];
            ws[i] = a.t.ws[i];
        }
    }
    __syncthreads();
    const int gw = blockIdx.x * W + wave;
    if (gw >= a.n_streams * a.n_chunks) return;
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
    auto valid = [&](int m) { return m + 1 < E || lane < LAST; };

    for (int i = lane; i < RL; i += 64) ring[i] = 0.0f;
    dev::wave_lds_fence();

    // frame k: x[origin + lane + 64 m] (samples outside [0, T) read 0: the
    // descriptor's range check, a negative offset wraps past it)
    auto load_frame = [&](float (&f)[E], int origin) {
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int v = valid(m) ? (origin + lane + 64 * m) * 4 : 0x7ffffff0;
            f[m] = dev::bload1(rx, v, 0);
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
    // produce(H) of block k: ring / den (Markstein with {den, 1/den} when the plan
    // allows it, sums outside [2^-64, 2^64] flag the walk; else IEEE), clear
    const float2* const dr2 = reinterpret_cast<const float2*>(a.t.den_rden);
    const __amdgpu_buffer_rsrc_t rden = dev::make_rsrc(dr2, uint32_t(ring_blocks * H) * 8u);
    auto produce = [&](int k) {
        const int base = k * H;
        const int dbase = (k % ring_blocks) * H;
        const __amdgpu_buffer_rsrc_t rk = k >= f0 ? ry : ry_null;
        if (dr2) {
            for (int j0 = lane; j0 < H; j0 += 4 * 64) {
                float2 d[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) d[i] = dev::bload2(rden, (j0 + 64 * i) * 8, dbase * 8);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int j = j0 + 64 * i;
                    if (j < H) {
                        const int pos = (base + j) & RM;
                        const float v = ring[pos];
                        ring[pos] = 0.0f;
                        const float o = mk_div(v, d[i].x, d[i].y);
                        bad |= uint32_t(__builtin_amdgcn_frexp_expf(v) + 63) > 128u;
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o), rk, (base + j) * 4, 0, 0);
                    }
                }
            }
        } else {
            for (int j = lane; j < H; j += 64) {
                const int pos = (base + j) & RM;
                const float v = ring[pos];
                ring[pos] = 0.0f;
                const float o = v / a.t.den[dbase + j];
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o), rk, (base + j) * 4, 0, 0);
            }
        }
        dev::wave_lds_fence();
    };

    float fa[E], fb[E];
#ifndef CRLOT_PN_NOPREFETCH
    load_frame(fa, fs * H - a.pad);
    load_frame(fb, (fs + 1) * H - a.pad);
#endif
    for (int k = fs; k < f1; k += 2) {
#ifdef CRLOT_PN_NOPREFETCH
        load_frame(fa, k * H - a.pad);
        load_frame(fb, (k + 1) * H - a.pad);
#endif
        check(fa);
        check(fb);
        const bool partner = k + 1 < a.F;  // frame k+1 past the last: imaginary part 0
#pragma unroll
        for (int m = 0; m < E; ++m) {
            if (valid(m)) {
                const int n = lane + 64 * m;
                const float w = wa[n];
                buf[n] = dev::pc_mk(fa[m] * w, partner ? fb[m] * w : 0.0f);
            }
        }
        // the next pair's frames, in flight during this pair's transforms
#ifndef CRLOT_PN_NOPREFETCH
        load_frame(fa, (k + 2) * H - a.pad);
        load_frame(fb, (k + 3) * H - a.pad);
#endif
        dev::wave_lds_fence();
        dev::pn_fft<false, N>(buf, tw, lane);
        if constexpr (HAS_GAIN) {  // real gain, symmetric over the N bins (L2-resident table)
#pragma unroll
            for (int m = 0; m < E; ++m) {
                if (valid(m)) {
                    const int n = lane + 64 * m;
                    buf[n] = buf[n] * a.t.gain[n <= N / 2 ? n : N - n];
                }
            }
            dev::wave_lds_fence();
        }
        dev::pn_fft<true, N>(buf, tw, lane);
        // push frame k (the real part) and k+1 (the imaginary part) straight from
        // the buffer: o = v (1/N), then o * ws; the output sanitize threshold
        // 1e-30 = 2^-99.66: exponents <= -99 flag the walk
        {
            int e = 0;
            const int base = k * H + lane;
#pragma unroll
            for (int m = 0; m < E; ++m) {
                if (valid(m)) {
                    const int n = lane + 64 * m;
                    const dev::pc v = buf[n] * dev::pc{inv_n, inv_n};
                    e = min(e, min(__builtin_amdgcn_frexp_expf(v.x), __builtin_amdgcn_frexp_expf(v.y)));
                    const int pos = (base + 64 * m) & RM;
                    ring[pos] = __builtin_fmaf(v.x * ws[n], g, ring[pos]);
                }
            }
            bad |= e <= -99;
        }
        dev::wave_lds_fence();
        produce(k);
        {
            const int base = (k + 1) * H + lane;
#pragma unroll
            for (int m = 0; m < E; ++m) {
                if (valid(m)) {
                    const int n = lane + 64 * m;
                    const dev::pc v = buf[n] * dev::pc{inv_n, inv_n};
                    const int pos = (base + 64 * m) & RM;
                    ring[pos] = __builtin_fmaf(v.y * ws[n], g, ring[pos]);
                }
            }
        }
        dev::wave_lds_fence();
        if (k + 1 < f1) produce(k + 1);
    }
    const uint64_t bal = __builtin_amdgcn_ballot_w64(bad);
    if (lane == 0) a.t.pflags[gw] = bal != 0 ? 1u : 0u;
}

namespace {
// the instantiated sizes
template <typename F>
bool pn_dispatch(int n, F&& f) {
    switch (n) {
        case 320: f(std::integral_constant<int, 320>{}); return true;
        case 400: f(std::integral_constant<int, 400>{}); return true;
        case 640: f(std::integral_constant<int, 640>{}); return true;
        case 882: f(std::integral_constant<int, 882>{}); return true;
        case 1000: f(std::integral_constant<int, 1000>{}); return true;
        case 1764: f(std::integral_constant<int, 1764>{}); return true;
        default: return false;
    }
}
}  // namespace

}  // namespace fk

bool pairn_size(int n) {
    return fk::pn_dispatch(n, [](auto) {});
}

bool pairn_supported(int n, int h, int ring_len) {
    if (!pairn_size(n)) return false;
    if (h < 32 || h > n || ring_len % h != 0) return false;
    return fk::pn_waves(n, h) >= 1;
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
    const int W = std::min(pn_waves(g.n, g.h), 4 * pn_wpe(g.n));
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    // chunks: about two resident rounds of walkers, each >= 48 frames
    const int64_t resident = int64_t(cus) * W;
    const int64_t n = std::max<int64_t>(1, std::min<int64_t>(F / 48, (2 * resident + n_streams - 1) / n_streams));
    a.M = int((F + n - 1) / n);
    a.n_chunks = int((F + a.M - 1) / a.M);
    const int64_t waves = int64_t(n_streams) * a.n_chunks;
    if (t.pflags_len < waves) return hipErrorInvalidValue;
    *n_chunks = a.n_chunks;
    const size_t lds = pn_tables(g.n) + size_t(W) * pn_per_wave(g.n, g.h);
    hipError_t e = hipSuccess;
    pn_dispatch(g.n, [&](auto nc) {
        constexpr int NN = decltype(nc)::value;
        auto k = t.gain ? k_pairn<NN, true> : k_pairn<NN, false>;
        if ((e = set_lds(k, lds)) != hipSuccess) return;
        hipLaunchKernelGGL(k, dim3(unsigned((waves + W - 1) / W)), dim3(64 * W), lds, stream, a);
        e = hipGetLastError();
    });
    return e;
}

// W_{ns r}^{q jm} per pass of fft_pairn.h's factorisation, float pairs
std::vector<float> build_pairn_twiddles(int n) {
    const dev::PnFac f = dev::pn_factor(n);
    std::vector<float> t(2 * size_t(f.tw_len));
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
