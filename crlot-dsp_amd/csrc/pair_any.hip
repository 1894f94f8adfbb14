// pair_any.hip -- K_pair960: the frame-pair round trip at N = 960 (20 ms at
// 48 kHz), any hop H whose ring the plan allows.
//
// Frames 2j and 2j+1 of a stream travel as one 960-point complex transform per
// wave (fft_pair15.h), z = x_2j w + i x_2j+1 w, as the power-of-two pair kernels
// do.  H is in general not a multiple of the 64 lanes, so a sample does not stay
// in its lane from frame to frame: every pair loads its two frames whole (15
// dwords per lane each, mostly L2 hits -- each sample is read N/H times) and
// the overlap-add runs in a per-wave LDS ring of H (ceil(N/H) + 1) floats:
// push frame k (fma(o * ws, g, ring) in ascending k), produce block k (ring /
// den, IEEE division, then clear), push frame k+1, produce block k+1 -- the
// reference's streaming-interleaved order.  o = v * (1/N) after the inverse, as
// kissfft_adapter.cc:154 scales.
//
// Paired regime only (like the hot walkers of pair_hot.hip): a sample outside
// [px_lo, px_hi] (or NaN / Inf), or an output below the sanitize threshold,
// flags the walk; a stream with any flagged walk is then recomputed whole by
// the per-frame mixed-radix walker (k_stft_ola_any, kissfft's algorithm with the
// full sanitize), so a stream's bits depend only on its own samples.
#include <algorithm>
#include <cmath>
#include <vector>

#include "fft_pair15.h"
#include "fused_common.h"

namespace crlot {
namespace fk {

namespace {

// frame k of the walk: 15 samples per lane, x[origin + lane + 64 m]; out-of-range
// lanes (either side, zero padding) read 0 (see load_hop0)
__device__ __forceinline__ void load_frame15(float (&f)[15], __amdgpu_buffer_rsrc_t rx, int lane, int origin) {
    const int v = (origin + lane) * 4;
#pragma unroll
    for (int m = 0; m < 15; ++m) f[m] = dev::bload1(rx, v + m * 256, 0);
}

}  // namespace

template <int W>
__global__ __launch_bounds__(64 * W) void k_pair960_hot(const FusedArgs a) {
    constexpr int E = 15, N = 960;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int H = a.hop;
    const int NB = (N + H - 1) / H, RL = H * (NB + 1);
    dev::pc* buf = reinterpret_cast<dev::pc*>(smem) + wave * dev::kPairXbuf;
    float* ring = reinterpret_cast<float*>(reinterpret_cast<dev::pc*>(smem) + W * dev::kPairXbuf) + wave * RL;
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
    const int ring_blocks = a.ring_blocks;  // ring_len / H (the den table's blocks)
    const uint32_t xlo_b = __builtin_bit_cast(uint32_t, a.t.px_lo), xhi_b = __builtin_bit_cast(uint32_t, a.t.px_hi);

    dev::Pair15Tw tw;
    dev::pair15_tw_load(tw, reinterpret_cast<const dev::pc*>(a.t.ptw), lane);
    float wa[E], ws[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        wa[m] = a.t.wa[lane + 64 * m];
        ws[m] = a.t.ws[lane + 64 * m];
    }
    for (int i = lane; i < RL; i += 64) ring[i] = 0.0f;

    bool bad = false;
    auto check = [&](const float (&f)[E]) {
        uint32_t mx = 0u, mn = ~0u;
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const uint32_t u = __builtin_bit_cast(uint32_t, f[m]) & 0x7fffffffu;
            mx = max(mx, u);
            mn = min(mn, u - 1u);
        }
        bad |= (mx > xhi_b) | (mn < xlo_b - 1u);
    };
    // push one frame's window-weighted output into the ring at block k's position
    auto push = [&](const float (&p)[E], int k) {
        int base = (k % (NB + 1)) * H;  // k H mod RL
#pragma unroll
        for (int m = 0; m < E; ++m) {
            int pos = base + lane + 64 * m;
            pos = pos >= RL ? pos - RL : pos;
            ring[pos] = __builtin_fmaf(p[m], g, ring[pos]);
        }
        dev::wave_lds_fence();
    };
    // produce(H) of block k: ring / den (IEEE), clear; stored when k >= f0
    auto produce = [&](int k) {
        const int base = (k % (NB + 1)) * H;
        const int dbase = (k % ring_blocks) * H;
        const __amdgpu_buffer_rsrc_t rk = k >= f0 ? ry : ry_null;
        for (int j = lane; j < H; j += 64) {
            int pos = base + j;
            pos = pos >= RL ? pos - RL : pos;
            const float v = ring[pos];
            ring[pos] = 0.0f;
            const float o = v / a.t.den[dbase + j];
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o), rk, (k * H + j) * 4, 0, 0);
        }
        dev::wave_lds_fence();
    };

    float fa[E], fb[E];
    load_frame15(fa, rx, lane, fs * H - a.pad);
    load_frame15(fb, rx, lane, (fs + 1) * H - a.pad);
    for (int k = fs; k < f1; k += 2) {
        check(fa);
        check(fb);
        const bool partner = k + 1 < a.F;  // frame k+1 past the last: imaginary part 0
        dev::pc v[16];
#pragma unroll
        for (int m = 0; m < E; ++m) v[m] = dev::pc_mk(fa[m] * wa[m], partner ? fb[m] * wa[m] : 0.0f);
        v[15] = dev::pc_mk(0.0f, 0.0f);
        // the next pair's frames, in flight during this pair's transforms
        load_frame15(fa, rx, lane, (k + 2) * H - a.pad);
        load_frame15(fb, rx, lane, (k + 3) * H - a.pad);
        dev::pair15_fwd(v, buf, tw, lane);
        dev::pair15_inv(v, buf, tw, lane);
        // o = v / N; its sanitize threshold 1e-30 = 2^-99.66: frexp exponents <= -99 flag the walk
        {
            int e[4] = {0, 0, 0, 0};
#pragma unroll
            for (int m = 0; m < E; ++m) {
                v[m] = v[m] * dev::pc{inv_n, inv_n};
                e[m & 3] = min(e[m & 3], min(__builtin_amdgcn_frexp_expf(v[m].x), __builtin_amdgcn_frexp_expf(v[m].y)));
            }
            bad |= min(min(e[0], e[1]), min(e[2], e[3])) <= -99;
        }
        float p[E];
#pragma unroll
        for (int m = 0; m < E; ++m) {
            v[m] = v[m] * dev::pc{ws[m], ws[m]};
            p[m] = v[m].x;
        }
        push(p, k);
        produce(k);
#pragma unroll
        for (int m = 0; m < E; ++m) p[m] = v[m].y;
        push(p, k + 1);
        if (k + 1 < f1) produce(k + 1);
    }
    const bool any_bad = __builtin_amdgcn_ballot_w64(bad) != 0;
    if (lane == 0) a.t.pflags[gw] = any_bad ? 1u : 0u;
}

constexpr int kP960Waves = 2;  // per workgroup; LDS (transpose + ring per wave) sets the CU's share

size_t pair960_lds(int h) {
    const int nb = (960 + h - 1) / h, rl = h * (nb + 1);
    return size_t(kP960Waves) * (sizeof(dev::pc) * dev::kPairXbuf + sizeof(float) * rl);
}

}  // namespace fk

bool pair960_supported(int n, int h, int ring_len) {
    return n == 960 && h >= 64 && h <= 960 && ring_len % h == 0 && fk::pair960_lds(h) <= 64 * 1024;
}

hipError_t launch_pair960(const Geometry& g, const DevTables& t, const float* x, float* y, int n_streams,
                          int64_t T, int64_t ld_x, int64_t ld_y, int64_t F, int64_t out_len, int* n_chunks,
                          hipStream_t stream) {
    using namespace fk;
    if (!pair960_supported(g.n, g.h, g.ring_len) || !t.ptw || !t.pflags || F <= 0 || n_streams <= 0 ||
        T >= (int64_t(1) << 29) || out_len >= (int64_t(1) << 29))
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
    // chunks: about two resident rounds of walkers, each >= 48 frames
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    const size_t lds = pair960_lds(g.h);
    const int64_t resident = int64_t(cus) * kP960Waves * int64_t(std::max<size_t>(1, 160 * 1024 / lds));
    int64_t n = std::max<int64_t>(1, std::min<int64_t>(F / 48, (2 * resident + n_streams - 1) / n_streams));
    a.M = int((F + n - 1) / n);
    a.n_chunks = int((F + a.M - 1) / a.M);
    const int64_t waves = int64_t(n_streams) * a.n_chunks;
    if (t.pflags_len < waves) return hipErrorInvalidValue;
    *n_chunks = a.n_chunks;
    auto k = k_pair960_hot<kP960Waves>;
    hipError_t e = set_lds(k, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3(unsigned((waves + kP960Waves - 1) / kP960Waves)), dim3(64 * kP960Waves), lds,
                       stream, a);
    return hipGetLastError();
}

std::vector<float> build_pair15_twiddles() {
    std::vector<float> t;
    for (int k1 = 1; k1 < 15; ++k1)
        for (int l = 0; l < 64; ++l) {
            const double ph = -2.0 * M_PI * double(l * k1) / 960.0;
            t.push_back(float(std::cos(ph)));
            t.push_back(float(std::sin(ph)));
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
