// pair30.hip -- K_pair30: the frame-pair round trip at N = 1920 (40 ms at
// 48 kHz) as two 960-point transforms on two waves.
//
// Frames 2j, 2j+1 travel as one complex sequence z (pair_any.hip explains the
// pairing).  Its 1920-point DFT splits by decimation in time: wave 0 transforms
// the even samples E = z[2i], wave 1 the odd samples O = z[2i+1], each with
// K_pair15's 960-point transform (fft_pair15.h: Good-Thomas 15 over the
// registers, the 64-lane stage); both spectra land at the same (lane, register)
// bins, so one LDS exchange gives every wave E[k] and O[k] side by side:
//   X[k] = E[k] + W1920^k O[k],  X[k + 960] = E[k] - W1920^k O[k]
// and the inverse runs the split backwards: wave 0 the 960-point inverse of
// X[k] + X[k + 960] (the even outputs), wave 1 of (X[k] - X[k + 960]) W1920^-k
// (the odd outputs).  W1920^k at bin k = k1 + 15 (k'' + 4 d) of (lane, d) is
// c_lane W32^d: a per-lane table entry times a per-register constant.
// With an even hop every ring position is written and read by one wave only
// (sample n of frame k sits at k H + n, parity n's), so the overlap-add and the
// produce need no cross-wave synchronisation; the exchange costs two barriers.
// Everything else is K_pair15's walk: frames loaded whole (L2 hits), the OLA in
// an LDS ring, Markstein division, flags -> the per-frame walker redoes the
// stream (a stream's bits depend on its samples only).
#include <cstdlib>

#include "fft_pair15.h"
#include "fused_common.h"

namespace crlot {
namespace fk {

namespace {

constexpr int kP30Ring = 2048;  // >= H ceil(N / H) for every even hop the host allows

__host__ __device__ inline int p30_ring(int h) {
    const int span = h * ((1920 + h - 1) / h);
    int r = 1;
    while (r < span) r <<= 1;
    return r;
}

constexpr size_t p30_lds() { return sizeof(dev::pc) * 2 * dev::kPairXbuf + sizeof(float) * kP30Ring; }

// W32^d (forward); INV: conjugate
template <bool INV>
__device__ __forceinline__ dev::pc w32c(int d) {
    // cos / sin of 2 pi d / 32, d < 16
    constexpr float C[9] = {1.0f, 0.98078528040323044913f, 0.92387953251128675613f, 0.83146961230254523708f,
                            0.70710678118654752440f, 0.55557023301960222474f, 0.38268343236508977173f,
                            0.19509032201612826785f, 0.0f};
    const float c = d <= 8 ? C[d] : -C[16 - d];
    const float s = d <= 8 ? C[8 - d] : C[d - 8];
    return INV ? dev::pc_mk(c, s) : dev::pc_mk(c, -s);
}

}  // namespace

// HAS_GAIN: the spectral hook, a real gain per bin (symmetric over the 1920 bins).
// WPE waves per SIMD; PRE: the next pair's frames loaded during this pair's
// transforms; WSREG: the synthesis window in registers (else from L1/L2 per use)
template <bool HAS_GAIN, int WPE, bool PRE, bool WSREG>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(WPE))) void k_pair30_hot(const FusedArgs a) {
    constexpr int E = 15, N = 1920;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // 0: even samples, 1: odd
    const int H = a.hop;
    const int RL = p30_ring(H), RM = RL - 1;
    const int NB = (N + H - 1) / H;
    dev::pc* bufs = reinterpret_cast<dev::pc*>(smem);
    dev::pc* buf = bufs + w * dev::kPairXbuf;
    const dev::pc* obuf = bufs + (1 - w) * dev::kPairXbuf;
    float* ring = reinterpret_cast<float*>(bufs + 2 * dev::kPairXbuf);
    const int gw = blockIdx.x;
    if (gw >= a.n_streams * a.n_chunks) return;  // (the whole workgroup)
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

    dev::Pair15Tw tw;
    dev::pair15_tw_load(tw, reinterpret_cast<const dev::pc*>(a.t.ptw), lane);
    const dev::pc cl = reinterpret_cast<const dev::pc*>(a.t.ptw)[dev::kP15Tw + lane];  // W1920^{k1 + 15 k''}
    // this wave's bins: k1 = 15 is the 960-point transform's zero row (no bin)
    const bool live = ((lane & 3) + 4 * (lane >> 4)) != 15;
    float war[E];
    float wsr[WSREG ? E : 1];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        war[m] = a.t.wa[2 * (lane + 64 * m) + w];
        if constexpr (WSREG) wsr[m] = a.t.ws[2 * (lane + 64 * m) + w] * a.inv_n * a.gain;  // (folded: the push)
    }
    for (int i = threadIdx.x; i < RL; i += 128) ring[i] = 0.0f;
    __syncthreads();

    // this wave's samples of frame k: x[origin + 2 (lane + 64 m) + w]; outside
    // [0, T) the buffer range check reads 0 (zero padding)
    auto load_frame = [&](float (&f)[E], int origin) {
        const int v = (origin + 2 * lane + w) * 4;
#pragma unroll
        for (int m = 0; m < E; ++m) f[m] = dev::bload1(rx, v + m * 512, 0);
    };
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
    // push: this wave's samples of the frame at block k's position (its parity's ring slots)
    // (WSREG: p is the unscaled inverse output and the push multiplies by the staged
    // factor ws / N g, one rounding for three -- inside the FFT tolerance; a flagged
    // stream is redone whole by the per-frame walker.  Else p = (v / N) ws and the
    // push is fma(p, g, ring).)
    auto push = [&](const float (&p)[E], int k) {
        const int base = k * H + 2 * lane + w;  // k H < 2^27 (host-checked)
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int pos = (base + 128 * m) & RM;
            ring[pos] = __builtin_fmaf(p[m], WSREG ? wsr[m] : g, ring[pos]);
        }
        dev::wave_lds_fence();
    };
    // produce(H) of block k, this wave's parity rows j = 2 i + w: ring / den by
    // Markstein's correction (the {den, 1/den} pairs), clear; flagged outside its range
    const __amdgpu_buffer_rsrc_t rden =
        dev::make_rsrc(reinterpret_cast<const float2*>(a.t.den_rden), uint32_t(ring_blocks * H) * 8u);
    auto produce = [&](int k) {
        const int base = k * H;
        const int dbase = (k % ring_blocks) * H;
        const __amdgpu_buffer_rsrc_t rk = k >= f0 ? ry : ry_null;
        if (!a.t.den_rden) {  // divisors outside Markstein's range: the IEEE division
            for (int j = 2 * lane + w; j < H; j += 128) {
                const int pos = (base + j) & RM;
                const float v = ring[pos];
                ring[pos] = 0.0f;
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v / a.t.den[dbase + j]), rk,
                                                      (base + j) * 4, 0, 0);
            }
            dev::wave_lds_fence();
            return;
        }
        for (int j0 = 2 * lane + w; j0 < H; j0 += 4 * 128) {
            float2 d[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) d[i] = dev::bload2(rden, (j0 + 128 * i) * 8, dbase * 8);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int j = j0 + 128 * i;
                if (j < H) {
                    const int pos = (base + j) & RM;
                    const float v = ring[pos];
                    ring[pos] = 0.0f;
                    const float o = mk_div(v, d[i].x, d[i].y);
                    bad |= uint32_t(__builtin_amdgcn_frexp_expf(v) + 63) > 128u;  // exponent outside [-63, 65]
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o), rk, (base + j) * 4, 0, 0);
                }
            }
        }
        dev::wave_lds_fence();
    };

    float fa[E], fb[E];
    if constexpr (PRE) {
        load_frame(fa, fs * H - a.pad);
        load_frame(fb, (fs + 1) * H - a.pad);
    }
    for (int k = fs; k < f1; k += 2) {
        if constexpr (!PRE) {
            load_frame(fa, k * H - a.pad);
            load_frame(fb, (k + 1) * H - a.pad);
        }
        check(fa);
        check(fb);
        const bool partner = k + 1 < a.F;  // frame k+1 past the last: imaginary part 0
        dev::pc v[16];
#pragma unroll
        for (int m = 0; m < E; ++m) v[m] = dev::pc_mk(fa[m] * war[m], partner ? fb[m] * war[m] : 0.0f);
        v[15] = dev::pc_mk(0.0f, 0.0f);
        if constexpr (PRE) {
            load_frame(fa, (k + 2) * H - a.pad);  // the next pair's, during this pair's transforms
            load_frame(fb, (k + 3) * H - a.pad);
        }
        dev::pair15_fwd(v, buf, tw, lane);
        // exchange the half spectra (the same bins on both waves)
#pragma unroll
        for (int d = 0; d < 16; ++d) buf[64 * d + lane] = v[d];
        __syncthreads();
#pragma unroll
        for (int d = 0; d < 16; ++d) {
            const dev::pc ot = obuf[64 * d + lane];  // the other half's bin, used at once
            const dev::pc ev = w == 0 ? v[d] : ot, od = w == 0 ? ot : v[d];
            const dev::pc t = dev::pc_mul(dev::pc_mul(od, cl), w32c<false>(d));  // W1920^k O[k]
            dev::pc x0 = ev + t, x1 = ev - t;                                     // X[k], X[k + 960]
            if constexpr (HAS_GAIN) {  // bins k and k + 960: gain[k], gain[960 - k] (k <= 960)
                const int kb = dev::pair15_bin(lane, d);
                x0 = x0 * a.t.gain[live ? kb : 0];
                x1 = x1 * a.t.gain[live ? 960 - kb : 0];
            }
            // (X[k] - X[k + 960]) W1920^-k: conj(W32^d), then conj(c_lane)
            const dev::pc r = w == 0 ? x0 + x1 : dev::pc_mulc(dev::pc_mul(x0 - x1, w32c<true>(d)), cl);
            v[d] = live ? r : dev::pc_mk(0.0f, 0.0f);
        }
        __syncthreads();  // both read before either transposes into its buffer again
        dev::pair15_inv(v, buf, tw, lane);
        // the output sanitize acts on o = v / N below 1e-30 = 2^-99.66: on o, frexp
        // exponents <= -99 flag the walk; on the unscaled v (WSREG), |v| < 2^-88
        // covers every |v / N| < 1e-30 N / N = 2^-88.75 (and a few harmless others)
        {
            constexpr int kSanExp = WSREG ? -88 : -99;
            int e[4] = {0, 0, 0, 0};
#pragma unroll
            for (int m = 0; m < E; ++m) {
                if constexpr (!WSREG) v[m] = v[m] * dev::pc{inv_n, inv_n};
                e[m & 3] = min(e[m & 3], min(__builtin_amdgcn_frexp_expf(v[m].x), __builtin_amdgcn_frexp_expf(v[m].y)));
            }
            bad |= min(min(e[0], e[1]), min(e[2], e[3])) <= kSanExp;
        }
        float p[E];
#pragma unroll
        for (int m = 0; m < E; ++m) {
            if constexpr (!WSREG) {
                const float wsm = a.t.ws[2 * (lane + 64 * m) + w];
                v[m] = v[m] * dev::pc{wsm, wsm};
            }
            p[m] = v[m].x;
        }
        push(p, k);
        produce(k);
#pragma unroll
        for (int m = 0; m < E; ++m) p[m] = v[m].y;
        push(p, k + 1);
        if (k + 1 < f1) produce(k + 1);
    }
    const bool any_bad = __syncthreads_or(bad);
    if (threadIdx.x == 0) a.t.pflags[gw] = any_bad ? 1u : 0u;
}

}  // namespace fk

bool pair30_supported(int n, int h, int ring_len) {
    if (n != 1920 || h < 32 || h > n || h % 2 != 0 || ring_len % h != 0) return false;
    return fk::p30_ring(h) <= fk::kP30Ring;
}

hipError_t launch_pair30(const Geometry& g, const DevTables& t, const float* x, float* y, int n_streams, int64_t T,
                         int64_t ld_x, int64_t ld_y, int64_t F, int64_t out_len, int* n_chunks, hipStream_t stream) {
    using namespace fk;
    if (!pair30_supported(g.n, g.h, g.ring_len) || !t.ptw || !t.pflags || F <= 0 ||
        n_streams <= 0 || T >= (int64_t(1) << 27) || out_len >= (int64_t(1) << 27))
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
    // chunks: about two resident rounds of walks (two waves each), each >= 48 frames
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    constexpr size_t lds = p30_lds();
    // 3 waves/SIMD with the frames loaded at the top of each pair (no prefetch: 167
    // VGPRs) measured 121k / 207k Msamples/s at 1920/480 / 1920/960 against 115k /
    // 182k for 2 waves with the prefetch and 104k / 184k for 3 waves with the
    // synthesis window read from L1 (profiles/r03_pair30_ab.jsonl); CRLOT_P30_VARIANT=1
    // selects the 2-wave form (A/B).  The gain walker needs the 2-wave budget.
    static const int venv = [] {
        const char* e = ab_env("CRLOT_P30_VARIANT");
        return e ? std::atoi(e) : 0;
    }();
    const int wpe = t.gain || venv == 1 ? 2 : 3;
    const int64_t walks_per_cu = std::min<int64_t>(int64_t(160 * 1024 / lds), 2 * wpe);
    const int64_t resident = int64_t(cus) * walks_per_cu;
    const int64_t nc = chunks_or(std::max<int64_t>(1, std::min<int64_t>(F / 48, (2 * resident + n_streams - 1) / n_streams)), F);
    a.M = int((F + nc - 1) / nc);
    a.n_chunks = int((F + a.M - 1) / a.M);
    const int64_t walks = int64_t(n_streams) * a.n_chunks;
    if (t.pflags_len < walks) return hipErrorInvalidValue;
    *n_chunks = a.n_chunks;
    note_chunks(a.n_chunks);
    auto k = t.gain      ? k_pair30_hot<true, 2, true, false>
             : venv == 1 ? k_pair30_hot<false, 2, true, true>
                         : k_pair30_hot<false, 3, false, true>;
    hipError_t e = set_lds(k, lds);
    if (e != hipSuccess) return e;
    note_launch(CRLOT_K_PAIR30, walks);
    hipLaunchKernelGGL(k, dim3(unsigned(walks)), dim3(128), lds, stream, a);
    return hipGetLastError();
}

// the 960-point pair transform's tables (build_pair15_twiddles(960)), then [64]
// of W1920^{k1 + 15 k''}, k1 = (l & 3) + 4 (l >> 4), k'' = (l >> 2) & 3
std::vector<float> build_pair30_twiddles() {
    std::vector<float> t = build_pair15_twiddles(960);
    for (int l = 0; l < 64; ++l) {
        const int k = ((l & 3) + 4 * (l >> 4)) + 15 * ((l >> 2) & 3);
        const double ph = -2.0 * M_PI * double(k) / 1920.0;
        t.push_back(float(std::cos(ph)));
        t.push_back(float(std::sin(ph)));
    }
    return t;
}

}  // namespace crlot
