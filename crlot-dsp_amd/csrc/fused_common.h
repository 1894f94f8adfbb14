// fused_common.h -- device and host pieces shared by the fused walker kernels
// (kernels.hip: K_fused*, K_pair512/2k/4k, K_fused_wg; pair1k.hip: K_pair).
#pragma once

#include <cstdint>

#include "fft_wave.h"
#include "kernels.h"

namespace crlot {
namespace fk {

struct FusedArgs {
    DevTables t;
    const float* x;
    float* y;
    int64_t ld_x, ld_y;
    int T, out_len;  // per stream, T * 4 and out_len * 4 < 2^31 (checked on the host)
    int n_streams, F, n_chunks, M, ring_blocks;
    int pad, pad_mode;  // framing (Geometry)
    float inv_n, gain;
    int fix_all = 0;  // K_pair: the fix-up walker redoes every chunk (padding rules it alone handles)
    int hop = 0;      // K_pair960 (runtime hop; the power-of-two walkers take it as a template constant)
    int cs = 1;       // K_pair interleaved groups: channels per group (stream g*cs + c is sample i at
                      // x[g*ld_x + i*cs + c]); 1 = planar rows
};

// Wave gw of a chunked walk -> stream s, chunk c and the element offsets of the
// stream's first input / output sample.  Planar rows: stream-major.  Interleaved
// groups (ILV, a.cs channels): the channels of one group and chunk on
// consecutive waves, so the waves of a workgroup read and write whole sample
// rows together (lines shared in their XCD's L2 instead of refetched).
struct WalkId {
    int s, c;
    int64_t xo, yo;
};
template <bool ILV>
__device__ __forceinline__ WalkId walk_id(const FusedArgs& a, int gw) {
    WalkId w;
    if constexpr (!ILV) {
        w.s = gw / a.n_chunks;
        w.c = gw - w.s * a.n_chunks;
        w.xo = int64_t(w.s) * a.ld_x;
        w.yo = int64_t(w.s) * a.ld_y;
    } else {
        const int r = gw / a.cs, ch = gw - r * a.cs;
        const int g = r / a.n_chunks;
        w.c = r - g * a.n_chunks;
        w.s = g * a.cs + ch;
        w.xo = int64_t(g) * a.ld_x + ch;
        w.yo = int64_t(g) * a.ld_y + ch;
    }
    return w;
}

// FrameQueue padding (Indexing.h:18-37): left side i -> -i-1, right side
// i -> 2n-2-i, repeated until inside.
__device__ __forceinline__ int reflect101(int i, int n) {
    if (n <= 1) return 0;
    while (i < 0 || i >= n) i = i < 0 ? -i - 1 : 2 * n - 2 - i;
    return i;
}

// x[j] of a T-sample stream with the plan's padding outside [0, T)
// (getPaddingValueSafe, Indexing.h:48-68): 0 zeros, 1 reflect101, 2 edge.
__device__ __forceinline__ float fetch_x(__amdgpu_buffer_rsrc_t rx, int j, int T, int mode) {
    if (mode == 1) j = reflect101(j, T);
    else if (mode == 2) j = j < 0 ? 0 : (j >= T ? T - 1 : j);
    const bool ok = j >= 0 && j < T;
    const float v = dev::bload1(rx, (ok ? j : 0) * 4, 0);
    return ok ? v : 0.0f;
}


// Division acc / den by Markstein's correction with r = RN(1/den): exact (equal
// to the IEEE quotient) for den in [2^-40, 2^40] (host-checked) and acc = 0 or
// |acc| in [2^-64, 2^64]; any other value sends the whole wave to the IEEE
// division.  Verified exhaustively over den significands.
__device__ __forceinline__ bool mk_ok(float a) {
    const float t = __builtin_fabsf(a);
    return t <= 0x1p64f && (t >= 0x1p-64f || t == 0.0f);
}
__device__ __forceinline__ float mk_div(float a, float d, float r) {
    const float q = a * r;
    return __builtin_fmaf(__builtin_fmaf(-q, d, a), r, q);
}

// ------------------------------------------------------------------ pair-walker hop helpers
template <int SH>
__device__ __forceinline__ void load_hop1(float* dst, __amdgpu_buffer_rsrc_t rx, int lane, int origin,
                                          int T, int mode) {
    constexpr int H = 64 * SH;
#ifdef CRLOT_ABL_NOLOAD  // timing-only ablation: wrong results
#pragma unroll
    for (int q = 0; q < SH; ++q) dst[q] = float(lane + q + origin) * 1e-3f;
    return;
#endif
#ifdef CRLOT_ABL_HOTONLY  // ISA-count builds: interior hops only (wrong at stream edges)
    if (true) {
#else
    if (origin >= 0 && origin + H <= T) {
#endif
#pragma unroll
        for (int q = 0; q < SH; ++q) dst[q] = dev::bload1(rx, lane * 4, origin * 4 + q * 256);
    } else {
#pragma unroll
        for (int q = 0; q < SH; ++q) dst[q] = fetch_x(rx, origin + lane + 64 * q, T, mode);
    }
}

// The same for framing whose padding is zeros (Framer ZERO_PAD / DROP, FrameQueue
// CONSTANT): the whole offset rides in voffset + the immediate, which the raw
// buffer's range check covers per lane, so every sample outside [0, T) -- past
// the end, or before 0 through the unsigned wrap of a negative offset (T * 4 <
// 2^31, host-checked) -- reads 0 and edge hops need no branch.
template <int SH>
__device__ __forceinline__ void load_hop0(float* dst, __amdgpu_buffer_rsrc_t rx, int lane, int origin) {
    const int v = (origin + lane) * 4;
#pragma unroll
    for (int q = 0; q < SH; ++q) dst[q] = dev::bload1(rx, v + q * 256, 0);
}
// bytes a stream's descriptor spans: n samples cs floats apart
__device__ __forceinline__ uint32_t span_bytes(int n, int cs) {
    return n > 0 ? uint32_t((n - 1) * cs + 1) * 4u : 0u;
}
// Hop loads with samples cs floats apart (interleaved channels; (T + 2N) * cs
// * 4 < 2^31, host-checked): one descriptor per q starting at sample 64 q and
// ending after sample T-1, so the one per-lane offset (origin + lane) * 4 cs
// is range-checked for every q (zeros outside [0, T)) without a VGPR per q.
template <int SH>
struct HopRsrc {
    __amdgpu_buffer_rsrc_t r[SH];
};
template <int SH>
__device__ __forceinline__ HopRsrc<SH> hop_rsrc(const float* base, int T, int cs) {
    HopRsrc<SH> h;
#pragma unroll
    for (int q = 0; q < SH; ++q) h.r[q] = dev::make_rsrc(base + int64_t(64 * q) * cs, span_bytes(T - 64 * q, cs));
    return h;
}
template <int SH>
__device__ __forceinline__ void load_hop0s(float* dst, const HopRsrc<SH>& rx, int lane, int origin, int cs) {
    const int v = (origin + lane) * (4 * cs);
#pragma unroll
    for (int q = 0; q < SH; ++q) dst[q] = dev::bload1(rx.r[q], v, 0);
}

// 1 when every sample of the hop (SH per lane, whole wave) keeps the paired regime.
template <int SH>
__device__ __forceinline__ uint32_t hop_ok(const float* h, float lo, float hi) {
    bool bad = false;
#pragma unroll
    for (int q = 0; q < SH; ++q) {
        const float t = __builtin_fabsf(h[q]);
        bad |= !((t >= lo) & (t <= hi)) & (t != 0.0f);
    }
    return __builtin_amdgcn_ballot_w64(bad) == 0 ? 1u : 0u;
}

// hop_ok on the bit patterns: with u = |x| as bits (float order == unsigned
// order for |x|, NaN above every finite bit pattern), a sample keeps the regime
// iff u == 0 or lo_bits <= u <= hi_bits, i.e. u <= hi_bits and u - 1 >= lo_bits - 1
// (unsigned, 0 wrapping to the top): per sample an and, a subtract and half a
// max3 / min3, one compare pair per hop.
template <int SH>
__device__ __forceinline__ uint32_t hop_ok_bits(const float* h, uint32_t lo_bits, uint32_t hi_bits) {
    uint32_t mx = 0u, mn = ~0u;
#pragma unroll
    for (int q = 0; q < SH; ++q) {
        const uint32_t u = __builtin_bit_cast(uint32_t, h[q]) & 0x7fffffffu;
        mx = max(mx, u);
        mn = min(mn, u - 1u);
    }
    return __builtin_amdgcn_ballot_w64((mx > hi_bits) | (mn < lo_bits - 1u)) == 0 ? 1u : 0u;
}

// den / rden of OLA block b for this lane (DevTables::pden: [block][lane][den SH | rden SH]).
template <int SH>
__device__ __forceinline__ void load_den(float (&dr)[2 * SH], __amdgpu_buffer_rsrc_t rp, int lane, int b) {
#ifdef CRLOT_ABL_NODEN  // timing-only ablation: wrong results
#pragma unroll
    for (int q = 0; q < SH; ++q) {
        dr[q] = 1.5f;
        dr[SH + q] = 0.6666667f;
    }
    return;
#endif
#pragma unroll
    for (int j = 0; j < 2 * SH / 4; ++j) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rp, lane * (8 * SH), b * (512 * SH) + 16 * j, 0);
        const unsigned u0 = v[0], u1 = v[1], u2 = v[2], u3 = v[3];  // (see bload2)
        dr[4 * j] = __builtin_bit_cast(float, u0);
        dr[4 * j + 1] = __builtin_bit_cast(float, u1);
        dr[4 * j + 2] = __builtin_bit_cast(float, u2);
        dr[4 * j + 3] = __builtin_bit_cast(float, u3);
    }
}

template <typename K>
hipError_t set_lds(K kernel, size_t lds) {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
}

// K_pair (pair1k.hip): waves a CU holds, and the launch for H = 64 * sh.
int pair_waves_per_cu();
hipError_t launch_pair(int sh, const FusedArgs& a, int64_t waves, hipStream_t stream);
// K_pair4k's paired-only hot walker (pair_hot.hip), H = 256 * sh; writes pflags per workgroup.
hipError_t launch_pair4k_hot(int sh, const FusedArgs& a, int64_t grid, hipStream_t stream);
// ... at three workgroups per CU (one exchange buffer, windows from L2; no gain)
hipError_t launch_pair4k_hot3(int sh, const FusedArgs& a, int64_t grid, hipStream_t stream);
// ... and K_pair2k's (H = 128 * sh)
hipError_t launch_pair2k_hot(int sh, const FusedArgs& a, int64_t grid, hipStream_t stream);
hipError_t launch_pair2k_hot3(int sh, const FusedArgs& a, int64_t grid, hipStream_t stream);
// ... and K_pair512's (H = 64 * sh, sh = 2 or 4; w waves per workgroup, flags per wave)
hipError_t launch_pair512_hot(int sh, const FusedArgs& a, int64_t waves, int w, hipStream_t stream);
// K_pair_stft / K_pair_istft (pair_stft.hip): N = 1024, H = 128, 256, 512; N = 512, H = 128, 256
struct PairSpecArgs {
    FusedArgs f;       // stft: x, T, ld_x; istft: y, out_len, ld_y, the OLA tables
    float* spec;       // stft output rows
    const float* sin;  // istft input rows
    int64_t ld_spec, ld_frame;
    SpecMask mask;     // istft: the per-frame mask (p null: none)
};
int pair_spec_walkers_per_cu(int n);
hipError_t launch_pair_stft(int n, int h, const PairSpecArgs& a, int64_t walkers, hipStream_t stream);
hipError_t launch_pair_istft(int n, int h, const PairSpecArgs& a, int64_t walkers, hipStream_t stream);
// ... at N = 4096 (H = 512, 1024) and 2048 (H = 256, 512): one workgroup per walk
// (pair_wg_spec.hip), the masked round trip too
bool pair_wg_supported(int n, int h);
int pair_wg_walkers_per_cu(int n);
hipError_t launch_pairwg_stft(int n, int h, const PairSpecArgs& a, int64_t walkers, hipStream_t stream);
hipError_t launch_pairwg_istft(int n, int h, const PairSpecArgs& a, int64_t walkers, hipStream_t stream);
hipError_t launch_pairwg_mask(int n, int h, const PairSpecArgs& a, int64_t walkers, hipStream_t stream);
// K_pair_mask (pair_mask.hip): walkers a CU holds, and the launch (N = 1024: H = 128, 256, 512; N = 512: H = 128, 256)
int pair_mask_walkers_per_cu(int n);
hipError_t launch_pair_mask(int n, int h, const FusedArgs& f, const SpecMask& m, int64_t walkers,
                            hipStream_t stream);

}  // namespace fk
}  // namespace crlot
