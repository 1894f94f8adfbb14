// pair1k.hip -- K_pair, the N = 1024 frame-pair walker (the headline kernel).
// Numerics as kernels.hip (header comment there); the transform is fft_pair.h.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "fft_pair.h"
#include "fused_common.h"
#include "ola_pair.h"

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

#ifndef CRLOT_PAIR_REG_TW
#define CRLOT_PAIR_REG_TW 1  // measured: LDS twiddles at 4 waves/SIMD take 5 % more cycles
#endif
// Cache policy of the hot walker's hop loads and output stores: nt (streaming;
// each sample is read by one walk and written once).  Measured +0.1-1.6 % over
// the default policy in four interleaved A/B runs (scripts/ab_bench.py).  The
// interleaved-group walk keeps the default policy for its stores: its rows are
// written a word per lane by several waves, which L2 must merge (nt stores
// there: C = 4 251k -> 142k Msamples/s).
#ifndef CRLOT_PAIR_LD_AUX
#define CRLOT_PAIR_LD_AUX 2
#endif
#ifndef CRLOT_PAIR_ST_AUX
#define CRLOT_PAIR_ST_AUX 2
#endif
#ifndef CRLOT_PAIR_HOT2
#define CRLOT_PAIR_HOT2 1  // ... and at H = 128
#endif
#ifndef CRLOT_PAIR_HOT8
#define CRLOT_PAIR_HOT8 1  // the paired-only walker at H = 512 too
#endif
#ifndef CRLOT_PAIR_PK2
#define CRLOT_PAIR_PK2 2  // the hot walker's packing: bit 0 hop-slot pairs (window products; spills, measured slower), bit 1 block pairs (OLA adds, divisions)
#endif
#define CRLOT_PAIR_PKX (CRLOT_PAIR_PK2 & 1)
#ifndef CRLOT_PAIR_OSCREEN
#define CRLOT_PAIR_OSCREEN 1  // output-sanitize screen (v_min3 over |v|) off the window-edge registers, the exact test only where it fails
#endif
#define CRLOT_PAIR_PKA ((CRLOT_PAIR_PK2 >> 1) & 1)
#ifndef CRLOT_PAIR_MIN_WAVES
#define CRLOT_PAIR_MIN_WAVES (CRLOT_PAIR_REG_TW ? 3 : 4)
#endif

// Register rotation of the walk.  Hop h of the chunk (counted from fs) lives in
// slot h % R of a ring of R hop slots (the pair at k reads hops k .. k+NB and
// prefetches k+NB+1, k+NB+2, so R >= NB + 3), OLA block b in acc[b % NB].  The
// loop body is unrolled U = R/2 pairs so every slot and block index is a
// compile-time constant: no register shifting, and the block a frame opens (its
// last, k+NB-1 for frame k) starts from a literal zero instead of a cleared
// register (the register held a block already produced).
template <typename F, int... I>
__device__ __forceinline__ void static_for_(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>()), ...);
}
// f(integral_constant<int, i>) for i = 0 .. n-1
template <int n, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_(f, std::make_integer_sequence<int, n>());
}

template <int NB>
struct PairRot {
    static constexpr int R = NB == 1 ? 4 : NB == 2 ? 6 : NB == 4 ? 8 : 16;
    static constexpr int U = R / 2;
    static_assert(R >= NB + 3 && (2 * U) % NB == 0, "ring");
};

// the synthesis window and gain folded into the OLA adds (ola_pair.h
// ola_pair_push_w: +1.9 % at H = 256, +1.4 % at H = 512) except at H = 128, where
// the 16 live window values double the walk's spills (-5.6 %): there the window
// product and fma(., g, acc) stay separate.  Both walkers follow the same choice.
template <int SH>
constexpr bool kPairFoldWs = SH != 2;

template <int SH, int NB, int W, bool ILV, bool HAS_GAIN>
__global__ __launch_bounds__(64 * W, CRLOT_PAIR_MIN_WAVES) void k_stft_ola_pair(const FusedArgs a) {
    constexpr int E = 16, N = 1024, H = 64 * SH;
    constexpr int R = PairRot<NB>::R, U = PairRot<NB>::U;
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
            ws4[d] = kPairFoldWs<SH> ? a.t.wsn[i] * a.gain : a.t.wsn[i];  // (ws g: ola_pair.h ola_pair_push_w)
        }
        __syncthreads();
    }
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    dev::pc* buf = reinterpret_cast<dev::pc*>(smem + PairLds<W>::bufs) + wave * dev::kPairXbuf;
    const dev::pc* t2 = t2s + (lane & 15);  // t2[16 (c-1)] = W64^{(lane & 15) c}
#if CRLOT_PAIR_REG_TW  // twiddles held in registers (3 waves per SIMD)
    // FMA-form twiddles (fft_pair.h PairTwF) at H = 256 only: at H = 128 and 512
    // their 6 extra VGPRs spill the walk (-5 % / -19 %, profiles/r05b_pairtw_ab.log)
    std::conditional_t<SH == 4, dev::PairTwReg, dev::PairTw> tw;
    dev::pair_tw_load(tw, t1, t2, lane);
    const auto& tw1 = tw;
    const auto& tw2 = tw;
#else
    const dev::pc* const tw1 = t1;
    const dev::pc* const tw2 = t2;
#endif
    // spectral gain (the spectral hook, the two-regime walker's operation): once
    // every wave holds its twiddles in registers, the per-bin gain [N] replaces
    // the twiddle table in LDS (no room for both beside three workgroups per CU)
    const float* const gl = reinterpret_cast<const float*>(smem + PairLds<W>::t1) + dev::pair_bin_lane(lane);
    if constexpr (HAS_GAIN) {
        static_assert(CRLOT_PAIR_REG_TW, "the gain table overlays the twiddle table");
        __syncthreads();
        float* gw_ = reinterpret_cast<float*>(smem + PairLds<W>::t1);
        for (int i = threadIdx.x; i < N; i += 64 * W) gw_[i] = a.t.gain[i <= N / 2 ? i : N - i];
        __syncthreads();
    }
    const int gw = blockIdx.x * W + wave;
    if (gw >= a.n_streams * a.n_chunks) return;
    const WalkId wid = walk_id<ILV>(a, gw);
    const int c = wid.c;
    const int cs = ILV ? a.cs : 1;
    const int f0 = c * a.M;
    const int f1 = min(a.F, f0 + a.M);
    const int fs = max(0, f0 - (NB - 1)) & ~1;  // pairs start on even frames
    const __amdgpu_buffer_rsrc_t rx = dev::make_rsrc(a.x + wid.xo, span_bytes(a.T, cs));
    const HopRsrc<ILV ? SH : 1> rxq = hop_rsrc<ILV ? SH : 1>(a.x + wid.xo, ILV ? a.T : 0, cs);
    auto load_hop = [&](float* dst, int origin) {
        if constexpr (ILV) {
            load_hop0s<SH>(dst, rxq, lane, origin, cs);
        } else {
            const int v = (origin + lane) * 4;
#pragma unroll
            for (int q = 0; q < SH; ++q)
                dst[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, v + q * 256, 0,
                                                                                        CRLOT_PAIR_LD_AUX));
        }
    };
    const __amdgpu_buffer_rsrc_t ry = dev::make_rsrc(a.y + wid.yo, span_bytes(a.out_len, cs));
#if CRLOT_PAIR_PKA
    const __amdgpu_buffer_rsrc_t rp2 = dev::make_rsrc(a.t.pden2, uint32_t(a.ring_blocks * H) * 16u);
#else
    const __amdgpu_buffer_rsrc_t rp = dev::make_rsrc(a.t.pden, uint32_t(a.ring_blocks * H) * 8u);
#endif
    const __amdgpu_buffer_rsrc_t ry_null = dev::make_rsrc(a.y, 0u);
    const uint32_t xlo_b = __builtin_bit_cast(uint32_t, a.t.px_lo), xhi_b = __builtin_bit_cast(uint32_t, a.t.px_hi);

    // XR(slot, q): sample lane + 64 q of the hop in that slot; bit j of hopok:
    // hop k + j (k = the current pair) keeps the paired regime.  PK2: slots 2i and
    // 2i+1 share a register pair (the pair's frames k, k+1 start on even slots), and
    // so do OLA blocks 2i and 2i+1, so half the window products, half the OLA adds
    // and every division of a frame pair run as packed operations, lane for lane
    // the same IEEE operations as the scalar ones.
#if CRLOT_PAIR_PKX
    dev::pc xr2[R / 2][SH];
#define XR(s, q) xr2[(s) / 2][q][(s) % 2]
#else
    float xr[R][SH];
#define XR(s, q) xr[s][q]
#endif
#if CRLOT_PAIR_PKA
    dev::pc acc2[NB / 2][SH];
#define CRLOT_ACC(b, q) acc2[(b) / 2][q][(b) % 2]
#pragma unroll
    for (int j = 0; j < NB / 2; ++j)
#pragma unroll
        for (int q = 0; q < SH; ++q) acc2[j][q] = dev::pc{0.f, 0.f};
#else
    float acc[NB][SH];
#define CRLOT_ACC(b, q) acc[b][q]
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int q = 0; q < SH; ++q) acc[j][q] = 0.f;
#endif
    auto load_slot = [&](auto sc, int origin) {
        constexpr int s = decltype(sc)::value;
        float t[SH];
        load_hop(t, origin);
#pragma unroll
        for (int q = 0; q < SH; ++q) XR(s, q) = t[q];
    };
    uint32_t hopok = 0;
    auto slot_ok = [&](auto sc, int at) {
        constexpr int s = decltype(sc)::value;
        // (each sample copied to a scalar before the bit cast: a bit cast applied to a
        // vector element directly is miscompiled by this clang)
        float h[SH];
#pragma unroll
        for (int q = 0; q < SH; ++q) h[q] = XR(s, q);
        uint32_t mx = 0u, mn = ~0u;
#pragma unroll
        for (int q = 0; q < SH; ++q) {  // hop_ok_bits (fused_common.h)
            const uint32_t u = __builtin_bit_cast(uint32_t, h[q]) & 0x7fffffffu;
            mx = max(mx, u);
            mn = min(mn, u - 1u);
        }
        hopok |= (__builtin_amdgcn_ballot_w64((mx > xhi_b) | (mn < xlo_b - 1u)) == 0 ? 1u : 0u) << at;
    };
    static_for<NB + 1>([&](auto hc) {
        constexpr int h = decltype(hc)::value;
        load_slot(hc, (fs + h) * H - a.pad);
        slot_ok(hc, h);
    });

    // bad: the current pair needs k_stft_ola_pair_fix (it left the paired regime,
    // an output fell below the sanitize threshold or a block outside Markstein's
    // range).  Flagged pairs (frame offsets from fs) gather in two clusters, A and
    // B: one within 2 NB frames of A's last joins A while B is empty, later ones
    // open or extend B; the fix-up walker redoes the blocks each cluster touches.
    // The divisions run for warm-up blocks too, only their stores are dropped
    // (zero-size descriptor), so the divisor loads are used unconditionally and
    // vmcnt bookkeeping stays exact at the next wait.
    bool bad = false;
    uint32_t a0 = ~0u, a1 = 0u, b0 = ~0u, b1 = 0u;
    // (k = -1: past the chunk, dropped like a warm-up store)
    auto store_block = [&](int k, const float (&o)[SH]) {
        const __amdgpu_buffer_rsrc_t rk = k >= f0 ? ry : ry_null;
#pragma unroll
        for (int q = 0; q < SH; ++q)
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o[q]), rk, lane * (4 * cs),
                                                  (k * (4 * H) + q * 256) * cs, ILV ? 0 : CRLOT_PAIR_ST_AUX);
    };
#if !CRLOT_PAIR_PKA
    // produce(H) of block k: IEEE acc / den by Markstein's correction.
    // Markstein is exact for acc = 0 and |acc| in [2^-64, 2^64] (finite sums
    // here): frexp exponents in [-63, 65], zero's being 0; any lane outside flags
    // the walk for the IEEE division of the fix-up walker (a block of sums below
    // 2^-64 or above 2^64)
    auto mk_range = [&](const auto& sums) {
        constexpr int n = sizeof(sums) / sizeof(float);
        int ex_lo = 0, ex_hi = 0;
#pragma unroll
        for (int q = 0; q < n; ++q) {
            const int e = __builtin_amdgcn_frexp_expf(sums[q]);
            ex_lo = min(ex_lo, e);
            ex_hi = max(ex_hi, e);
        }
        bad |= !((ex_lo >= -63) & (ex_hi <= 65));
    };
    auto emit = [&](int b, int k, const float (&dr)[2 * SH]) {
        mk_range(acc[b]);
        float o[SH];
#pragma unroll
        for (int q = 0; q < SH; ++q) o[q] = mk_div(acc[b][q], dr[q], dr[SH + q]);
        store_block(k, o);
    };
#endif

    constexpr uint32_t kPairHops = (1u << (NB + 1)) - 1;  // hops k .. k+NB

    // One pair (frames k, k+1) at unroll position PH: hop k in slot S0, frame
    // k's first block in acc[B0] (both even).
    auto step = [&](auto phc, int k) {
        constexpr int PH = decltype(phc)::value;
        constexpr int S0 = (2 * PH) % R, B0 = (2 * PH) % NB;
        // prefetch hops k+NB+1, k+NB+2 for the next pairs (their slots are free)
        load_slot(std::integral_constant<int, (S0 + NB + 1) % R>(), (k + NB + 1) * H - a.pad);
        load_slot(std::integral_constant<int, (S0 + NB + 2) % R>(), (k + NB + 2) * H - a.pad);
        const bool paired = (hopok & kPairHops) == kPairHops;
        bad = !paired;
        {
            // z = frame k * w + i frame k+1 * w
            dev::pc v[E];
#pragma unroll
            for (int m4 = 0; m4 < E / 4; ++m4) {
                const float4 w = *reinterpret_cast<const float4*>(wa4 + m4 * 256 + lane * 4);
                const float wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int m = 4 * m4 + u, s = (S0 + m / SH) % R;
#ifdef CRLOT_ABL_NOANAWIN  // timing-only ablation: wrong results
                    (void)wv;
                    v[m] = dev::pc_mk(XR(s, m % SH), XR((s + 1) % R, m % SH));
#else
#if CRLOT_PAIR_PKX
                    if ((m / SH) % 2 == 0)  // hops k + 2i, k + 2i + 1 share a register pair
                        v[m] = xr2[s / 2][m % SH] * dev::pc{wv[u], wv[u]};
                    else
#endif
                        v[m] = dev::pc_mk(XR(s, m % SH) * wv[u], XR((s + 1) % R, m % SH) * wv[u]);
#endif
                }
            }
            // (frame k+1 = F past the last frame of an odd count still transforms
            // the framed samples there -- zeros for ZERO_PAD, the padding rule's
            // values otherwise: deterministic per stream, and never produced)
            dev::pair_fft_fwd(v, buf, tw1, tw2, lane);
            if constexpr (HAS_GAIN) {  // real gain, symmetric over the N bins (as the two-regime walker)
#pragma unroll
                for (int d = 0; d < E; ++d) v[d] = v[d] * gl[64 * d];
            }
            // both blocks' divisors (L2-resident table) during the inverse, before
            // this pair's stores: vmcnt retires in order, so a load issued after
            // a store would also wait for that store
#if CRLOT_PAIR_PKA
            dev::pc d2[SH], r2[SH];  // (den_k, den_k+1) q and (rden_k, rden_k+1) q (DevTables::pden2)
            load_den_pair<64, SH>(d2, r2, rp2, lane, k % a.ring_blocks);
#else
            float dr0[2 * SH], dr1[2 * SH];
            load_den<SH>(dr0, rp, lane, k % a.ring_blocks);
            load_den<SH>(dr1, rp, lane, (k + 1) % a.ring_blocks);
#endif
            dev::pair_fft_inv(v, buf, tw1, tw2, lane);
            // output sanitize (kissfft_adapter.cc:156-163): finite here, so only its
            // threshold |v| < 1e-30 N (= 2^-89.66 N / 1024) can act, and only on a
            // nonzero v.  frexp exponents find every 0 < |v| < 2^-89 (zero's is 0):
            // one such value sends the walk to k_stft_ola_pair_fix (a value in
            // [1e-30 N, 2^-89) too, harmlessly), otherwise the sanitize is the identity.
            static_assert(N == 1024, "threshold exponent");
#if defined(CRLOT_ABL_NOOSAN)  // timing-only ablation
#elif CRLOT_PAIR_OSCREEN  // (the same test, screened: fft_pair.h)
            bad |= dev::out_min_exp_screened<E>(v, 0x1p-89f) <= -89;
#else
            {
                int e[4] = {0, 0, 0, 0};
#pragma unroll
                for (int m = 0; m < E; ++m)
                    e[m & 3] = min(e[m & 3], min(__builtin_amdgcn_frexp_expf(v[m].x), __builtin_amdgcn_frexp_expf(v[m].y)));
                bad |= min(min(e[0], e[1]), min(e[2], e[3])) <= -89;
            }
#endif
            // push_frame_AoS of both frames with the window and gain folded into
            // the adds, fma(v, ws g, acc) (ola_pair.h ola_pair_push_w); at H = 128
            // fma(fma(o, w, 0), g, acc) with the window product of both parts in one
            // packed multiply (v * (w, w) gives -0 only where fma(o, w, 0) gives +0,
            // and fma(-0, g, acc) == fma(+0, g, acc)) and wg = g
            float wg[E];
#pragma unroll
            for (int m4 = 0; m4 < E / 4; ++m4) {
                const float4 w = *reinterpret_cast<const float4*>(ws4 + m4 * 256 + lane * 4);
                const float wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if constexpr (kPairFoldWs<SH>) {
                        wg[4 * m4 + u] = wv[u];
                    } else {
                        v[4 * m4 + u] = v[4 * m4 + u] * dev::pc{wv[u], wv[u]};
                        wg[4 * m4 + u] = a.gain;
                    }
                }
            }
#if CRLOT_PAIR_PKA
            // (ola_pair.h: both frames' adds, then the produce of blocks k and k+1)
            ola_pair_push_w<E, SH, NB, B0>(acc2, v, wg);
            {
                float o0[SH], o1[SH];
                bad |= !mk_div_pair<SH>(acc2[B0 / 2], d2, r2, o0, o1);
                store_block(k, o0);
                store_block(k + 1 < f1 ? k + 1 : -1, o1);  // (past the chunk when k+1 == f1)
            }
            ola_pair_open_w<E, SH, NB, B0>(acc2, v, wg);
#else
            // frame k -> blocks k .. k+NB-1 (the last opens), produce block k
#pragma unroll
            for (int m = 0; m < E; ++m) {
                CRLOT_ACC((B0 + m / SH) % NB, m % SH) =
                    __builtin_fmaf(v[m].x, wg[m], m / SH == NB - 1 ? 0.0f : CRLOT_ACC((B0 + m / SH) % NB, m % SH));
            }
            emit(B0, k, dr0);
            // frame k+1 -> blocks k+1 .. k+NB (k+NB opens in acc[B0]), produce block k+1
            // (past the chunk when k+1 == f1: dropped like a warm-up store)
#pragma unroll
            for (int m = 0; m < E; ++m) {
                CRLOT_ACC((B0 + 1 + m / SH) % NB, m % SH) =
                    __builtin_fmaf(v[m].y, wg[m], m / SH == NB - 1 ? 0.0f : CRLOT_ACC((B0 + 1 + m / SH) % NB, m % SH));
            }
            emit((B0 + 1) % NB, k + 1 < f1 ? k + 1 : -1, dr1);
#endif
        }
        {  // (selects, no branch: wave-uniform scalar state)
            const bool f = __builtin_amdgcn_ballot_w64(bad) != 0;
            const uint32_t o = uint32_t(k - fs);
            const bool new_a = f & (a0 == ~0u);
            const bool to_a = f & !new_a & (b0 == ~0u) & (o <= a1 + 2 * NB);
            const bool to_b = f & !new_a & !to_a;
            a0 = new_a ? o : a0;
            a1 = (new_a | to_a) ? o : a1;
            b0 = (to_b & (b0 == ~0u)) ? o : b0;
            b1 = to_b ? o : b1;
        }
#ifdef CRLOT_ABL_NOHOPCHK  // timing-only ablation
        hopok = ~0u;
#else
        slot_ok(std::integral_constant<int, (S0 + NB + 1) % R>(), NB + 1);
        slot_ok(std::integral_constant<int, (S0 + NB + 2) % R>(), NB + 2);
        hopok >>= 2;
#endif
    };
    for (int k = fs; k < f1; k += 2 * U) {
        step(std::integral_constant<int, 0>(), k);
        if constexpr (U > 1) {
            if (k + 2 >= f1) break;
            step(std::integral_constant<int, 1>(), k + 2);
        }
        if constexpr (U > 2) {
            if (k + 4 >= f1) break;
            step(std::integral_constant<int, 2>(), k + 4);
        }
        if constexpr (U > 3) {
            if (k + 6 >= f1) break;
            step(std::integral_constant<int, 3>(), k + 6);
        }
        if constexpr (U > 4) {
            if (k + 8 >= f1) break;
            step(std::integral_constant<int, 4>(), k + 8);
            if (k + 10 >= f1) break;
            step(std::integral_constant<int, 5>(), k + 10);
            if (k + 12 >= f1) break;
            step(std::integral_constant<int, 6>(), k + 12);
            if (k + 14 >= f1) break;
            step(std::integral_constant<int, 7>(), k + 14);
        }
    }
    // flag words of the walker (cluster A at gw, B at gw + walkers): pair offsets
    // from fs + 1 of its first and last pair, 16 bits each; 1 = the whole chunk
    // (offsets that do not fit), 0 = nothing to redo
    const uint32_t pl = (b0 != ~0u ? b1 : a1) / 2u + 1u;
    const uint32_t fa = a0 == ~0u ? 0u : pl >= 0xffffu ? 1u : (a0 / 2u + 1u) | (a1 / 2u + 1u) << 16;
    const uint32_t fb = (b0 == ~0u || pl >= 0xffffu) ? 0u : (b0 / 2u + 1u) | (b1 / 2u + 1u) << 16;
    if (lane == 0) {
        a.t.pflags[gw] = fa;
        a.t.pflags[gw + a.n_streams * a.n_chunks] = fb;
    }
}
#undef CRLOT_ACC
#undef XR


// K_pair fix-up walker k_stft_ola_pair_fix: the walk with both regimes, run
// after k_stft_ola_pair over the chunks it flagged (never on finite audio; the
// launch exits at once otherwise).  Its paired pairs compute exactly what the
// paired-only walker computes, so a redone chunk has the same bits wherever
// both regimes would have agreed.
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
template <int SH, int NB, int W, bool HAS_GAIN, bool ILV>
__global__ __launch_bounds__(64 * W, CRLOT_PAIR_MIN_WAVES) void k_stft_ola_pair_fix(const FusedArgs a) {
    constexpr int E = 16, N = 1024, H = 64 * SH;
    static_assert(NB * SH == E, "N = NB * H");
    static_assert(SH >= 2, "den rows are read 16 bytes at a time");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    {  // only walkers the paired-only pass flagged; whole workgroups leave together.
       // The vote goes through the (still unused) transpose buffers rather than
       // __syncthreads_or, whose 256 B of static LDS would not fit beside a
       // 16-wave workgroup's 160 KB.
        const int64_t w0 = int64_t(blockIdx.x) * W;
        const int t = threadIdx.x;
        uint32_t* vote = reinterpret_cast<uint32_t*>(smem + PairLds<W>::bufs);
        if (t < W)
            vote[t] = (w0 + t < int64_t(a.n_streams) * a.n_chunks && (a.fix_all || a.t.pflags[w0 + t] != 0u)) ? 1u : 0u;
        __syncthreads();
        uint32_t any = 0;
#pragma unroll
        for (int i = 0; i < W; ++i) any |= vote[i];
        if (!any) return;
    }
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
            ws4[d] = kPairFoldWs<SH> ? a.t.wsn[i] * a.gain : a.t.wsn[i];  // (ws g: ola_pair.h ola_pair_push_w)
        }
        __syncthreads();
    }
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    dev::pc* buf = reinterpret_cast<dev::pc*>(smem + PairLds<W>::bufs) + wave * dev::kPairXbuf;
    const dev::pc* t2 = t2s + (lane & 15);  // t2[16 (c-1)] = W64^{(lane & 15) c}
    const int gw = blockIdx.x * W + wave;
    if (gw >= a.n_streams * a.n_chunks || (!a.fix_all && a.t.pflags[gw] == 0u)) return;
    const WalkId wid = walk_id<ILV>(a, gw);
    const int c = wid.c;
    const int cs = ILV ? a.cs : 1;  // interleaved groups: zero padding only (host-checked)
    // Block ranges to redo.  The hot walker's flag words name up to two clusters of
    // pairs it could not finish (first and last pair, offsets from its walk start
    // + 1, low / high halves; 1: the whole chunk): the blocks a cluster touches,
    // [k_first, k_last + NB], are redone from NB-1 frames of warm-up before them.
    const int c0 = c * a.M, c1 = min(a.F, c0 + a.M);
    int rng[2][2] = {{c0, c1}, {c0, c0}};
    {
        const uint32_t fa = a.fix_all ? 1u : a.t.pflags[gw];
        if (fa > 1u) {
            const uint32_t fb = a.t.pflags[gw + a.n_streams * a.n_chunks];
            const int ws0 = max(0, c0 - (NB - 1)) & ~1;
            const uint32_t fl[2] = {fa, fb};
#pragma unroll
            for (int r = 0; r < 2; ++r)
                if (fl[r] > 1u) {
                    rng[r][0] = max(c0, ws0 + 2 * int((fl[r] & 0xffffu) - 1u));
                    rng[r][1] = min(c1, ws0 + 2 * int((fl[r] >> 16) - 1u) + NB + 1);
                }
        }
    }
    int f0 = c0, f1 = c1;  // the range being redone
    const __amdgpu_buffer_rsrc_t rx = dev::make_rsrc(a.x + wid.xo, span_bytes(a.T, cs));
    const __amdgpu_buffer_rsrc_t ry = dev::make_rsrc(a.y + wid.yo, span_bytes(a.out_len, cs));
    const HopRsrc<ILV ? SH : 1> rxq = hop_rsrc<ILV ? SH : 1>(a.x + wid.xo, ILV ? a.T : 0, cs);
    auto load_hop = [&](float* dst, int origin) {
        if constexpr (ILV)
            load_hop0s<SH>(dst, rxq, lane, origin, cs);
        else
            load_hop1<SH>(dst, rx, lane, origin, a.T, a.pad_mode);
    };
    const __amdgpu_buffer_rsrc_t rp = dev::make_rsrc(a.t.pden, uint32_t(a.ring_blocks * H) * 8u);
    const __amdgpu_buffer_rsrc_t ry_null = dev::make_rsrc(a.y, 0u);
    const float xlo = a.t.px_lo, xhi = a.t.px_hi;

    for (int r = 0; r < 2; ++r) {
    f0 = rng[r][0];
    f1 = rng[r][1];
    if (f0 >= f1) continue;
    const int fs = max(0, f0 - (NB - 1)) & ~1;  // pairs start on even frames
    // xin[h*SH + q]: hop (k + h), h = 0..NB, sample lane + 64 q of the hop;
    // bit h of hopok: hop k + h keeps the paired regime
    float xin[E + SH];
    uint32_t hopok = 0;
#pragma unroll
    for (int h = 0; h <= NB; ++h) {
        load_hop(xin + h * SH, (fs + h) * H - a.pad);
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
            const float4 w = *reinterpret_cast<const float4*>(ws4 + m4 * 256 + lane * 4);
            const float wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int m = 4 * m4 + u;
                const float x = imag ? v[m].y : v[m].x;
                const float o = paired ? dev::sanit_scaled_finite<N>(x) : dev::sanit_scaled<N>(x);
                float& r = acc[m / SH][m % SH];
                if constexpr (kPairFoldWs<SH>)
                    r = __builtin_fmaf(o, wv[u], r);  // (ws g staged: ola_pair.h ola_pair_push_w)
                else
                    r = __builtin_fmaf(__builtin_fmaf(o, wv[u], 0.0f), a.gain, r);
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
        // warm-up blocks (k < f0) store through a zero-size descriptor: every
        // lane is out of range and the store is dropped.  No branch around the
        // stores, so vmcnt bookkeeping stays exact at the next divisor wait.
        const __amdgpu_buffer_rsrc_t rk = k >= f0 ? ry : ry_null;
#pragma unroll
        for (int q = 0; q < SH; ++q)
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o[q]), rk, lane * (4 * cs),
                                                  (k * (4 * H) + q * 256) * cs, 0);
#pragma unroll
        for (int j = 0; j < NB - 1; ++j)
#pragma unroll
            for (int q = 0; q < SH; ++q) acc[j][q] = acc[j + 1][q];
#pragma unroll
        for (int q = 0; q < SH; ++q) acc[NB - 1][q] = 0.f;
    };

#if CRLOT_PAIR_REG_TW  // twiddles held in registers (3 waves per SIMD)
    // FMA-form twiddles (fft_pair.h PairTwF) at H = 256 only: at H = 128 and 512
    // their 6 extra VGPRs spill the walk (-5 % / -19 %, profiles/r05b_pairtw_ab.log)
    std::conditional_t<SH == 4, dev::PairTwReg, dev::PairTw> tw;
    dev::pair_tw_load(tw, t1, t2, lane);
    const auto& tw1 = tw;
    const auto& tw2 = tw;
#else
    const dev::pc* const tw1 = t1;
    const dev::pc* const tw2 = t2;
#endif
    auto transform = [&](dev::pc (&v)[E]) {  // forward, spectral gain, inverse (unnormalised)
        dev::pair_fft_fwd(v, buf, tw1, tw2, lane);
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
    };
    constexpr uint32_t kPairHops = (1u << (NB + 1)) - 1;  // hops k .. k+NB
    for (int k = fs; k < f1; k += 2) {
        // prefetch hops k+NB+1, k+NB+2 for the next pair
        float nxt[2 * SH];
        load_hop(nxt, (k + NB + 1) * H - a.pad);
        load_hop(nxt + SH, (k + NB + 2) * H - a.pad);
        const bool paired = (hopok & kPairHops) == kPairHops;
        if (paired) {
            dev::pc v[E];
#pragma unroll
            for (int m4 = 0; m4 < E / 4; ++m4) {
                const float4 w = *reinterpret_cast<const float4*>(wa4 + m4 * 256 + lane * 4);
                const float wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int m = 4 * m4 + u;
                    v[m] = dev::pc_mk(xin[m] * wv[u], xin[m + SH] * wv[u]);
                }
            }
            transform(v);
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
    }  // ranges
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

// Diagnostic builds only (-DCRLOT_PAIR_NOFIX_DIAG, e.g. `make variant`):
// CRLOT_PAIR_NOFIX=1 then skips the fix-up walker to time how much it redoes,
// leaving flagged chunks wrong.  The release library always runs it.
bool pair_nofix() {
#ifdef CRLOT_PAIR_NOFIX_DIAG
    static const bool v = [] {
        const char* e = ab_env("CRLOT_PAIR_NOFIX");
        return e && e[0] == '1';
    }();
    return v;
#else
    return false;
#endif
}

// The paired-only walker at hops of 128, 256 and 512, with or without a spectral
// gain (the gain table overlays the twiddle table, so only with register
// twiddles).  H = 512 keeps 6 hop slots (a few VGPR spills, outside the hot
// path's cost: +10 % over the two-regime walker, profiles/r03_pair_hot_hops_ab.jsonl);
// H = 128 spills more and gains 1.5 %.
// Other hops and reflect / edge padding run the two-regime walker over every chunk.
template <int SH>
constexpr bool pair_hot() {
    return (SH == 2 && CRLOT_PAIR_HOT2) || SH == 4 || (SH == 8 && CRLOT_PAIR_HOT8);
}

#ifdef CRLOT_PAIR32_EXPERIMENT
bool pair32_enabled();                                            // tools/experiments/pair32.hip
hipError_t launch_pair32(const FusedArgs& a, hipStream_t stream);
#endif

template <int SH, bool ILV>
hipError_t pair_sh(const FusedArgs& a, int64_t waves, hipStream_t stream) {
    constexpr int NB = 16 / SH, W = kPairWaves;
    const size_t lds = PairLds<W>::bytes;
    const int64_t grid = (waves + W - 1) / W;
    hipError_t e;
    if (ILV && (a.cs < 1 || a.pad_mode != 0)) return hipErrorInvalidValue;
    auto kf = a.t.gain ? k_stft_ola_pair_fix<SH, NB, W, true, ILV> : k_stft_ola_pair_fix<SH, NB, W, false, ILV>;
    if ((e = set_lds(kf, lds)) != hipSuccess) return e;
    if (!a.t.pflags || a.t.pflags_len < waves) return hipErrorInvalidValue;
    if constexpr (pair_hot<SH>()) {
#ifdef CRLOT_PAIR32_EXPERIMENT
        if (!ILV && pair32_enabled() && a.pad_mode == 0 && a.t.hot && !a.t.gain) {
            if ((e = launch_pair32(a, stream)) != hipSuccess) return e;
            note_launch(CRLOT_K_PAIR_FIX, grid);
            hipLaunchKernelGGL(kf, dim3(unsigned(grid)), dim3(64 * W), lds, stream, a);
            return hipGetLastError();
        }
#endif
        if (a.pad_mode == 0 && a.t.hot && (!a.t.gain || CRLOT_PAIR_REG_TW)) {
            if (CRLOT_PAIR_PKA && !a.t.pden2) return hipErrorInvalidValue;
            if (a.t.pflags_len < 2 * waves) return hipErrorInvalidValue;  // two flag words per walker
            auto k = a.t.gain ? k_stft_ola_pair<SH, NB, W, ILV, CRLOT_PAIR_REG_TW != 0> : k_stft_ola_pair<SH, NB, W, ILV, false>;
            if ((e = set_lds(k, lds)) != hipSuccess) return e;
            note_launch(CRLOT_K_PAIR_HOT, grid);
            hipLaunchKernelGGL(k, dim3(unsigned(grid)), dim3(64 * W), lds, stream, a);
            if ((e = hipGetLastError()) != hipSuccess) return e;
            if (pair_nofix()) return hipSuccess;  // diagnostics only: flagged chunks stay wrong
            note_launch(CRLOT_K_PAIR_FIX, grid);
            hipLaunchKernelGGL(kf, dim3(unsigned(grid)), dim3(64 * W), lds, stream, a);
            return hipGetLastError();
        }
    }
    FusedArgs b = a;
    b.fix_all = 1;
    note_launch(CRLOT_K_PAIR_ALL, grid);
    hipLaunchKernelGGL(kf, dim3(unsigned(grid)), dim3(64 * W), lds, stream, b);
    return hipGetLastError();
}

hipError_t launch_pair(int sh, const FusedArgs& a, int64_t waves, hipStream_t stream) {
    if (a.cs != 1) {
        switch (sh) {
            case 2: return pair_sh<2, true>(a, waves, stream);
            case 4: return pair_sh<4, true>(a, waves, stream);
            case 8: return pair_sh<8, true>(a, waves, stream);
            default: return hipErrorInvalidValue;
        }
    }
    switch (sh) {
        case 2: return pair_sh<2, false>(a, waves, stream);
        case 4: return pair_sh<4, false>(a, waves, stream);
        case 8: return pair_sh<8, false>(a, waves, stream);
        case 16: return pair_sh<16, false>(a, waves, stream);
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

