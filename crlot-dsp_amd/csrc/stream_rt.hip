// stream_rt.hip -- K_stream_rt: the resident low-latency streaming kernel
// (BASELINE config 4: 64 channels, N = 512, H = 128, one hop every 2.67 ms).
//
// A per-hop launch costs ~6 us of device time and ~15 us of host wall time
// even for an empty kernel (harness/stream_latency), far more than the hop's
// arithmetic (~1.5 us).  K_stream_rt is launched once and stays resident:
//   * the tables (twiddles, super twiddles, both windows, spectral gain) are
//     staged into LDS once per launch;
//   * each channel's state -- the last N-H input samples and the N/H OLA blocks
//     still open -- lives in the wave's registers between hops (saved to HBM
//     only when the kernel exits, restored on the next launch);
//   * hops arrive through pinned host memory: the host writes hop q into ring
//     slot q % depth (channel-major [C][H]) and bumps `seq`; thread 0 of every
//     workgroup polls `seq`, each wave reads its channel's H samples straight
//     from host memory (system-coherent loads, one PCIe read per 128-byte line),
//     transforms, writes its H output samples straight into the host output
//     slot and the workgroup publishes `done[wg] = q + 1` (system-scope release).
//     Interleaved PCM is transposed by the host while it copies a hop in or out.
// The arithmetic per hop is k_stream_hop's operation for operation (kernels.hip:
// sanitize(x*wa) -> fft_wave -> real_split_hook_merge -> fft_wave^-1 ->
// sanitize(*1/N) -> fma(fma(o, ws, 0), g, acc) -> acc / den), so the output is
// bit-identical to crlot_stream_push_hop and to the batched DROP round trip with
// frame pairing off.
//
// Exit conditions every wave reaches: `stop` set by the host, or no new hop for
// `idle_ticks` of the 100 MHz s_memrealtime clock.  The host relaunches on the
// next hop when it finds the kernel gone (abi.cpp crlot_stream_rt_*).  There is
// no inter-workgroup dependency: each workgroup waits only on the host.
#include "fft_wave.h"
#include "kernels.h"

namespace crlot {

using dev::cf;

namespace {

constexpr int kRtWaves = 4;
constexpr int kRtBlock = 64 * kRtWaves;

template <int E>
struct RtLds {
    static constexpr int P = 64 * E, N = 2 * P;
    static constexpr int TW = dev::twiddle_table_size(E);
    // [tw TW cf][st P cf][sth P cf][bufs 4 P cf][wa N][ws N][gain P + 64][cmd 2 x u32]
    static constexpr size_t cf_elems = size_t(TW) + 2 * P + size_t(kRtWaves) * P;
    static constexpr size_t f_elems = 2 * size_t(N) + P + 64;
    static constexpr size_t fixed = sizeof(cf) * cf_elems + sizeof(float) * f_elems + 16;
};

// Host-memory reads: relaxed system-scope loads (sc0 sc1: straight to memory,
// no cache line kept) rather than an acquire fence, which would invalidate the
// whole L2 on every hop.  The hop's bytes are read only after thread 0 saw the
// doorbell and the workgroup passed a barrier; the host wrote them before it.
__device__ __forceinline__ uint64_t ld_sys64(const void* p) {
    return __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ float ld_sys32(const float* p) {
    return __uint_as_float(
        __hip_atomic_load(reinterpret_cast<const uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
}
__device__ __forceinline__ float2 ld_sys2(const float* p) {
    const uint64_t v = ld_sys64(p);
    return make_float2(__uint_as_float(uint32_t(v)), __uint_as_float(uint32_t(v >> 32)));
}

template <int E, int S, bool HAS_GAIN>
__global__ __launch_bounds__(kRtBlock) void k_stream_rt(const RtArgs a) {
    constexpr int P = 64 * E, N = 2 * P, H = 128 * S, NB = E / S, TW = RtLds<E>::TW;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    cf* st = tw + TW;
    cf* sth = st + P;
    cf* bufs = sth + P;
    float* wa = reinterpret_cast<float*>(bufs + kRtWaves * P);
    float* ws = wa + N;
    float* gain = ws + N;
    uint32_t* cmd = reinterpret_cast<uint32_t*>(gain + P + 64);

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c0 = blockIdx.x * kRtWaves;
    const int c = c0 + wave;
    const bool live = c < a.channels;
    const int C = a.channels;
    RtCtl* ctl = a.ctl;

    // ---- once per launch: tables into LDS, channel state into registers
    {
        const cf* gtw = reinterpret_cast<const cf*>(a.t.tw);
        const cf* gst = reinterpret_cast<const cf*>(a.t.st);
        for (int i = threadIdx.x; i < TW; i += kRtBlock) tw[i] = gtw[i];
        for (int i = threadIdx.x; i < P; i += kRtBlock) {
            const cf w = gst[i];
            st[i] = w;
            sth[i] = cf{w.r * 0.5f, w.i * 0.5f};  // exact
        }
        for (int i = threadIdx.x; i < N; i += kRtBlock) {
            wa[i] = a.t.wa[i];
            ws[i] = a.t.ws[i];
        }
        if (HAS_GAIN)
            for (int i = threadIdx.x; i <= P; i += kRtBlock) gain[i] = a.t.gain[i];
    }
    // lane owns frame samples i0, i0 + 1 of register m, i0 = 2 (lane + 64 m) =
    // 128 m + 2 lane, so a shift by one hop (H = 128 S samples) moves m by S and
    // keeps every sample in its lane.
    float2 hist[NB > 1 ? E - S : 1];  // frame samples H .. N-1 of the next frame's predecessor
    float2 acc[E];                    // OLA blocks f .. f+NB-1 (S registers each)
    {
        const float* sv = a.state + int64_t(live ? c : 0) * (2 * N);
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int i0 = 2 * (lane + 64 * m);
            if (m < E - S) hist[m] = *reinterpret_cast<const float2*>(sv + i0);
            acc[m] = *reinterpret_cast<const float2*>(sv + N + i0);
        }
    }
    uint64_t my = __hip_atomic_load(&ctl->done[blockIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __syncthreads();

    uint64_t t_last = wall_clock64();
    for (;;) {
        const int64_t q = int64_t(my);
        const bool frame = q >= NB - 1;
        const int64_t f = q - (NB - 1);
        // divisors of block f (device memory, independent of the hop's data):
        // requested before the wait
        float2 dd[S];
#pragma unroll
        for (int m = 0; m < S; ++m) {
            const int64_t n = f * H + 2 * (lane + 64 * m);
            dd[m] = frame ? make_float2(a.t.den[n % a.ring_len], a.t.den[(n + 1) % a.ring_len])
                          : make_float2(1.f, 1.f);
        }
        // ---- wait for hop `my` (thread 0 polls, the workgroup follows)
        if (threadIdx.x == 0) {
            uint32_t k = 0;
            for (;;) {
                // seq first, stop only when seq has not moved (requesting both
                // together measured 1-2 us slower per hop on the same box)
                if (ld_sys64(&ctl->seq) > my) {
                    k = 1;
                    break;
                }
                if (ld_sys64(&ctl->stop) != 0) break;
                if (wall_clock64() - t_last > a.idle_ticks) {
                    // idle exit, decided once for the whole grid: stop = 2 makes every
                    // other workgroup leave at its next poll too, so the kernel is gone
                    // (and the host relaunches it for the next doorbell) instead of
                    // some workgroups serving hops while others wait out their own timers
                    __hip_atomic_store(&ctl->stop, uint64_t(2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            cmd[my & 1] = k;
        }
        __syncthreads();
        if (cmd[my & 1] == 0) break;
        const uint64_t t0 = wall_clock64();
#ifdef CRLOT_RT_PHASES
#define RT_PH(i) if (threadIdx.x == 0 && blockIdx.x == 0) ctl->phase[i] = wall_clock64() - t0
#else
#define RT_PH(i)
#endif
        const int slot = int(q % a.depth);
        const float* in_slot = a.in_ring + int64_t(slot) * C * H;
        float* out_slot = a.out_ring + int64_t(slot) * C * H;
        // slots are channel-major [C][H]: a wave reads its channel's H samples as
        // coalesced 512-byte rows (one PCIe read per line, no line shared
        // between workgroups)
        float2 hop[S];
#pragma unroll
        for (int s2 = 0; s2 < S; ++s2)
            hop[s2] = live ? ld_sys2(in_slot + int64_t(c) * H + 2 * (lane + 64 * s2)) : make_float2(0.f, 0.f);
        RT_PH(0);
        if (live && frame) {
            cf* buf = bufs + wave * P;
            cf v[E];
#pragma unroll
            for (int m = 0; m < E; ++m) {
                const int i0 = 2 * (lane + 64 * m);
                const float2 x2 = m >= E - S ? hop[m - (E - S)] : hist[m];
                v[m].r = dev::sanit(x2.x * wa[i0]);
                v[m].i = dev::sanit(x2.y * wa[i0 + 1]);
            }
            dev::fft_wave<E, false>(v, buf, tw, lane);
            dev::real_split_hook_merge<E, HAS_GAIN, false>(v, buf, st, sth, gain, lane);
            dev::fft_wave<E, true>(v, buf, tw, lane);
#pragma unroll
            for (int m = 0; m < E; ++m) {
                const int i0 = 2 * (lane + 64 * m);
                const float o0 = dev::sanit(v[m].r * a.inv_n);
                const float o1 = dev::sanit(v[m].i * a.inv_n);
                acc[m].x = __builtin_fmaf(__builtin_fmaf(o0, ws[i0], 0.0f), a.gain, acc[m].x);
                acc[m].y = __builtin_fmaf(__builtin_fmaf(o1, ws[i0 + 1], 0.0f), a.gain, acc[m].y);
            }
            RT_PH(2);
            // block f is complete: produce(H), straight into the host slot
#pragma unroll
            for (int m = 0; m < S; ++m) {
                const int pos = 2 * (lane + 64 * m);
                *reinterpret_cast<float2*>(out_slot + int64_t(c) * H + pos) =
                    make_float2(acc[m].x / dd[m].x, acc[m].y / dd[m].y);
            }
            RT_PH(3);
        }
        // slide the state by one hop
        if (frame) {
#pragma unroll
            for (int m = 0; m < E; ++m) acc[m] = m + S < E ? acc[m + S] : make_float2(0.f, 0.f);
        }
#pragma unroll
        for (int m = 0; m < E - S; ++m) hist[m] = m + S < E - S ? hist[m + S] : hop[m + S - (E - S)];
        // ---- publish: outputs visible system-wide, then done[wg]
        RT_PH(4);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        RT_PH(5);
        __syncthreads();
        RT_PH(6);
        my += 1;
        if (threadIdx.x == 0) {
            ctl->ticks[blockIdx.x] = wall_clock64() - t0;
            __hip_atomic_store(&ctl->done[blockIdx.x], my, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        t_last = wall_clock64();
    }
    // ---- exit: save the channel state for the next launch
    if (live) {
        float* sv = a.state + int64_t(c) * (2 * N);
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const int i0 = 2 * (lane + 64 * m);
            if (m < E - S) *reinterpret_cast<float2*>(sv + i0) = hist[m];
            *reinterpret_cast<float2*>(sv + N + i0) = acc[m];
        }
    }
}

template <int E, int S>
hipError_t rt_es(const RtArgs& a, hipStream_t stream) {
    auto k = a.t.gain ? k_stream_rt<E, S, true> : k_stream_rt<E, S, false>;
    const size_t lds = RtLds<E>::fixed;
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3(unsigned(stream_rt_workgroups(a.channels))), dim3(kRtBlock), lds, stream, a);
    return hipGetLastError();
}

template <int E>
hipError_t rt_e(int s, const RtArgs& a, hipStream_t stream) {
    if constexpr (E >= 1) {
        if (s == 1) return rt_es<E, 1>(a, stream);
    }
    if constexpr (E >= 2) {
        if (s == 2) return rt_es<E, 2>(a, stream);
    }
    if constexpr (E >= 4) {
        if (s == 4) return rt_es<E, 4>(a, stream);
    }
    if constexpr (E >= 8) {
        if (s == 8) return rt_es<E, 8>(a, stream);
    }
    if constexpr (E >= 16) {
        if (s == 16) return rt_es<E, 16>(a, stream);
    }
    return hipErrorInvalidValue;
}

}  // namespace

int stream_rt_workgroups(int channels) { return (channels + kRtWaves - 1) / kRtWaves; }

hipError_t launch_stream_rt(const Geometry& g, const RtArgs& a, hipStream_t stream) {
    if (!fused_supported(g.n, g.h) || a.channels <= 0 || a.channels > kRtMaxChannels || a.depth <= 0)
        return hipErrorInvalidValue;
    const int s = g.h / 128;
    switch (g.n) {
        case 256: return rt_e<2>(s, a, stream);
        case 512: return rt_e<4>(s, a, stream);
        case 1024: return rt_e<8>(s, a, stream);
        case 2048: return rt_e<16>(s, a, stream);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace crlot
