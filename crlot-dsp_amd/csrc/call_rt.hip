// call_rt.hip -- K_call: the resident server behind the reference's
// host-pointer, one-call-at-a-time API (the drop-in per-frame loop of
// bench/e2e_benchmark.cc:152-170: Framer::pop -> IFftPlan::forward ->
// IFftPlan::inverse -> OLAAccumulator::push_frame_AoS -> produce).
//
// A launch + synchronize costs ~15 us of host wall time even for an empty kernel
// (DESIGN.md section 5), several times the reference's whole per-frame CPU cost.
// K_call is launched once per object and stays resident (one 256-thread
// workgroup); a call is a request descriptor:
//   * the host copies the call's input (a frame, a spectrum, OLA samples) and the
//     128-byte descriptor into fine-grained DEVICE memory through the BAR with
//     write-combined stores, then bumps `seq` there (posted PCIe writes land in
//     order), so the kernel polls and reads its own HBM, not host memory;
//   * the kernel runs the call (the same device arithmetic as the launched
//     kernels: fft_wave + kiss_fftr split / merge, the OLA ring ops, the scalar
//     OLA kernels), writes the result straight into pinned HOST memory, fences
//     at system scope and publishes done = seq;
//   * speculation (bit-identical, validated by the host): after a forward real
//     FFT the kernel also runs the inverse of the spectrum it just produced
//     (IFftPlan::inverse is almost always called next on exactly those bits),
//     and after an OLA add it computes the produce(n) block the host predicts,
//     without clearing; each lands in a host slot with its own counter.  The
//     host serves the next call from a slot only when the call's inputs match
//     the speculated ones bit for bit (memcmp of the spectrum; equal read
//     position and count with no call in between), else it submits the call.
//     A served produce is committed by a clear-only request.
// Exit conditions every thread reaches: `stop` (host 1, or 2 written by the
// kernel itself on idle), or no request for `idle_ticks` of the 100 MHz clock;
// the host relaunches on the next call (call.cpp).
#include <map>
#include <mutex>

#include "fft_any.h"
#include "fft_wave.h"
#include "kernels.h"

namespace crlot {

using dev::cf;

namespace {

constexpr int kCallBlock = 256;
constexpr int kCallWaves = kCallBlock / 64;
// the first kCallPre floats of a request's input slot are fetched together with
// its descriptor (the slot's place is known before the descriptor is read), so a
// call of up to 4 KB of input pays one memory latency, not two
constexpr int kCallPre = 4 * kCallBlock;
constexpr size_t kAnyPlanBytes = (sizeof(dev::any::Plan) + 15) / 16 * 16;

// input float i (and i + 1) of the request: from the prefetched copy in LDS
// when the whole input fits it (PRE, decided once per request), else memory
template <bool PRE>
struct CallIn {
    const float* mem;
    const float* pre;
    __device__ __forceinline__ float at(int64_t i) const { return PRE ? pre[i] : ld_sys32_(mem + i); }
    __device__ __forceinline__ float2 at2(int64_t i) const {
        if constexpr (PRE) return *reinterpret_cast<const float2*>(pre + i);
        const uint64_t v = __hip_atomic_load(reinterpret_cast<const uint64_t*>(mem + i), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM);
        return make_float2(__uint_as_float(uint32_t(v)), __uint_as_float(uint32_t(v >> 32)));
    }
    __device__ static __forceinline__ float ld_sys32_(const float* p) {
        return __uint_as_float(
            __hip_atomic_load(reinterpret_cast<const uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    }
};

// fine-grained device memory written by the host (relaxed system-scope loads:
// straight from memory, nothing kept in L2) and host memory written by us
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
__device__ __forceinline__ void st_sys64(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// LDS: [tw TW cf][st P cf][sth P cf][bufs kCallWaves x P cf][spec kCallWaves x (P+1) cf][req 128 B][cmd]
// (the speculation buffers hold each wave's spectrum for the speculative
// inverse; N = 4096 plans go without speculation to stay within 160 KB)
// E < 0 (any size, fft_any.h): the request's static part first, then per FFT
// wave its Stockham buffers A, B (P cf each) and the spectrum S (P + 1 cf) kept
// for the speculated inverse, P = CallArgs::any_p at run time; tables stay in
// global memory (L2)
template <int E>
struct CallLds {
    static constexpr int P = E > 0 ? 64 * E : 1;
    static constexpr int TW = E > 0 ? dev::twiddle_table_size(E) : 1;
    static constexpr bool SPEC = E > 0 && E <= 16;
    static constexpr int SP = SPEC ? P + 1 : 0;
    static constexpr int CH = SPEC ? 2 * P : 0;  // a chained frame (one inverse output, floats)
    // two of them, by request parity: a late commit (kCallPendLate) reads the
    // previous request's frame while this request keeps its own
    static constexpr size_t bytes = sizeof(cf) * (size_t(TW) + 2 * P + size_t(kCallWaves) * (P + SP)) +
                                    sizeof(float) * (kCallPre + 2 * CH) + sizeof(CallReq) + 16;
};

// ---- FFTs, one wave per transform (k_rfft / k_irfft / k_cfft's arithmetic)
template <int E>
__device__ __forceinline__ void rfft_core(cf (&v)[E], cf* buf, const cf* tw, int lane) {
    dev::fft_wave<E, false>(v, buf, tw, lane);
}

// forward real FFT of in[0..N) (dense, fine-grained device memory) into the
// spectrum sp[0..P] (cf, host memory); the spectrum also stays in `buf`+regs
// for the speculative inverse: xs[m] = X[lane + 64 m], xp0 = X[P] (lane 0)
template <int E, bool PRE>
__device__ __forceinline__ void call_rfft(const CallIn<PRE>& in, int64_t off, float* sp, cf* buf, const cf* tw,
                                          const cf* sth, int lane, cf (&xs)[E], cf& xpp) {
    constexpr int P = 64 * E;
    cf v[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const float2 x2 = in.at2(off + 2 * (lane + 64 * m));
        v[m].r = dev::sanit(x2.x);
        v[m].i = dev::sanit(x2.y);
    }
    rfft_core<E>(v, buf, tw, lane);
#pragma unroll
    for (int m = 0; m < E; ++m) buf[lane + 64 * m] = v[m];
    dev::wave_lds_fence();
    xpp = cf{0.0f, 0.0f};
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const int k = lane + 64 * m;
        const cf zk = v[m];
        const cf fpnk = dev::conj(buf[(P - k) & (P - 1)]);
        const cf f1 = dev::cadd(zk, fpnk);
        const cf f2 = dev::csub(zk, fpnk);
        const cf t = dev::cmul(f2, sth[k]);
        cf xk = {__builtin_fmaf(f1.r, 0.5f, t.r), __builtin_fmaf(f1.i, 0.5f, t.i)}, xp;
        if (k == 0) {
            dev::dc_split(zk, xk, xp);
            xpp = xp;
            *reinterpret_cast<float2*>(sp + 2 * P) = make_float2(xp.r, xp.i);
        }
        *reinterpret_cast<float2*>(sp + 2 * k) = make_float2(xk.r, xk.i);
        xs[m] = xk;
    }
    dev::wave_lds_fence();
}

// inverse real FFT: spectrum X (bins 0..P) given by get(k) -> out[0..N) (host memory)
template <int E, typename G>
__device__ __forceinline__ void call_irfft(G get, float* out, cf* buf, const cf* tw, const cf* st, float inv_n,
                                           int lane, float* lds_copy = nullptr) {
    constexpr int P = 64 * E;
    cf v[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const int k = lane + 64 * m;
        const cf xk = get(k);
        const cf xpk = get(P - k);
        const cf w = st[k];
        const cf fek = {xk.r + xpk.r, xk.i - xpk.i};
        const cf tmp = {xk.r - xpk.r, xk.i + xpk.i};
        v[m].r = __builtin_fmaf(tmp.r, w.r, __builtin_fmaf(tmp.i, w.i, fek.r));
        v[m].i = __builtin_fmaf(tmp.i, w.r, __builtin_fmaf(-tmp.r, w.i, fek.i));
        if (k == 0) v[m] = dev::dc_merge(xk, xpk);
    }
    dev::fft_wave<E, true>(v, buf, tw, lane);
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const int i0 = 2 * (lane + 64 * m);
        const float2 o = make_float2(dev::sanit(v[m].r * inv_n), dev::sanit(v[m].i * inv_n));
        *reinterpret_cast<float2*>(out + i0) = o;
        if (lds_copy) *reinterpret_cast<float2*>(lds_copy + i0) = o;
    }
}

template <int E, bool INV, bool PRE>
__device__ __forceinline__ void call_cfft(const CallIn<PRE>& in, int64_t off, float* out, cf* buf, const cf* tw,
                                          float inv_p, int lane) {
    cf v[E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const float2 x2 = in.at2(off + 2 * (lane + 64 * m));
        v[m] = {x2.x, x2.y};
    }
    dev::fft_wave<E, INV>(v, buf, tw, lane);
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const int i = lane + 64 * m;
        if constexpr (INV)
            *reinterpret_cast<float2*>(out + 2 * i) =
                make_float2(dev::sanit(v[m].r * inv_p), dev::sanit(v[m].i * inv_p));
        else
            *reinterpret_cast<float2*>(out + 2 * i) = make_float2(v[m].r, v[m].i);
    }
}

// any size: fft_any.h's fft with the pass plan read from LDS into scalar
// registers (the plan in global memory cost a scalar-cache miss per pass)
// WG: the whole workgroup runs each pass (thread t of kCallBlock, barriers
// between passes); else one wave (lane of 64, wave fences)
__device__ __forceinline__ void any_sync(bool wg) {
    if (wg)
        __syncthreads();
    else
        dev::wave_lds_fence();
}
template <bool INV, bool WG>
__device__ __forceinline__ const cf* any_fft(cf* x, cf* y, const dev::any::Plan* pl, const cf* tw, int lane) {
    const int n = __builtin_amdgcn_readfirstlane(pl->n_pass), p = __builtin_amdgcn_readfirstlane(pl->p);
    for (int i = 0; i < n; ++i) {
        dev::any::PassDesc d;
        d.r = __builtin_amdgcn_readfirstlane(pl->pass[i].r);
        d.ns = __builtin_amdgcn_readfirstlane(pl->pass[i].ns);
        d.off = __builtin_amdgcn_readfirstlane(pl->pass[i].off);
        d.woff = __builtin_amdgcn_readfirstlane(pl->pass[i].woff);
        d.rcp_ns = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, pl->pass[i].rcp_ns)));
        dev::any::pass<INV>(x, y, tw, p, d, lane, WG ? kCallBlock : 64);
        any_sync(WG);
        cf* t = x;
        x = y;
        y = t;
    }
    return x;
}

template <int E>
__global__ __launch_bounds__(kCallBlock) void k_call(const CallArgs a) {
    constexpr int P = CallLds<E>::P, TW = CallLds<E>::TW;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    cf* tw = reinterpret_cast<cf*>(smem);
    cf* st = tw + TW;
    cf* sth = st + P;
    cf* bufs = sth + P;
    cf* specs = bufs + kCallWaves * P;
    constexpr bool ANY = E < 0;
    float* pre = ANY ? reinterpret_cast<float*>(smem) : reinterpret_cast<float*>(specs + kCallWaves * CallLds<E>::SP);
    float* chainbuf = pre + kCallPre;  // the frame a chained forward kept for the push that follows
    CallReq* rq = reinterpret_cast<CallReq*>(chainbuf + 2 * CallLds<E>::CH);
    uint32_t* cmd = reinterpret_cast<uint32_t*>(rq + 1);
    // ANY: [plan][tw any_tw cf][st P cf][chain frame 2P f][per wave A, B (P cf), S (P + 1 cf)]
    dev::any::Plan* const aplan = reinterpret_cast<dev::any::Plan*>(reinterpret_cast<char*>(cmd) + 16);
    cf* const dyn = reinterpret_cast<cf*>(reinterpret_cast<char*>(aplan) + (ANY ? kAnyPlanBytes : 0));
    cf* const atw = dyn;
    cf* const ast = atw + (ANY ? a.any_tw : 0);
    float* const achain = reinterpret_cast<float*>(ast + (ANY ? a.any_p : 0));
    cf* const awaves = reinterpret_cast<cf*>(achain + (ANY ? (a.any_two ? 4 : 2) * a.any_p : 0));
    // the frame kept by chained request q (a forward's speculated inverse or an
    // inverse request's output): buffer q % 2 (any size: one buffer unless any_two)
    auto chain_buf = [&](uint64_t q) -> float* {
        return ANY ? achain + ((q & 1) && a.any_two ? 2 * a.any_p : 0) : chainbuf + ((q & 1) ? CallLds<E>::CH : 0);
    };

    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    cf* buf = bufs + wave * P;
    cf* spb = specs + wave * CallLds<E>::SP;  // this wave's last spectrum (speculation)
    CallCtl* ctl = a.ctl;
    const float* staged_tw = nullptr;  // tables now in LDS (uniform)

    uint64_t my = a.first;
    uint64_t t_last = wall_clock64();
    uint64_t chain_req[2] = {0, 0};  // the chained requests (1-based) whose frames this launch holds, by parity
    for (;;) {
        // ---- wait for request `my` (thread 0 polls device memory, the workgroup follows)
        if (t == 0) {
            uint32_t k = 0;
            for (;;) {
                if (ld_sys64(&ctl->seq) > my) {
                    k = 1;
                    break;
                }
                if (ld_sys64(&ctl->stop) != 0) break;
                if (wall_clock64() - t_last > a.idle_ticks) {
                    __hip_atomic_store(&ctl->stop, uint64_t(2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
            }
            cmd[0] = k;
        }
        __syncthreads();
        if (cmd[0] == 0) break;
        // the descriptor (16 lanes x 8 bytes) and the first 4 KB of the slot's input,
        // requested together
        const int slot = int(my % uint64_t(a.depth));
        const CallReq* src = a.reqs + slot;
        {
            const uint64_t* pin = reinterpret_cast<const uint64_t*>(a.in_arena + int64_t(slot) * a.in_cap);
            const uint64_t v0 = ld_sys64(pin + t), v1 = ld_sys64(pin + kCallBlock + t);
            if (t < int(sizeof(CallReq) / 8))
                reinterpret_cast<uint64_t*>(rq)[t] = ld_sys64(reinterpret_cast<const uint64_t*>(src) + t);
            reinterpret_cast<uint64_t*>(pre)[t] = v0;
            reinterpret_cast<uint64_t*>(pre)[kCallBlock + t] = v1;
        }
        __syncthreads();
#ifdef CRLOT_CALL_PHASES
        const uint64_t ph0 = wall_clock64();
#define CALL_PH(i) if (t == 0) a.hctl->ph[i] = wall_clock64() - ph0
#else
#define CALL_PH(i)
#endif
        // the descriptor into scalar registers: every branch on it is uniform
        CallReq r;
        {
            const uint32_t* s = reinterpret_cast<const uint32_t*>(rq);
            uint32_t* d = reinterpret_cast<uint32_t*>(&r);
#pragma unroll
            for (int i = 0; i < int(sizeof(CallReq) / 4); ++i) d[i] = __builtin_amdgcn_readfirstlane(s[i]);
        }
        if (r.flags & kCallAcquire)  // device-form calls ran on streams since the last request
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        auto run_pend = [&]() {
            if (!r.pend.flags) return;
            // deferred ring work: the push of the kept frame (the push's arithmetic on
            // the frame bits the host compared), then a served produce's clear
            float* ring = r.pend.ring;
            const int64_t R = r.pend.R;
            if constexpr (CallLds<E>::CH > 0 || ANY) {
                if (r.pend.flags & kPendCommit) {
                    const float* wobj = r.pend.win;
                    // the LDS copy only survives within the launch that kept it (the
                    // kernel may have idled out and been relaunched since); else the
                    // same bits from the forward's speculation slot in host memory
                    const bool lds = r.pend.src_index != 0 && chain_req[r.pend.src_index & 1] == r.pend.src_index;
                    const float* const chainp = chain_buf(r.pend.src_index);
                    const float* hsrc = a.out_arena + r.pend.src_off;
                    for (int64_t j = t; j < r.pend.len; j += kCallBlock) {
                        int64_t p = r.pend.start + j;
                        if (p >= R) p -= R;
                        const float s = lds ? chainp[j] : ld_sys32(hsrc + j);
                        ring[p] = wobj ? __builtin_fmaf(__builtin_fmaf(s, wobj[j], 0.0f), r.pend.gain, ring[p])
                                       : __builtin_fmaf(s, r.pend.gain, ring[p]);
                    }
                    __syncthreads();
                }
            }
            if (r.pend.flags & kPendClear) {
                for (int64_t q = t; q < r.pend.n; q += kCallBlock) {
                    int64_t p = r.pend.rp + q;
                    if (p >= R) p -= R;
                    ring[p] = 0.0f;
                }
            }
            __syncthreads();
        };
        // kCallPendLate: the ring work waits until this request's chained produce
        // block (which adds the committed frame itself) is published
        // (only where this request computes a chained produce block and then runs
        // late_ring_work: a single-frame chained inverse, or forward with its
        // speculation; a flag set anywhere else runs the work now and still
        // publishes ring_done, so no host wait can miss it)
        const bool late = (CallLds<E>::CH > 0 || (ANY && a.any_two)) && (r.flags & kCallPendLate) != 0 && (r.pend.flags & kPendCommit) != 0 &&
                          (r.flags & kCallChain) != 0 && r.batch == 1 &&
                          (r.op == kCallIrfft || (r.op == kCallRfft && (r.flags & kCallSpec) != 0));
        if (!late) {
            run_pend();
            if (r.flags & kCallPendLate) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                __syncthreads();
                if (t == 0) st_sys64(&a.hctl->ring_done, my + 1);
            }
        }
        // the late commit's frame added to a produce value at ring position p: the
        // commit's own arithmetic on the ring value before it (bit for bit what the
        // produce would read after the commit)
        // (pw: the commit's window value at p when the caller loaded it already)
        auto prev_add = [&](int64_t p, float v, const float* pw = nullptr) -> float {
            if (!late) return v;
            int64_t d = p - r.pend.start;
            if (d < 0) d += r.pend.R;
            if (d < r.pend.len) {
                const bool lds = r.pend.src_index != 0 && chain_req[r.pend.src_index & 1] == r.pend.src_index;
                const float s0 = lds ? chain_buf(r.pend.src_index)[d] : ld_sys32(a.out_arena + r.pend.src_off + d);
                v = r.pend.win ? __builtin_fmaf(__builtin_fmaf(s0, pw ? *pw : r.pend.win[d], 0.0f), r.pend.gain, v)
                               : __builtin_fmaf(s0, r.pend.gain, v);
            }
            return v;
        };
        auto late_ring_work = [&]() {
            if (!late) return;
            run_pend();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            __syncthreads();
            if (t == 0) st_sys64(&a.hctl->ring_done, my);
        };
        CALL_PH(4);  // deferred ring work done
        // a chained inverse's produce block reads the ring (after the deferred work
        // above), the divisors and the window values it multiplies (its own frame's,
        // a late commit's): loaded now, in flight during the transform
        constexpr int KI = 2;
        float irv[KI], idv[KI], iwv[KI], ipw[KI];
        if constexpr (CallLds<E>::CH > 0 || ANY) {
            if (r.op == kCallIrfft && (r.flags & kCallChain) != 0 && r.batch == 1) {
                const int64_t R = r.j[0], Nfp = 2 * int64_t(ANY ? a.any_p : P);
#pragma unroll
                for (int k = 0; k < KI; ++k) {
                    const int64_t q = t + int64_t(k) * kCallBlock;
                    irv[k] = idv[k] = iwv[k] = ipw[k] = 1.0f;
                    if (q < r.j[3]) {
                        int64_t p = r.j[2] + q;
                        if (p >= R) p -= R;
                        irv[k] = r.p2[p];
                        idv[k] = r.p3[p];
                        int64_t d = p - r.j[1];
                        if (d < 0) d += R;
                        if (d < Nfp && r.p4) iwv[k] = r.p4[d];
                        if (late && r.pend.win) {
                            int64_t d2 = p - r.pend.start;
                            if (d2 < 0) d2 += r.pend.R;
                            if (d2 < r.pend.len) ipw[k] = r.pend.win[d2];
                        }
                    }
                }
            }
        }
        const float* in = a.in_arena + r.in_off;  // r.in_off is the slot's start
        // the input floats this request reads: when they fit the prefetched 4 KB,
        // every read comes from LDS
        const int64_t Pr = ANY ? a.any_p : P;  // complex points of an FFT request
        const int64_t need = r.op == kCallOlaAdd ? r.i[2] * r.channels + (r.win_off >= 0 ? r.i[2] : 0)
                             : r.op == kCallRfft ? int64_t(r.batch) * 2 * Pr
                             : r.op == kCallIrfft ? int64_t(r.batch) * (2 * Pr + 2)
                             : (r.op == kCallCfft || r.op == kCallIcfft) ? int64_t(r.batch) * 2 * Pr
                             : (r.op == kCallAxpy || r.op == kCallNormalize) ? 2 * r.i[0]
                             : r.op == kCallAxpyWin ? 3 * r.i[0] : 0;
        const bool pre_all = need <= kCallPre;
        float* out = a.out_arena + r.out_off;
        bool spec = false;
        // body(cin) with the input reader of this request
        auto with_in = [&](auto body) {
            if (pre_all)
                body(CallIn<true>{in, pre});
            else
                body(CallIn<false>{in, pre});
        };

        if constexpr (E > 0) {
            if (r.op >= kCallRfft && r.op <= kCallIcfft && r.p0 != staged_tw) {
                // stage the plan's tables (k_rfft's load_tables)
                const cf* gtw = reinterpret_cast<const cf*>(r.p0);
                const cf* gst = reinterpret_cast<const cf*>(r.p1);
                for (int i = t; i < TW; i += kCallBlock) tw[i] = gtw[i];
                for (int i = t; i < P; i += kCallBlock) {
                    const cf w = gst[i];
                    st[i] = w;
                    sth[i] = cf{w.r * 0.5f, w.i * 0.5f};  // exact
                }
                staged_tw = r.p0;
                __syncthreads();
            }
            if (r.op == kCallRfft) {
                // speculation keeps each wave's spectrum in LDS: one transform per wave
                spec = CallLds<E>::SPEC && (r.flags & kCallSpec) != 0 && r.batch <= kCallWaves;
                with_in([&](const auto& cin) {
                for (int b = wave; b < r.batch; b += kCallWaves) {
                    cf xs[E > 0 ? E : 1];
                    cf xpp;
                    float* sp = out + int64_t(b) * (2 * P + 2);
                    call_rfft<E>(cin, int64_t(b) * 2 * P, sp, buf, tw, sth, lane, xs, xpp);
                    if (CallLds<E>::SPEC && spec) {
#pragma unroll
                        for (int m = 0; m < E; ++m) spb[lane + 64 * m] = xs[m];
                        if (lane == 0) spb[P] = xpp;
                    }
                }
                });
            } else if (r.op == kCallIrfft) {
                // a chained inverse (a single frame an OLA object will push) also
                // keeps its output in LDS for the produce block after the publish
                const bool ich = CallLds<E>::CH > 0 && (r.flags & kCallChain) != 0 && r.batch == 1;
                with_in([&](const auto& cin) {
                for (int b = wave; b < r.batch; b += kCallWaves) {
                    const int64_t x = int64_t(b) * (2 * P + 2);
                    call_irfft<E>([&](int k) {
                        const float2 v = cin.at2(x + 2 * k);
                        return cf{v.x, v.y};
                    }, out + int64_t(b) * 2 * P, buf, tw, st, r.f0, lane, ich ? chain_buf(my + 1) : nullptr);
                }
                });
            } else if (r.op == kCallCfft || r.op == kCallIcfft) {
                with_in([&](const auto& cin) {
                for (int b = wave; b < r.batch; b += kCallWaves) {
                    if (r.op == kCallCfft)
                        call_cfft<E, false>(cin, int64_t(b) * 2 * P, out + int64_t(b) * 2 * P, buf, tw, r.f0, lane);
                    else
                        call_cfft<E, true>(cin, int64_t(b) * 2 * P, out + int64_t(b) * 2 * P, buf, tw, r.f0, lane);
                }
                });
            }
        }
        if constexpr (ANY) {
            // any size: k_fft_any's arithmetic (Stockham passes of fft_any.h through the
            // wave's A / B buffers, rsplit / rmerge), one transform per wave, the
            // first any_waves waves; tables and the pass plan from global memory
            // (r.p0 twiddles, r.p1 super twiddles, r.p3 the plan: uniform loads)
            if (r.op >= kCallRfft && r.op <= kCallIcfft) {
                const int Pn = a.any_p, W = a.any_waves;
                if (r.p0 != staged_tw) {  // the server's plan and tables into LDS, once
                    const cf* g0 = reinterpret_cast<const cf*>(r.p0);
                    const cf* g1 = reinterpret_cast<const cf*>(r.p1);
                    const uint32_t* gp = reinterpret_cast<const uint32_t*>(r.p5);
                    for (int i = t; i < int(sizeof(dev::any::Plan) / 4); i += kCallBlock)
                        reinterpret_cast<uint32_t*>(aplan)[i] = gp[i];
                    for (int i = t; i < a.any_tw; i += kCallBlock) atw[i] = g0[i];
                    for (int i = t; i < Pn; i += kCallBlock) ast[i] = g1[i];
                    staged_tw = r.p0;
                    __syncthreads();
                }
                const cf* gtw = atw;
                const cf* gst = ast;
                // one transform (the per-call case): the whole workgroup runs each pass
                // between barriers; several: one wave each, the first any_waves waves
                const bool wg = r.batch == 1;
                const int tid = wg ? t : lane, nth = wg ? kCallBlock : 64;
                cf* A = awaves + size_t(wg ? 0 : wave) * (3 * Pn + 1);
                cf* B = A + Pn;
                cf* S = B + Pn;
                spec = r.op == kCallRfft && (r.flags & kCallSpec) != 0 && r.batch <= W;
                if (wg || wave < W) {
                    with_in([&](const auto& cin) {
                    for (int b = wg ? 0 : wave; b < r.batch; b += W) {
                        if (r.op == kCallRfft) {
                            const int64_t x = int64_t(b) * 2 * Pn;
                            for (int i = tid; i < Pn; i += nth) {
                                const float2 v = cin.at2(x + 2 * i);
                                A[i] = {dev::sanit(v.x), dev::sanit(v.y)};
                            }
                            any_sync(wg);
                            const cf* z = wg ? any_fft<false, true>(A, B, aplan, gtw, t)
                                             : any_fft<false, false>(A, B, aplan, gtw, lane);
                            float* sp = out + int64_t(b) * (2 * Pn + 2);
                            for (int k = tid; k < Pn; k += nth) {
                                cf xk, xp;
                                dev::any::rsplit(z, Pn, gst, k, xk, xp);
                                *reinterpret_cast<float2*>(sp + 2 * k) = make_float2(xk.r, xk.i);
                                if (spec) S[k] = xk;
                                if (k == 0) {
                                    *reinterpret_cast<float2*>(sp + 2 * Pn) = make_float2(xp.r, xp.i);
                                    if (spec) S[Pn] = xp;
                                }
                            }
                        } else if (r.op == kCallIrfft) {
                            const int64_t x = int64_t(b) * (2 * Pn + 2);
                            for (int k = tid; k < Pn; k += nth) {
                                const float2 u = cin.at2(x + 2 * k), w = cin.at2(x + 2 * (Pn - k));
                                A[k] = dev::any::rmerge(cf{u.x, u.y}, cf{w.x, w.y}, gst[k], k);
                            }
                            any_sync(wg);
                            const cf* z = wg ? any_fft<true, true>(A, B, aplan, gtw, t)
                                             : any_fft<true, false>(A, B, aplan, gtw, lane);
                            float* o = out + int64_t(b) * 2 * Pn;
                            const bool ich = wg && (r.flags & kCallChain) != 0;  // (kept for the chained produce)
                            for (int i = tid; i < Pn; i += nth) {
                                const float2 v = make_float2(dev::sanit(z[i].r * r.f0), dev::sanit(z[i].i * r.f0));
                                *reinterpret_cast<float2*>(o + 2 * i) = v;
                                if (ich) *reinterpret_cast<float2*>(chain_buf(my + 1) + 2 * i) = v;
                            }
                        } else {
                            const int64_t x = int64_t(b) * 2 * Pn;
                            for (int i = tid; i < Pn; i += nth) {
                                const float2 v = cin.at2(x + 2 * i);
                                A[i] = {v.x, v.y};
                            }
                            any_sync(wg);
                            const bool inv = r.op == kCallIcfft;
                            const cf* z = inv ? (wg ? any_fft<true, true>(A, B, aplan, gtw, t)
                                                    : any_fft<true, false>(A, B, aplan, gtw, lane))
                                              : (wg ? any_fft<false, true>(A, B, aplan, gtw, t)
                                                    : any_fft<false, false>(A, B, aplan, gtw, lane));
                            float* o = out + int64_t(b) * 2 * Pn;
                            for (int i = tid; i < Pn; i += nth)
                                *reinterpret_cast<float2*>(o + 2 * i) =
                                    inv ? make_float2(dev::sanit(z[i].r * r.f0), dev::sanit(z[i].i * r.f0))
                                        : make_float2(z[i].r, z[i].i);
                        }
                        any_sync(wg);  // A / B are rewritten by the next transform
                    }
                    });
                }
            }
        }
        if (r.op == kCallOlaAdd) {
            // add_frame_SoA / push_frame_AoS (ola.hip k_ola_add): element e = channel-major
            // for SoA frames, interleaved for AoS; window from the request (caller's) or
            // the object.  K elements per thread per pass, every load of a pass issued
            // before its first store.  With speculation, an element that lands in the
            // predicted produce block [srp, srp + sn) also writes its quotient to the
            // speculation slot (the sum it just formed / den), and the block's positions
            // the add does not touch are read afterwards.
            constexpr int K = 8;
            float* ring = r.p2;
            const float* den = r.p1;
            const int64_t R = r.i[0], start = r.i[1], len = r.i[2], C = r.channels;
            const bool aos = r.i[3] != 0;
            const int64_t woff = r.win_off >= 0 ? r.win_off - r.in_off : -1;  // the window slice, in the slot
            const float* wobj = r.p0;
            const bool win = woff >= 0 || wobj;
            spec = (r.flags & kCallSpec) != 0;
            const int64_t srp = r.i[4], sn = spec ? r.i[5] : 0;
            float* so = a.out_arena + r.spec_off;
            // channels outer, samples inner: no division per element; inactive lanes load
            // a clamped (valid) element and store nothing
            with_in([&](const auto& cin) {
            for (int64_t c = 0; c < C; ++c) {
                for (int64_t jb = 0; jb < len; jb += int64_t(kCallBlock) * K) {
                    float s[K], w[K], acc[K], dv[K];
                    int64_t at[K], sj[K];
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const int64_t jr = jb + int64_t(k) * kCallBlock + t;
                        const bool ok = jr < len;
                        const int64_t j = ok ? jr : len - 1;
                        int64_t p = start + j;
                        if (p >= R) p -= R;
                        at[k] = c * R + p;
                        int64_t q = p - srp;  // offset in the speculated block
                        if (q < 0) q += R;
                        sj[k] = (ok && q < sn) ? c * sn + q : -1;
                        s[k] = cin.at(aos ? j * C + c : c * len + j);
                        w[k] = woff >= 0 ? cin.at(woff + j) : wobj ? wobj[j] : 1.0f;
                        acc[k] = ring[at[k]];
                        dv[k] = den[p];
                        if (!ok) at[k] = -1;
                    }
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        if (at[k] < 0) continue;
                        const float v = win ? __builtin_fmaf(__builtin_fmaf(s[k], w[k], 0.0f), r.f0, acc[k])
                                            : __builtin_fmaf(s[k], r.f0, acc[k]);
#ifdef CRLOT_CALL_NT_RING
                        __builtin_nontemporal_store(v, ring + at[k]);
#else
                        ring[at[k]] = v;
#endif
                        if (sj[k] >= 0) so[sj[k]] = v / dv[k];
                    }
                }
            }
            });
            if (spec) {
                // block positions outside this add: the ring as it stands
                for (int64_t c = 0; c < C; ++c)
                    for (int64_t q = t; q < sn; q += kCallBlock) {
                        int64_t p = srp + q;
                        if (p >= R) p -= R;
                        int64_t d = p - start;  // inside [start, start + len) was written above
                        if (d < 0) d += R;
                        if (d < len) continue;
                        so[c * sn + q] = ring[c * R + p] / den[p];
                    }
            }
        } else if (r.op == kCallOlaProduce) {
            // produce -> normalize_and_clear (ola.hip k_ola_produce), or the clear
            // alone for a produce already served from the speculation slot
            float* ring = r.p2;
            const float* den = r.p1;
            const int64_t R = r.i[0], rp = r.i[1], len = r.i[2], C = r.channels;
            const bool clear_only = (r.flags & kCallClearOnly) != 0;
            for (int64_t c = 0; c < C; ++c)
                for (int64_t j = t; j < len; j += kCallBlock) {
                    int64_t p = rp + j;
                    if (p >= R) p -= R;
                    float* rr = ring + c * R + p;
                    if (!clear_only) out[c * len + j] = *rr / den[p];
                    *rr = 0.0f;
                }
        } else if (r.op == kCallAxpy || r.op == kCallAxpyWin) {
            // dsp::axpy / axpy_windowed (kernels.cc:18-28): in = dst | src [| win]
            constexpr int K = 8;
            const int64_t n = r.i[0];
            with_in([&](const auto& cin) {
            for (int64_t base = 0; base < n; base += int64_t(kCallBlock) * K) {
                float d[K], s[K], w[K];
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const int64_t j = base + int64_t(k) * kCallBlock + t;
                    const bool ok = j < n;
                    d[k] = ok ? cin.at(j) : 0.0f;
                    s[k] = ok ? cin.at(n + j) : 0.0f;
                    w[k] = ok && r.op == kCallAxpyWin ? cin.at(2 * n + j) : 0.0f;
                }
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const int64_t j = base + int64_t(k) * kCallBlock + t;
                    if (j >= n) continue;
                    const float x = r.op == kCallAxpyWin ? __builtin_fmaf(s[k], w[k], 0.0f) : s[k];
                    out[j] = __builtin_fmaf(x, r.f0, d[k]);
                }
            }
            });
        } else if (r.op == kCallNormalize) {
            // dsp::normalize_and_clear (kernels.cc:30-36): in = acc | norm; out = out | acc
            constexpr int K = 8;
            const int64_t n = r.i[0];
            with_in([&](const auto& cin) {
            for (int64_t base = 0; base < n; base += int64_t(kCallBlock) * K) {
                float ac[K], nv[K];
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const int64_t j = base + int64_t(k) * kCallBlock + t;
                    ac[k] = j < n ? cin.at(j) : 0.0f;
                    nv[k] = j < n ? cin.at(n + j) : 1.0f;
                }
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const int64_t j = base + int64_t(k) * kCallBlock + t;
                    if (j >= n) continue;
                    out[j] = ac[k] / ((nv[k] > r.f0) ? nv[k] : r.f0);
                    out[n + j] = 0.0f;
                }
            }
            });
        }

        // ---- publish: results visible system-wide, then done.  An add's only
        // reader is its speculated produce: it publishes once, with the speculation.
        CALL_PH(0);
        my += 1;
        // (A chained forward publishing its spectrum, inverse and produce block
        // behind one fence measured 12.2 us per e2e frame against 11.4 us with
        // three publishes: the host waits for the spectrum first.)
        const bool chained =
            (CallLds<E>::SPEC || ANY) && spec && r.op == kCallRfft && (r.flags & kCallChain) != 0 && r.batch == 1;
        const bool merged = spec && r.op == kCallOlaAdd;
        if (!merged) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            CALL_PH(1);
            __syncthreads();
            if (t == 0) st_sys64(&a.hctl->done, my);
        }
        // ---- a chained inverse (the caller edited the spectrum it pushes): the
        // produce(n) block at rp after pushing the frame just returned at start --
        // the forward chain's arithmetic below, on the frame kept in LDS -- into the
        // speculation slot after one frame's floats
        // (computing it before the publish, behind the output's fence, measured
        // inverse +1.4 us, produce -1.15 us per e2e mask frame: published after)
        const bool ichain = (CallLds<E>::CH > 0 || ANY) && r.op == kCallIrfft && (r.flags & kCallChain) != 0 &&
                            r.batch == 1;
        auto ichain_block = [&](uint64_t me) {
            chain_req[me & 1] = me;
            const float* const chainp = chain_buf(me);
            float* ring = r.p2;
            const float* den = r.p3;
            const float* wobj = r.p4;
            const int64_t R = r.j[0], start = r.j[1], rp = r.j[2], n = r.j[3], Nf = 2 * Pr;
            float* co = a.out_arena + r.spec_off + Nf;
            // (pre: the window values came with the preload, wv / pw)
            auto one = [&](int64_t q, float v, float dn, bool pre, const float& wv, const float& pw) {
                int64_t p = rp + q;
                if (p >= R) p -= R;
                v = prev_add(p, v, pre ? &pw : nullptr);  // (a late commit's frame first, as the ring would hold it)
                int64_t d = p - start;
                if (d < 0) d += R;
                if (d < Nf) {
                    const float s0 = chainp[d];
                    v = wobj ? __builtin_fmaf(__builtin_fmaf(s0, pre ? wv : wobj[d], 0.0f), r.f1, v)
                             : __builtin_fmaf(s0, r.f1, v);
                }
                co[q] = v / dn;
            };
#pragma unroll
            for (int k = 0; k < KI; ++k) {
                const int64_t q = t + int64_t(k) * kCallBlock;
                if (q < n) one(q, irv[k], idv[k], true, iwv[k], ipw[k]);
            }
            for (int64_t q = t + int64_t(KI) * kCallBlock; q < n; q += kCallBlock) {
                int64_t p = rp + q;
                if (p >= R) p -= R;
                one(q, ring[p], den[p], false, 0.0f, 0.0f);
            }
        };
        if constexpr (CallLds<E>::CH > 0 || ANY) {
            if (ichain) {
                ichain_block(my);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                __syncthreads();
                if (t == 0) st_sys64(&a.hctl->chain_done, my);
                late_ring_work();
            }
        }

        // ---- speculation after the publish (the host is already running)
        if (spec) {
            float* so = a.out_arena + r.spec_off;
            if ((CallLds<E>::SPEC || ANY) && r.op == kCallRfft) {
                // inverse of the spectrum just written (the same bits, from LDS; the
                // inverse call's code), kept in LDS too for a chained produce
                const bool chain = chained;
                const int64_t Nf = 2 * Pr;  // frame floats
                // the chained produce's ring and den values, loaded under the inverse
                constexpr int KC = 4;
                float rv[KC], dv[KC];
                if (chain) {
#pragma unroll
                    for (int k = 0; k < KC; ++k) {
                        const int64_t q = t + int64_t(k) * kCallBlock;
                        rv[k] = dv[k] = 1.0f;
                        if (q < r.j[3]) {
                            int64_t p = r.j[2] + q;
                            if (p >= r.j[0]) p -= r.j[0];
                            rv[k] = r.p2[p];
                            dv[k] = r.p3[p];
                        }
                    }
                }
                dev::wave_lds_fence();
                if constexpr (E > 0) {
                    for (int b = wave; b < r.batch; b += kCallWaves)
                        call_irfft<E>([&](int k) { return spb[k]; }, so + int64_t(b) * 2 * P, buf, tw, st, r.f0,
                                      lane, chain ? chain_buf(my) : nullptr);
                }
                if constexpr (ANY) {
                    const bool wg = r.batch == 1;  // as the forward: its S buffer
                    if (wg || wave < a.any_waves) {
                        const int Pn = a.any_p, tid = wg ? t : lane, nth = wg ? kCallBlock : 64;
                        cf* A = awaves + size_t(wg ? 0 : wave) * (3 * Pn + 1);
                        cf* B = A + Pn;
                        const cf* S = B + Pn;
                        for (int b = wg ? 0 : wave; b < r.batch; b += a.any_waves) {  // (batch <= any_waves)
                            any_sync(wg);  // the forward's S writes
                            for (int k = tid; k < Pn; k += nth) A[k] = dev::any::rmerge(S[k], S[Pn - k], ast[k], k);
                            any_sync(wg);
                            const cf* z = wg ? any_fft<true, true>(A, B, aplan, atw, t)
                                             : any_fft<true, false>(A, B, aplan, atw, lane);
                            float* o = so + int64_t(b) * 2 * Pn;
                            for (int i = tid; i < Pn; i += nth) {
                                const float2 v = make_float2(dev::sanit(z[i].r * r.f0), dev::sanit(z[i].i * r.f0));
                                *reinterpret_cast<float2*>(o + 2 * i) = v;
                                if (chain) *reinterpret_cast<float2*>(chain_buf(my) + 2 * i) = v;
                            }
                            any_sync(wg);
                        }
                    }
                }
                if (chain) {
                    chain_req[my & 1] = my;
                    const float* const chainp = chain_buf(my);
                    // publish the inverse first: the host's inverse call waits for it
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                    __syncthreads();
                    if (t == 0) st_sys64(&a.hctl->spec_done, my);
                    // the produce(n) block at rp after pushing that frame at start: the
                    // push's arithmetic (axpy_windowed / axpy) on the ring as it stands
                    __syncthreads();
                    float* ring = r.p2;
                    const float* den = r.p3;
                    const float* wobj = r.p4;
                    const int64_t R = r.j[0], start = r.j[1], rp = r.j[2], n = r.j[3];
                    float* co = so + Nf;
                    auto one = [&](int64_t q, float v, float dn) {
                        int64_t p = rp + q;
                        if (p >= R) p -= R;
                        v = prev_add(p, v);  // (a late commit's frame first, as the ring would hold it)
                        int64_t d = p - start;
                        if (d < 0) d += R;
                        if (d < Nf) {
                            const float s = chainp[d];
                            v = wobj ? __builtin_fmaf(__builtin_fmaf(s, wobj[d], 0.0f), r.f1, v)
                                     : __builtin_fmaf(s, r.f1, v);
                        }
                        co[q] = v / dn;
                    };
#pragma unroll
                    for (int k = 0; k < KC; ++k) {
                        const int64_t q = t + int64_t(k) * kCallBlock;
                        if (q < n) one(q, rv[k], dv[k]);
                    }
                    for (int64_t q = t + int64_t(KC) * kCallBlock; q < n; q += kCallBlock) {
                        int64_t p = rp + q;
                        if (p >= R) p -= R;
                        one(q, ring[p], den[p]);
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                    __syncthreads();
                    if (t == 0) st_sys64(&a.hctl->chain_done, my);
                    late_ring_work();
                }
            }
            CALL_PH(2);
            if (!chained) {  // (a chained forward published each part as it went)
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                CALL_PH(3);
                __syncthreads();
                if (t == 0) {
                    if (merged) st_sys64(&a.hctl->done, my);
                    st_sys64(&a.hctl->spec_done, my);
                }
            }
        }
        t_last = wall_clock64();
    }
}

}  // namespace

// any size: FFT waves whose A, B, S buffers fit beside the static part (0: none)
// (tables: the twiddles of build_any_twiddles and P super twiddles; the chained
// frames: 2P floats each, two where the second costs no FFT wave)
static int any_tw_len(int p) {  // float pairs of build_any_twiddles(p), built once per size
    static std::mutex mu;
    static std::map<int, int> len;
    std::lock_guard<std::mutex> lk(mu);
    auto it = len.find(p);
    if (it == len.end()) it = len.emplace(p, int(build_any_twiddles(p).size() / 2)).first;
    return it->second;
}
static size_t call_any_fixed(int p, bool two) {
    return CallLds<-1>::bytes + kAnyPlanBytes + sizeof(cf) * (size_t(any_tw_len(p)) + size_t(p)) +
           sizeof(float) * (two ? 4 : 2) * size_t(p);
}
static int any_waves_for(int p, bool two) {
    const size_t per = sizeof(cf) * (3 * size_t(p) + 1), fixed = call_any_fixed(p, two), cap = 160 * 1024;
    return fixed >= cap ? 0 : int(std::min<size_t>(kCallWaves, (cap - fixed) / per));
}
// a second chained frame (late commits, kCallPendLate) where it costs no FFT wave
bool call_any_two(int p) {
    if (p < 1 || p > 8192) return false;
    const int w = any_waves_for(p, false);
    return w > 0 && any_waves_for(p, true) == w;
}
int call_any_waves(int p) {
    if (p < 1 || p > 8192) return 0;
    return any_waves_for(p, false);
}

size_t call_lds_bytes(int e) {
    if (e < 0) {
        const int w = call_any_waves(-e);
        return w ? call_any_fixed(-e, call_any_two(-e)) + sizeof(cf) * (3 * size_t(-e) + 1) * size_t(w) : 0;
    }
    switch (e) {
        case 0: return CallLds<0>::bytes;
        case 2: return CallLds<2>::bytes;
        case 4: return CallLds<4>::bytes;
        case 8: return CallLds<8>::bytes;
        case 16: return CallLds<16>::bytes;
        case 32: return CallLds<32>::bytes;
        default: return 0;
    }
}

hipError_t launch_call(int e, const CallArgs& a, hipStream_t s) {
    const size_t lds = call_lds_bytes(e);
    if (!lds) return hipErrorInvalidValue;
    void (*k)(const CallArgs) = nullptr;
    CallArgs b = a;
    if (e < 0) {
        b.any_p = -e;
        b.any_waves = call_any_waves(-e);
        b.any_tw = any_tw_len(-e);
        b.any_two = call_any_two(-e) ? 1 : 0;
        k = k_call<-1>;
    }
    switch (e < 0 ? -1 : e) {
        case -1: break;
        case 0: k = k_call<0>; break;
        case 2: k = k_call<2>; break;
        case 4: k = k_call<4>; break;
        case 8: k = k_call<8>; break;
        case 16: k = k_call<16>; break;
        case 32: k = k_call<32>; break;
        default: return hipErrorInvalidValue;
    }
    if (lds > 65536) {
        hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
        if (err != hipSuccess) return err;
    }
    hipLaunchKernelGGL(k, dim3(1), dim3(kCallBlock), lds, s, b);
    return hipGetLastError();
}

}  // namespace crlot
