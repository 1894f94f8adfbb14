// call_rtt: the floor under a synchronous host-pointer call served by a
// resident kernel (the drop-in per-call path: IFftPlan::forward on one 1024-
// point frame = 4 KB in, 4 KB out).  The host copies the payload in, rings a
// doorbell, the kernel (one 256-thread workgroup) reads the payload, writes a
// 4 KB result into pinned host memory, fences and acks; the host copies the
// result out.  Where the doorbell and the payload live:
//   mode 0: both in pinned coherent host memory (the kernel reads over PCIe)
//   mode 1: both in fine-grained device memory written by the host through the
//           BAR mapping (the kernel reads its own HBM, bypassing L2)
//   mode 2: doorbell in pinned host memory, payload in fine-grained device memory
//   mode 3: mode 1 with the payload copied in by the host as non-temporal 16-byte
//           stores (write-combined) followed by sfence
// Every mode's kernel exits on `stop` or after 50 ms without a doorbell.
// Build: hipcc --offload-arch=gfx950 -O2 -o call_rtt call_rtt.hip
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define HC(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(2);                                                         \
        }                                                                         \
    } while (0)

__device__ __forceinline__ uint64_t ld_sys64(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_call(const uint64_t* bell, uint64_t* ack, const uint64_t* stop, const uint64_t* payload,
                       float* result) {
    uint64_t my = 0;
    uint64_t t_last = wall_clock64();
    __shared__ uint32_t cmd;
    for (;;) {
        if (threadIdx.x == 0) {
            uint32_t k = 0;
            for (;;) {
                if (ld_sys64(bell) > my) {
                    k = 1;
                    break;
                }
                if (ld_sys64(stop)) break;
                if (wall_clock64() - t_last > 5000000) break;  // 50 ms
                __builtin_amdgcn_s_sleep(1);
            }
            cmd = k;
        }
        __syncthreads();
        if (!cmd) break;
        my += 1;
        // 4 KB payload: 256 threads x 2 x 8 bytes, system-scope loads
        const uint64_t a = ld_sys64(payload + threadIdx.x);
        const uint64_t b = ld_sys64(payload + 256 + threadIdx.x);
        const float x = __uint_as_float(uint32_t(a)) + __uint_as_float(uint32_t(a >> 32));
        const float y = __uint_as_float(uint32_t(b)) + __uint_as_float(uint32_t(b >> 32));
        float4* r = reinterpret_cast<float4*>(result);
        r[threadIdx.x] = make_float4(x, y, x * y, float(my));
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_store(ack, my, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        t_last = wall_clock64();
    }
}

static void copy_nt(void* dst, const void* src, size_t bytes) {
    auto* d = static_cast<__m128i*>(dst);
    auto* s = static_cast<const __m128i*>(src);
    for (size_t i = 0; i < bytes / 16; ++i) _mm_stream_si128(d + i, _mm_loadu_si128(s + i));
    _mm_sfence();
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 3000;
    HC(hipSetDeviceFlags(hipDeviceScheduleSpin));
    hipStream_t s;
    HC(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const unsigned fl = hipHostMallocCoherent | hipHostMallocMapped;
    uint64_t *h_bell, *h_ack, *h_stop, *h_pay;
    float* h_res;
    HC(hipHostMalloc((void**)&h_bell, 64, fl));
    HC(hipHostMalloc((void**)&h_ack, 64, fl));
    HC(hipHostMalloc((void**)&h_stop, 64, fl));
    HC(hipHostMalloc((void**)&h_pay, 4096, fl));
    HC(hipHostMalloc((void**)&h_res, 4096, fl));
    uint64_t *d_bell = nullptr, *d_pay = nullptr;
    const bool fg = hipExtMallocWithFlags((void**)&d_bell, 64, hipDeviceMallocFinegrained) == hipSuccess &&
                    hipExtMallocWithFlags((void**)&d_pay, 4096, hipDeviceMallocFinegrained) == hipSuccess;
    std::vector<float> src(1024), dst(1024);
    for (int i = 0; i < 1024; ++i) src[i] = float(i) * 0.5f;
    std::printf("{\"rounds\": %d, \"modes\": [", rounds);
    for (int mode = 0; mode < 4; ++mode) {
        if (mode > 0 && !fg) continue;
        uint64_t* bell = (mode == 1 || mode == 3) ? d_bell : h_bell;
        uint64_t* pay = mode == 0 ? h_pay : d_pay;
        *bell = 0;
        *h_ack = 0;
        *h_stop = 0;
        std::atomic_thread_fence(std::memory_order_seq_cst);
        hipLaunchKernelGGL(k_call, dim3(1), dim3(256), 0, s, bell, h_ack, h_stop, pay, h_res);
        std::vector<double> us;
        bool ok = true;
        for (int r = 1; r <= rounds && ok; ++r) {
            src[0] = float(r);
            auto t0 = std::chrono::steady_clock::now();
            if (mode == 3)
                copy_nt(pay, src.data(), 4096);
            else
                std::memcpy(pay, src.data(), 4096);
            __atomic_store_n(bell, uint64_t(r), __ATOMIC_RELEASE);
            while (__atomic_load_n(h_ack, __ATOMIC_ACQUIRE) < uint64_t(r)) {
                if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
                    ok = false;
                    break;
                }
            }
            std::memcpy(dst.data(), h_res, 4096);
            us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
            if (dst[3] != float(r)) ok = false;
        }
        __atomic_store_n(h_stop, uint64_t(1), __ATOMIC_RELEASE);
        HC(hipStreamSynchronize(s));
        std::sort(us.begin(), us.end());
        std::printf("%s{\"mode\": %d, \"ok\": %s, \"p50_us\": %.2f, \"p90_us\": %.2f, \"p99_us\": %.2f}",
                    mode ? ", " : "", mode, ok ? "true" : "false", us[us.size() / 2], us[size_t(us.size() * 0.9)],
                    us[size_t(us.size() * 0.99)]);
    }
    std::printf("]}\n");
    return 0;
}
