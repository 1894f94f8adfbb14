// signal_rtt: host <-> resident-kernel signalling round trip on this box, the
// floor under the resident streaming path (stream_rt.hip).  One workgroup polls
// a doorbell and answers on an ack word; the host times doorbell -> ack.
//   mode 0: doorbell and ack in pinned coherent host memory
//   mode 1: doorbell in fine-grained device memory written by the host (BAR),
//           ack in pinned host memory
//   mode 2: as 0, plus a 4 KB payload read from host memory per round
// Every mode's kernel exits on `stop` or after 50 ms without a doorbell.
// Build: hipcc --offload-arch=gfx950 -O2 -o signal_rtt signal_rtt.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define HC(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(2);                                                         \
        }                                                                         \
    } while (0)

__global__ void k_echo(const uint64_t* bell, uint64_t* ack, const uint64_t* stop, const float4* payload,
                       float* sink, int mode) {
    uint64_t my = 0;
    uint64_t t_last = wall_clock64();
    __shared__ uint32_t cmd;
    for (;;) {
        if (threadIdx.x == 0) {
            uint32_t k = 0;
            for (;;) {
                const uint64_t b = __hip_atomic_load(bell, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
                if (b > my) {
                    k = 1;
                    break;
                }
                if (__hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
                if (wall_clock64() - t_last > 5000000) break;  // 50 ms
                __builtin_amdgcn_s_sleep(1);
            }
            cmd = k;
        }
        __syncthreads();
        if (!cmd) break;
        __syncthreads();
        my += 1;
        float acc = 0.f;
        if (mode == 2) {
            const float4 v = payload[threadIdx.x];
            acc = v.x + v.y + v.z + v.w;
            if (acc == 12345.f) sink[threadIdx.x] = acc;
            __syncthreads();
        }
        if (threadIdx.x == 0) __hip_atomic_store(ack, my, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        t_last = wall_clock64();
    }
}

int main() {
    HC(hipSetDeviceFlags(hipDeviceScheduleSpin));
    hipStream_t s;
    HC(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint64_t *h_bell, *h_ack, *h_stop, *d_bell;
    float4* h_pay;
    float* d_sink;
    const unsigned fl = hipHostMallocCoherent | hipHostMallocMapped;
    HC(hipHostMalloc((void**)&h_bell, 64, fl));
    HC(hipHostMalloc((void**)&h_ack, 64, fl));
    HC(hipHostMalloc((void**)&h_stop, 64, fl));
    HC(hipHostMalloc((void**)&h_pay, 256 * sizeof(float4), fl));
    HC(hipMalloc(&d_sink, 1024));
    const int rounds = 2000;
    for (int mode = 0; mode < 3; ++mode) {
        const uint64_t* bell_dev = h_bell;
        uint64_t* bell_host = h_bell;
        if (mode == 1) {
            if (hipExtMallocWithFlags((void**)&d_bell, 64, hipDeviceMallocFinegrained) != hipSuccess) {
                std::printf("mode 1: fine-grained device malloc unavailable\n");
                continue;
            }
            bell_dev = d_bell;
            bell_host = d_bell;  // host access through the BAR mapping
        }
        *bell_host = 0;
        *h_ack = 0;
        *h_stop = 0;
        std::atomic_thread_fence(std::memory_order_seq_cst);
        hipLaunchKernelGGL(k_echo, dim3(1), dim3(256), 0, s, bell_dev, h_ack, h_stop, h_pay, d_sink, mode);
        std::vector<double> us;
        bool ok = true;
        for (int r = 1; r <= rounds && ok; ++r) {
            auto t0 = std::chrono::steady_clock::now();
            __atomic_store_n(bell_host, uint64_t(r), __ATOMIC_RELEASE);
            while (__atomic_load_n(h_ack, __ATOMIC_ACQUIRE) < uint64_t(r)) {
                if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
                    ok = false;
                    break;
                }
            }
            us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        }
        __atomic_store_n(h_stop, uint64_t(1), __ATOMIC_RELEASE);
        HC(hipStreamSynchronize(s));
        std::sort(us.begin(), us.end());
        std::printf("mode %d: %s rtt p50 %.2f us p99 %.2f us\n", mode, ok ? "ok" : "TIMEOUT", us[us.size() / 2],
                    us[size_t(us.size() * 0.99)]);
        if (mode == 1) HC(hipFree(d_bell));
    }
    return 0;
}
