// Micro-benchmark: cost of swapping a lane bit with a register bit on gfx950,
// v_permlane16_swap (one instruction per register pair, lane bit 4) against a
// quad-lane swap built from DPP (lane bit 0): new_a = bit0 ? b[l^1] : a,
// new_b = bit0 ? b : a[l^1], written as update_dpp + select.  16 waves per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int KIND>
__global__ __launch_bounds__(1024) void k(float* out, long long* cyc, int iters) {
    float a[8];
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 1e-3f + i;
    const bool b0 = threadIdx.x & 1;
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#pragma unroll
            for (int i = 0; i < 8; i += 2) {
                if (KIND == 0) {
                    const unsigned x = __builtin_bit_cast(unsigned, a[i]), y = __builtin_bit_cast(unsigned, a[i + 1]);
                    const auto s = __builtin_amdgcn_permlane16_swap(x, y, false, false);
                    const unsigned s0 = s[0], s1 = s[1];
                    a[i] = __builtin_bit_cast(float, s0);
                    a[i + 1] = __builtin_bit_cast(float, s1);
                } else {
                    const int x = __builtin_bit_cast(int, a[i]), y = __builtin_bit_cast(int, a[i + 1]);
                    const int px = __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
                    const int py = __builtin_amdgcn_update_dpp(0, y, 0xB1, 0xF, 0xF, false);
                    a[i] = __builtin_bit_cast(float, b0 ? py : x);
                    a[i + 1] = __builtin_bit_cast(float, b0 ? y : px);
                }
            }
            // some independent FP work between swaps, as in the FFT
#pragma unroll
            for (int i = 0; i < 8; ++i) a[i] = a[i] * 1.0001f + 0.5f;
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int i = 0; i < 8; ++i) s += a[i];
    out[blockIdx.x * 1024 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    float* out;
    long long* cyc;
    (void)hipMalloc(&out, 1 << 24);
    (void)hipMalloc(&cyc, 1 << 16);
    const int iters = 200;
    const char* names[] = {"permlane16_swap (4 per 8 regs)", "DPP quad swap (8 dpp + 8 select per 8 regs)"};
    for (int kind = 0; kind < 2; ++kind) {
        auto fn = kind == 0 ? k<0> : k<1>;
        hipLaunchKernelGGL(fn, dim3(256), dim3(1024), 0, 0, out, cyc, 4);
        hipLaunchKernelGGL(fn, dim3(256), dim3(1024), 0, 0, out, cyc, iters);
        (void)hipDeviceSynchronize();
        std::vector<long long> h(256);
        (void)hipMemcpy(h.data(), cyc, sizeof(long long) * 256, hipMemcpyDeviceToHost);
        double m = 0;
        for (auto v : h) m += double(v);
        m /= 256;
        printf("%-46s: %.1f cycles per swap group (+8 fma) per wave, 16 waves/CU\n", names[kind], m / (16.0 * iters));
    }
    return 0;
}
