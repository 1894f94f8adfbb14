// Micro-benchmark: SIMD issue rate for mixed instruction streams on gfx950
// (16 waves per CU): pure VALU, VALU + SALU, VALU + s_nop, VALU + ds_read,
// dependent VALU chains.  Shader cycles per instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int KIND>
__global__ __launch_bounds__(1024) void k(float* out, long long* cyc, int iters) {
    __shared__ float lds[4096];
    for (int i = threadIdx.x; i < 4096; i += 1024) lds[i] = i;
    float a[4];
    for (int i = 0; i < 4; ++i) a[i] = threadIdx.x * 1e-3f + i;
    int s = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 64; ++r) {
            if (KIND == 0)  // 4 independent VALU
                asm volatile("v_add_f32 %0, %0, %0\n v_add_f32 %1, %1, %1\n v_add_f32 %2, %2, %2\n v_add_f32 %3, %3, %3"
                             : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]));
            else if (KIND == 1)  // 3 VALU + 1 SALU
                asm volatile("v_add_f32 %0, %0, %0\n s_add_u32 %3, %3, 1\n v_add_f32 %1, %1, %1\n v_add_f32 %2, %2, %2"
                             : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+s"(s));
            else if (KIND == 2)  // 3 VALU + s_nop 0
                asm volatile("v_add_f32 %0, %0, %0\n s_nop 0\n v_add_f32 %1, %1, %1\n v_add_f32 %2, %2, %2"
                             : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]));
            else if (KIND == 3)  // dependent chain of 4
                asm volatile("v_add_f32 %0, %0, %0\n v_add_f32 %0, %0, %0\n v_add_f32 %0, %0, %0\n v_add_f32 %0, %0, %0"
                             : "+v"(a[0]));
            else if (KIND == 4)  // 3 VALU + v_cmp to SGPR + cndmask (sanitize shape)
                asm volatile("v_cmp_ge_f32_e64 s[60:61], |%0|, 1.0\n v_add_f32 %1, %1, %1\n v_cndmask_b32_e64 %2, 0, %2, s[60:61]\n v_add_f32 %0, %0, %0"
                             : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]) : : "s60", "s61");
            else  // 3 VALU pk + 1 v_permlane16_swap
                asm volatile("v_add_f32 %0, %0, %0\n v_permlane16_swap_b32 %1, %2\n v_add_f32 %3, %3, %3\n v_add_f32 %0, %0, %0"
                             : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]));
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 1024 + threadIdx.x] = a[0] + a[1] + a[2] + a[3] + s + lds[threadIdx.x];
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    float* out;
    long long* cyc;
    (void)hipMalloc(&out, 1 << 24);
    (void)hipMalloc(&cyc, 1 << 16);
    const int iters = 400;
    const char* names[] = {"4 VALU", "3 VALU + 1 SALU", "3 VALU + s_nop 0", "4 dependent VALU",
                           "v_cmp(sgpr)+cndmask+2 VALU", "3 VALU + 1 permlane16_swap"};
    for (int kind = 0; kind < 6; ++kind) {
        auto fn = kind == 0 ? k<0> : kind == 1 ? k<1> : kind == 2 ? k<2> : kind == 3 ? k<3> : kind == 4 ? k<4> : k<5>;
        for (int threads : {256, 1024}) {
            hipLaunchKernelGGL(fn, dim3(256), dim3(threads), 0, 0, out, cyc, 4);
            hipLaunchKernelGGL(fn, dim3(256), dim3(threads), 0, 0, out, cyc, iters);
            (void)hipDeviceSynchronize();
            std::vector<long long> h(256);
            (void)hipMemcpy(h.data(), cyc, sizeof(long long) * 256, hipMemcpyDeviceToHost);
            double m = 0;
            for (auto v : h) m += double(v);
            m /= 256;
            const int wps = threads / 256;
            const double ninst = 4.0 * 64 * iters;
            printf("%-30s waves/SIMD %d: %.2f cyc/instr/wave  %.2f cyc/instr/SIMD\n", names[kind], wps, m / ninst, m / ninst / wps);
        }
    }
    return 0;
}
