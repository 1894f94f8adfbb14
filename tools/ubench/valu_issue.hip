// Micro-benchmark: issue cost of v_add_f32 vs v_pk_add_f32 vs v_permlane16_swap on
// gfx950 at 1..8 waves per SIMD (independent chains).  Prints cycles per
// instruction per SIMD from s_memtime (shader clock).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int KIND>
__global__ void k(float* out, long long* cyc, int iters) {
    float a[8];
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 0.001f + i;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 b[4];
    for (int i = 0; i < 4; ++i) b[i] = (f2){a[2 * i], a[2 * i + 1]};
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (KIND == 0) {
#pragma unroll
                for (int i = 0; i < 8; ++i) asm volatile("v_add_f32 %0, %0, %0" : "+v"(a[i]));
            } else if (KIND == 1) {
#pragma unroll
                for (int i = 0; i < 4; ++i) asm volatile("v_pk_add_f32 %0, %0, %0" : "+v"(b[i]));
            } else if (KIND == 2) {
#pragma unroll
                for (int i = 0; i < 4; ++i) asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(b[i]));
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    unsigned x = __builtin_bit_cast(unsigned, a[2 * i]), y = __builtin_bit_cast(unsigned, a[2 * i + 1]);
                    auto r2 = __builtin_amdgcn_permlane16_swap(x, y, false, false);
                    unsigned r0 = r2[0], r1 = r2[1];
                    a[2 * i] = __builtin_bit_cast(float, r0);
                    a[2 * i + 1] = __builtin_bit_cast(float, r1);
                }
            }
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int i = 0; i < 8; ++i) s += a[i];
    for (int i = 0; i < 4; ++i) s += b[i].x + b[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    float* out;
    long long* cyc;
    hipMalloc(&out, 1 << 24);
    hipMalloc(&cyc, 1 << 16);
    const int iters = 2000;
    const char* names[] = {"v_add_f32 x8 chains", "v_pk_add_f32 x4 chains", "v_pk_fma_f32 x4 chains", "v_permlane16_swap x4 pairs"};
    for (int kind = 0; kind < 4; ++kind)
        for (int wps : {1, 2, 3, 4, 8}) {  // waves per SIMD: one workgroup of 4*wps waves per CU
            const int threads = 256 * wps > 1024 ? 1024 : 256 * wps;
            const int blocks = 256 * (256 * wps / threads);
            auto fn = kind == 0 ? k<0> : kind == 1 ? k<1> : kind == 2 ? k<2> : k<3>;
            hipLaunchKernelGGL(fn, dim3(blocks), dim3(threads), 0, 0, out, cyc, 10);
            hipLaunchKernelGGL(fn, dim3(blocks), dim3(threads), 0, 0, out, cyc, iters);
            hipDeviceSynchronize();
            std::vector<long long> h(blocks);
            hipMemcpy(h.data(), cyc, sizeof(long long) * blocks, hipMemcpyDeviceToHost);
            double m = 0;
            for (auto v : h) m += double(v);
            m /= blocks;
            const int ninst = (kind == 0 ? 8 : 4) * 16 * iters;
            // per wave: cycles per instruction; per SIMD: / waves per SIMD
            printf("%-28s waves/SIMD %d : %.2f cyc/instr/wave, %.2f cyc/instr/SIMD\n", names[kind], wps,
                   m / ninst, m / ninst / wps);
        }
    return 0;
}
