// Micro-benchmark: is a long straight-line loop body limited by instruction
// fetch on gfx950?  Same count of independent v_add_f32 per iteration, as
// (a) a 256-instruction body repeated, (b) a 4096-instruction body (16 KiB of
// 4-byte VOP2), (c) 4096 VOP3-encoded adds (8 bytes each, 32 KiB).
// 16 waves per CU (4 per SIMD); prints shader cycles per instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define ADD4(i) asm volatile("v_add_f32 %0, %0, %0\n v_add_f32 %1, %1, %1\n v_add_f32 %2, %2, %2\n v_add_f32 %3, %3, %3" \
                             : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]));
#define ADD4E(i) asm volatile("v_add_f32_e64 %0, %0, |%0|\n v_add_f32_e64 %1, %1, |%1|\n v_add_f32_e64 %2, %2, |%2|\n v_add_f32_e64 %3, %3, |%3|" \
                             : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]));

template <int KIND>
__global__ __launch_bounds__(1024) void k(float* out, long long* cyc, int iters) {
    float a[4];
    for (int i = 0; i < 4; ++i) a[i] = threadIdx.x * 1e-3f + i;
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    if (KIND == 0) {
        for (int it = 0; it < iters * 16; ++it) {
#pragma unroll
            for (int r = 0; r < 64; ++r) ADD4(r)
        }
    } else if (KIND == 1) {
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int r = 0; r < 1024; ++r) ADD4(r)
        }
    } else {
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int r = 0; r < 1024; ++r) ADD4E(r)
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 1024 + threadIdx.x] = a[0] + a[1] + a[2] + a[3];
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    float* out;
    long long* cyc;
    (void)hipMalloc(&out, 1 << 24);
    (void)hipMalloc(&cyc, 1 << 16);
    const int iters = 50;
    const char* names[] = {"256-instr body x16 (4 B each)", "4096-instr body (4 B each)", "4096-instr body (8 B VOP3)"};
    for (int kind = 0; kind < 3; ++kind) {
        auto fn = kind == 0 ? k<0> : kind == 1 ? k<1> : k<2>;
        for (int blocks : {256, 512}) {  // 1 or 2 workgroups of 16 waves per CU
            hipLaunchKernelGGL(fn, dim3(blocks), dim3(1024), 0, 0, out, cyc, 2);
            hipLaunchKernelGGL(fn, dim3(blocks), dim3(1024), 0, 0, out, cyc, iters);
            (void)hipDeviceSynchronize();
            std::vector<long long> h(blocks);
            (void)hipMemcpy(h.data(), cyc, sizeof(long long) * blocks, hipMemcpyDeviceToHost);
            double m = 0;
            for (auto v : h) m += double(v);
            m /= blocks;
            const double ninst = 4096.0 * iters;
            printf("%-32s waves/SIMD %d: %.3f cyc/instr/wave, %.3f cyc/instr/SIMD\n", names[kind], 4 * blocks / 256,
                   m / ninst, m / ninst / (4 * blocks / 256));
        }
    }
    return 0;
}
