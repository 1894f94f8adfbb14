// Micro-benchmark: issue cost on gfx950 of one wave64 VALU instruction of each
// kind the quad-lane radix-4 would use, 16 waves per CU (4 per SIMD), 16
// independent accumulators per wave: v_fmac_f32, v_fmac_f32_dpp (quad_perm
// operand), v_pk_fma_f32, v_permlane16_swap, v_permlane32_swap.  Cycles are
// s_memtime ticks per instruction per SIMD; the plain v_fmac_f32 row is the
// guide's 2-cycle reference (MI355X_MICROARCH.md, cycle constants).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int KIND>
__global__ __launch_bounds__(1024) void k(float* out, long long* cyc, int iters) {
    float a[16], s[4];
    for (int i = 0; i < 16; ++i) a[i] = threadIdx.x * 1e-3f + i;
    for (int i = 0; i < 4; ++i) s[i] = 1.0f - 1e-6f * (threadIdx.x + i);
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                if constexpr (KIND == 0) {
                    asm("v_fmac_f32_e32 %0, %1, %2" : "+v"(a[i]) : "v"(s[i & 3]), "v"(s[(i + 1) & 3]));
                } else if constexpr (KIND == 1) {
                    asm("v_fmac_f32_dpp %0, %1, %2 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf"
                        : "+v"(a[i]) : "v"(s[i & 3]), "v"(s[(i + 1) & 3]));
                } else if constexpr (KIND == 2) {
                    if (i % 2 == 0) {
                        typedef float f2 __attribute__((ext_vector_type(2)));
                        f2 x = {a[i], a[i + 1]};
                        const f2 p = {s[0], s[1]}, q = {s[2], s[3]};
                        asm("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(x) : "v"(p), "v"(q));
                        a[i] = x.x;
                        a[i + 1] = x.y;
                    }
                } else if constexpr (KIND == 3 || KIND == 4) {
                    if (i % 2 == 0) {
                        unsigned x = __builtin_bit_cast(unsigned, a[i]), y = __builtin_bit_cast(unsigned, a[i + 1]);
                        if constexpr (KIND == 3)
                            asm("v_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y));
                        else
                            asm("v_permlane32_swap_b32 %0, %1" : "+v"(x), "+v"(y));
                        a[i] = __builtin_bit_cast(float, x);
                        a[i + 1] = __builtin_bit_cast(float, y);
                    }
                }
            }
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    float acc = 0;
    for (int i = 0; i < 16; ++i) acc += a[i];
    out[blockIdx.x * 1024 + threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    float* out;
    long long* cyc;
    (void)hipMalloc(&out, 1 << 24);
    (void)hipMalloc(&cyc, 1 << 16);
    const int iters = 4000;
    const char* names[] = {"v_fmac_f32", "v_fmac_f32_dpp quad_perm", "v_pk_fma_f32", "v_permlane16_swap_b32",
                           "v_permlane32_swap_b32"};
    const int per_it[] = {128, 128, 64, 64, 64};  // instructions per wave per iteration
    void (*fns[])(float*, long long*, int) = {k<0>, k<1>, k<2>, k<3>, k<4>};
    for (int kind = 0; kind < 5; ++kind) {
        hipLaunchKernelGGL(fns[kind], dim3(256), dim3(1024), 0, 0, out, cyc, 4);
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(fns[kind], dim3(256), dim3(1024), 0, 0, out, cyc, iters);
        (void)hipEventRecord(e1, 0);
        (void)hipDeviceSynchronize();
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        std::vector<long long> h(256);
        (void)hipMemcpy(h.data(), cyc, sizeof(long long) * 256, hipMemcpyDeviceToHost);
        double m = 0;
        for (auto v : h) m += double(v);
        m /= 256;
        // 4 waves per SIMD issue per_it * iters instructions each
        // wall: ns per instruction per SIMD; at 2.4 GHz the cycles
        const double ns = ms * 1e6 / (4.0 * per_it[kind] * iters);
        printf("{\"instr\": \"%s\", \"ticks_per_instr_per_simd\": %.3f, \"ns_per_instr_per_simd\": %.4f, "
               "\"cycles_at_2p4GHz\": %.2f}\n",
               names[kind], m / (4.0 * per_it[kind] * iters), ns, ns * 2.4);
    }
    return 0;
}
