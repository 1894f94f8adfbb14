// Micro-benchmark: per-SIMD throughput cost (shader cycles per wave-instruction)
// of the VALU forms the frame-pair FFT uses, at 1..8 waves per SIMD, with 8
// independent chains per wave.  One workgroup per CU of 4*WPS waves (so WPS
// waves land on each SIMD); s_memtime (shader clock) brackets the loop.
// build: hipcc --offload-arch=gfx950 -O3 valu_cost.hip -o /tmp/valu_cost
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int KIND>
__global__ void k(float* out, long long* cyc, int iters) {
    float a[8];
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 0.001f + i;
    f2 b[8];
    for (int i = 0; i < 8; ++i) b[i] = (f2){a[i], a[7 - i]};
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if constexpr (KIND == 0) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
                if constexpr (KIND == 1) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(b[i]) : "v"(b[(i + 1) & 7]));
                if constexpr (KIND == 2)
                    asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(b[i]) : "v"(b[(i + 1) & 7]));
                if constexpr (KIND == 3) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(b[i]) : "v"(b[(i + 1) & 7]));
                if constexpr (KIND == 4) asm volatile("v_fma_f32 %0, %0, %1, %0" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
                if constexpr (KIND == 5)
                    if ((i & 1) == 0) asm volatile("v_permlane16_swap_b32 %0, %1" : "+v"(a[i]), "+v"(a[i + 1]));
                if constexpr (KIND == 6)
                    if ((i & 1) == 0) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a[i]), "+v"(a[i + 1]));
                if constexpr (KIND == 7) asm volatile("v_mov_b32 %0, %1" : "=v"(a[i]) : "v"(a[(i + 3) & 7]));
                if constexpr (KIND == 8)
                    asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
                if constexpr (KIND == 9)
                    asm volatile("v_add_f32_dpp %0, %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
                                 : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
                if constexpr (KIND == 10)
                    asm volatile("v_add_f32_dpp %0, %0, %1 row_ror:8 row_mask:0xf bank_mask:0xf"
                                 : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
                if constexpr (KIND == 11)
                    asm volatile("v_fmac_f32_dpp %0, %1, %2 row_ror:4 row_mask:0xf bank_mask:0xf"
                                 : "+v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(a[(i + 2) & 7]));
                if constexpr (KIND == 12)  // compare + select pair (sanitize threshold)
                    asm volatile("v_cmp_gt_f32 vcc, |%0|, %1\n\tv_cndmask_b32 %0, 0, %0, vcc"
                                 : "+v"(a[i]) : "v"(a[(i + 1) & 7]) : "vcc");
                if constexpr (KIND == 13)  // packed add with op_sel swap / neg modifiers
                    asm volatile("v_pk_add_f32 %0, %0, %1 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]"
                                 : "+v"(b[i]) : "v"(b[(i + 1) & 7]));
                if constexpr (KIND == 14)  // v_pk_mov_b32 (register pair shuffle)
                    asm volatile("v_pk_mov_b32 %0, %1, %0 op_sel:[1,0]" : "+v"(b[i]) : "v"(b[(i + 3) & 7]));
                if constexpr (KIND == 15)  // one packed + one scalar alternating
                    if (i & 1) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(b[i]) : "v"(b[(i + 1) & 7]));
                    else asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
                if constexpr (KIND == 16)  // v_mov_b32_dpp row_ror:8 (cross-half-row move)
                    asm volatile("v_mov_b32_dpp %0, %1 row_ror:8 row_mask:0xf bank_mask:0xf"
                                 : "=v"(a[i]) : "v"(a[(i + 3) & 7]));
                if constexpr (KIND == 17)  // v_max3 with abs (range checks)
                    asm volatile("v_max3_f32 %0, |%0|, |%1|, |%2|" : "+v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(a[(i + 2) & 7]));
            }
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int i = 0; i < 8; ++i) s += a[i] + b[i].x + b[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

static const char* names[] = {"v_add_f32",        "v_pk_add_f32",      "v_pk_fma_f32",     "v_pk_mul_f32",
                              "v_fma_f32",        "v_permlane16_swap", "v_permlane32_swap", "v_mov_b32",
                              "v_cndmask_b32",    "v_add_dpp_quad",    "v_add_dpp_ror8",    "v_fmac_dpp_ror4",
                              "cmp+cndmask(pair)", "v_pk_add_opsel",   "v_pk_mov_b32",      "pk_add/add alt",
                              "v_mov_dpp_ror8",   "v_max3_abs"};

template <int KIND>
void run(int wps) {
    const int cus = 256, threads = 256 * wps, iters = 2000;
    float* out;
    long long* cyc;
    hipMalloc(&out, sizeof(float) * cus * threads);
    hipMalloc(&cyc, sizeof(long long) * cus * threads / 64);
    hipLaunchKernelGGL(k<KIND>, dim3(cus), dim3(threads), 0, 0, out, cyc, 10);
    hipLaunchKernelGGL(k<KIND>, dim3(cus), dim3(threads), 0, 0, out, cyc, iters);
    hipDeviceSynchronize();
    std::vector<long long> h(cus * threads / 64);
    hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
    double mx = 0, sum = 0;
    for (auto v : h) {
        mx = v > mx ? v : mx;
        sum += v;
    }
    // instructions per wave: iters * 64 (permlanes: 32, each moves two registers)
    const double per_wave = double(iters) * 64 * ((KIND == 5 || KIND == 6) ? 0.5 : 1.0) * (KIND == 12 ? 2 : 1);
    // per-SIMD cost: wps waves share a SIMD -> cycles / (wps * per_wave)
    printf("%-20s wps=%d  cyc/instr/SIMD %.2f (mean wave %.2f)\n", names[KIND], wps, mx / (wps * per_wave),
           sum / h.size() / (wps * per_wave));
    hipFree(out);
    hipFree(cyc);
}

template <int K>
void all() {
    for (int w : {1, 2, 3, 4, 8}) run<K>(w);
}

int main() {
    all<0>(); all<1>(); all<2>(); all<3>(); all<4>(); all<5>(); all<6>(); all<7>(); all<8>();
    all<9>(); all<10>(); all<11>(); all<12>(); all<13>(); all<14>(); all<15>(); all<16>(); all<17>();
    return 0;
}
