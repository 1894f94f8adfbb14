// pair32_bench: the K_pair transform core in isolation -- fft_pair.h's 64-lane
// layout (radix-16, lane-bit-4/5 permlane swap, 16x16 LDS transpose; twiddles
// in registers, 3 waves/SIMD as in K_pair) against fft_pair32.h's half-wave
// 32 x 32 layout (one 32x32 LDS transpose, no permlanes; twiddles from LDS or
// registers, 2 or 3 waves/SIMD).  Each wave runs `iters` round trips
// fwd -> *1/1024 -> inv on register-resident data; prints ns per 1024-point
// round trip over the whole GPU, the max round-trip error, and checks the
// half-wave forward against a double-precision DFT.
// Usage: pair32_bench [iters=200]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "experiments/fft_pair32.h"

using namespace crlot::dev;

constexpr int kWaves = 4;  // per workgroup

template <int MINW>
__global__ __launch_bounds__(256, MINW) void k_old(const pc* in, pc* out, const pc* t1g, const pc* t2g, int iters) {
    __shared__ pc t1[kPairT1];
    __shared__ pc t2[48];
    __shared__ pc bufs[kWaves * kPairXbuf];
    for (int i = threadIdx.x; i < kPairT1; i += 256) t1[i] = t1g[i];
    for (int i = threadIdx.x; i < 48; i += 256) t2[i] = t2g[i];
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    pc* buf = bufs + wave * kPairXbuf;
    const long gw = long(blockIdx.x) * kWaves + wave;
    PairTw tw;
    pair_tw_load(tw, t1, t2 + (lane & 15), lane);
    pc v[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = in[gw * 1024 + lane + 64 * m];
    const pc sc = {1.0f / 1024, 1.0f / 1024};
    for (int it = 0; it < iters; ++it) {
        pair_fft_fwd(v, buf, tw, tw, lane);
#pragma unroll
        for (int m = 0; m < 16; ++m) v[m] = v[m] * sc;
        pair_fft_inv(v, buf, tw, tw, lane);
    }
#pragma unroll
    for (int m = 0; m < 16; ++m) out[gw * 1024 + lane + 64 * m] = v[m];
}

template <int MINW, bool REGTW>
__global__ __launch_bounds__(256, MINW) void k_new(const pc* in, pc* out, const pc* tg, int iters, int fwd_only) {
    __shared__ pc t[kP32T];
    __shared__ pc bufs[kWaves * kP32Xbuf];
    for (int i = threadIdx.x; i < kP32T; i += 256) t[i] = tg[i];
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, l = lane & 31;
    pc* buf = bufs + wave * kP32Xbuf;
    const long gt = (long(blockIdx.x) * kWaves + wave) * 2 + h;  // this half's transform
    pc v[32];
#pragma unroll
    for (int m = 0; m < 32; ++m) v[m] = in[gt * 1024 + l + 32 * m];
    if (fwd_only) {
        pair32_fft_fwd(v, buf, t, lane);
#pragma unroll
        for (int r = 0; r < 32; ++r) out[gt * 1024 + pair32_bin(lane, r)] = v[r];
        return;
    }
    const pc sc = {1.0f / 1024, 1.0f / 1024};
    pc w[31];
    if constexpr (REGTW) {
#pragma unroll
        for (int k1 = 1; k1 < 32; ++k1) w[k1 - 1] = t[pair32_t_index(k1, l)];
    }
    for (int it = 0; it < iters; ++it) {
        if constexpr (REGTW) {
            constexpr int idx[31] = {1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16,
                                     17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31};
            pdft32<false>(v);
            pc_tw_run<false>(v, idx, [&](int i) { return w[i]; });
            transpose32(v, buf, lane);
            pdft32<false>(v);
#pragma unroll
            for (int m = 0; m < 32; ++m) v[m] = v[m] * sc;
            pdft32<true>(v);
            transpose32(v, buf, lane);
            pc_tw_run<true>(v, idx, [&](int i) { return w[i]; });
            pdft32<true>(v);
        } else {
            pair32_fft_fwd(v, buf, t, lane);
#pragma unroll
            for (int m = 0; m < 32; ++m) v[m] = v[m] * sc;
            pair32_fft_inv(v, buf, t, lane);
        }
    }
#pragma unroll
    for (int m = 0; m < 32; ++m) out[gt * 1024 + l + 32 * m] = v[m];
}

static pc W(double num, double den) {
    const double a = -2.0 * M_PI * num / den;
    return pc{float(std::cos(a)), float(std::sin(a))};
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 200;
    const int blocks = 256 * 6;
    const long transforms = long(blocks) * kWaves * 2;  // enough for the half-wave kernel
    std::vector<pc> hin(size_t(transforms) * 1024);
    srand(1);
    for (auto& z : hin) z = pc{float(rand()) / RAND_MAX - 0.5f, float(rand()) / RAND_MAX - 0.5f};
    std::vector<pc> t1(kPairT1), t2(48), t32(kP32T);
    for (int k1 = 1; k1 < 16; ++k1)
        for (int l = 0; l < 64; ++l) t1[size_t(pair_t1_index(k1, l))] = W(double(l * k1), 1024);
    for (int c = 1; c < 4; ++c)
        for (int x = 0; x < 16; ++x) t2[size_t(16 * (c - 1) + x)] = W(double(x * c), 64);
    for (int k1 = 1; k1 < 32; ++k1)
        for (int l = 0; l < 32; ++l) t32[size_t(pair32_t_index(k1, l))] = W(double(l * k1), 1024);
    pc *din, *dout, *dt1, *dt2, *dt32;
    hipMalloc(&din, hin.size() * sizeof(pc));
    hipMalloc(&dout, hin.size() * sizeof(pc));
    hipMalloc(&dt1, t1.size() * sizeof(pc));
    hipMalloc(&dt2, t2.size() * sizeof(pc));
    hipMalloc(&dt32, t32.size() * sizeof(pc));
    hipMemcpy(din, hin.data(), hin.size() * sizeof(pc), hipMemcpyHostToDevice);
    hipMemcpy(dt1, t1.data(), t1.size() * sizeof(pc), hipMemcpyHostToDevice);
    hipMemcpy(dt2, t2.data(), t2.size() * sizeof(pc), hipMemcpyHostToDevice);
    hipMemcpy(dt32, t32.data(), t32.size() * sizeof(pc), hipMemcpyHostToDevice);

    // forward check of the half-wave layout against a double DFT (first 4 transforms)
    k_new<2, false><<<1, 256>>>(din, dout, dt32, 0, 1);
    std::vector<pc> hout(hin.size());
    hipMemcpy(hout.data(), dout, 8 * 1024 * sizeof(pc), hipMemcpyDeviceToHost);
    double ferr = 0, fmax = 0;
    for (int tr = 0; tr < 4; ++tr)
        for (int k = 0; k < 1024; k += 7) {
            double re = 0, im = 0;
            for (int n = 0; n < 1024; ++n) {
                const double a = -2.0 * M_PI * double((long(n) * k) % 1024) / 1024.0;
                const pc z = hin[size_t(tr) * 1024 + size_t(n)];
                re += z.x * std::cos(a) - z.y * std::sin(a);
                im += z.x * std::sin(a) + z.y * std::cos(a);
            }
            const pc g = hout[size_t(tr) * 1024 + size_t(k)];
            ferr = std::fmax(ferr, std::hypot(g.x - re, g.y - im));
            fmax = std::fmax(fmax, std::hypot(re, im));
        }
    std::printf("{\"forward_check\": {\"max_abs_err\": %.3e, \"max_abs\": %.3e}}\n", ferr, fmax);

    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto run = [&](const char* name, auto launch, long per_launch) {
        launch();
        hipDeviceSynchronize();
        float best = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
            hipEventRecord(a);
            launch();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            best = std::fmin(best, ms);
        }
        hipMemcpy(hout.data(), dout, size_t(per_launch) * 1024 * sizeof(pc), hipMemcpyDeviceToHost);
        double err = 0;
        for (size_t i = 0; i < size_t(per_launch) * 1024; ++i)
            err = std::fmax(err, std::hypot(hout[i].x - hin[i].x, hout[i].y - hin[i].y));
        const double rt = double(per_launch) * iters;
        std::printf("{\"kernel\": \"%s\", \"ms\": %.4f, \"ns_per_roundtrip\": %.4f, \"roundtrips_per_s\": %.4e, "
                    "\"max_err_after_iters\": %.3e}\n",
                    name, best, best * 1e6 / rt, rt / (best * 1e-3), err);
    };
    const long old_tr = long(blocks) * kWaves;  // one transform per wave
    run("old64_regtw_3w", [&] { k_old<3><<<blocks, 256>>>(din, dout, dt1, dt2, iters); }, old_tr);
    run("old64_regtw_4w", [&] { k_old<4><<<blocks, 256>>>(din, dout, dt1, dt2, iters); }, old_tr);
    run("new32_ldstw_2w", [&] { k_new<2, false><<<blocks, 256>>>(din, dout, dt32, iters, 0); }, transforms);
    run("new32_ldstw_3w", [&] { k_new<3, false><<<blocks, 256>>>(din, dout, dt32, iters, 0); }, transforms);
    run("new32_regtw_2w", [&] { k_new<2, true><<<blocks, 256>>>(din, dout, dt32, iters, 0); }, transforms);
    return 0;
}
