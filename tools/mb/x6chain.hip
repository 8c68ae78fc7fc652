// Microbenchmark: the x6 transposed chain (tgemm_x6 / tchain_x6) in isolation — 4 layers of
// 160→160 per column tile, relu between layers, weight images streamed from L2 (the encoder
// kernels' structure), vs variants. Build: hipcc -O3 --offload-arch=gfx950 -I../../spwgnn_amd/csrc
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "gemm_blocks.h"
using namespace spw;

// MODE 0: images from global (L2); 1: one image in LDS (all layers share it, 256 threads/WG)
template <int NC, int D, int MODE, int OCC>
__global__ __launch_bounds__(256, OCC) void k_x6chain(const uint4* img, float* out, int nblk) {
    __shared__ uint4 wl[MODE == 1 ? 50 * 3 * 64 : 1];
    if (MODE == 1) {
        for (int i = threadIdx.x; i < 50 * 3 * 64; i += 256) wl[i] = img[i];
        __syncthreads();
    }
    const int lane = threadIdx.x & 63;
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w * NC >= nblk) return;
    f32x16 X[NC][5], Y[NC][5];
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int t = 0; t < 5; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) X[c][t][r] = 0.001f * (lane + r + t + c + w);
    const uint4* src = MODE == 1 ? wl : img;
#pragma unroll 1
    for (int layer = 0; layer < 4; ++layer) {
#pragma unroll
        for (int c = 0; c < NC; ++c) zero_tiles(Y[c]);
        tchain_x6<5, 10, 5, NC, D>(X, Y, src + (MODE == 1 ? 0 : layer * 50 * 3 * 64), lane);
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int t = 0; t < 5; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) X[c][t][r] = relu(Y[c][t][r]);
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int t = 0; t < 5; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) s += X[c][t][r];
    out[(int64_t)w * 64 + lane] = s;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main() {
    const int nblk = 65536;   // 32-column blocks (2.1M rows)
    std::vector<uint4> himg(4 * 50 * 3 * 64);
    for (size_t i = 0; i < himg.size(); ++i) himg[i] = make_uint4(0x3c003c00u + (i & 7), 0x3c003c00u, 0x3c00bc00u, 0x3c003c00u);
    uint4* dimg;
    float* dout;
    CK(hipMalloc(&dimg, himg.size() * 16));
    CK(hipMalloc(&dout, (size_t)nblk * 64 * 4));
    CK(hipMemcpy(dimg, himg.data(), himg.size() * 16, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double mfma_ideal_ms = (double)nblk * 4 * 300 * 32 / (1024.0 * 2.4e9) * 1e3;
    auto run = [&](const char* name, auto kern, int nc) -> int {
        const int waves = (nblk + nc - 1) / nc;
        const dim3 g((waves + 3) / 4);
        hipLaunchKernelGGL(kern, g, dim3(256), 0, 0, dimg, dout, nblk);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(kern, g, dim3(256), 0, 0, dimg, dout, nblk);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= 5;
        printf("%-34s %.3f ms  (MFMA-ideal %.3f ms, %.0f%%)\n", name, ms, mfma_ideal_ms, 100.0 * mfma_ideal_ms / ms);
        return 0;
    };
    run("NC2 D3 L2 occ1", k_x6chain<2, 3, 0, 1>, 2);
    run("NC2 D6 L2 occ1", k_x6chain<2, 6, 0, 1>, 2);
    run("NC1 D3 L2 occ2", k_x6chain<1, 3, 0, 2>, 1);
    run("NC1 D4 L2 occ2", k_x6chain<1, 4, 0, 2>, 1);
    run("NC2 D3 LDS occ1", k_x6chain<2, 3, 1, 1>, 2);
    run("NC1 D3 LDS occ2", k_x6chain<1, 3, 1, 2>, 1);
    return 0;
}
