// Microbenchmark: MFMA rate of the transposed-orientation layer chain (tchain_acc) under
// different weight-fragment sources. Build: hipcc -O3 --offload-arch=gfx950 -I../../spwgnn_amd/csrc
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "gemm_blocks.h"
using namespace spw;

// MODE 0: W fragments from global (tchain_acc, PF ring); 1: W held in registers (no loads);
// MODE 2: W from LDS (ds_read per k-step)
template <int MODE, int PF>
__global__ __launch_bounds__(256, 2) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_chain(const float* W, float* out, int iters) {
    __shared__ __attribute__((aligned(16))) float wl[(MODE == 2 || MODE == 4) ? 128 * 132 : 4];
    const int lane = threadIdx.x & 63;
    if (MODE == 4) {   // [col][k] image, ld 132
        for (int idx = threadIdx.x; idx < 128 * 128; idx += 256) {
            const int k = idx / 128, col = idx - k * 128;
            wl[col * 132 + k] = W[idx];
        }
        __syncthreads();
    }
    if (MODE == 2) {
        for (int i = threadIdx.x; i < 128 * 128; i += 256) wl[i] = W[i];
        __syncthreads();
    }
    f32x16 X[4], Y[4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) X[t][r] = 0.001f * (lane + r + t);
    float wr[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) wr[t] = W[lane + 32 * t];
    for (int it = 0; it < iters; ++it) {
        zero_tiles(Y);
        if (MODE == 0) {
            tchain_acc<4, 4, 4, 128, PF>(X, Y, W, lane);
        } else if (MODE == 1) {
#pragma unroll
            for (int k = 0; k < 52; ++k)
#pragma unroll
                for (int t = 0; t < 4; ++t) Y[t] = mfma32(wr[t], X[k >> 4][k & 15], Y[t]);
        } else if (MODE == 3 || MODE == 4) {   // [col][k] image: 4 consecutive k per dwordx4 / b128
            const int i = lane & 31, h = lane >> 5;
            const float* wb = (MODE == 3 ? W : wl) + i * (MODE == 3 ? 128 : 132) + 4 * h;
            const int ldc = MODE == 3 ? 128 : 132;
#pragma unroll
            for (int tp = 0; tp < 4; ++tp)
#pragma unroll
                for (int g = 0; g < (tp == 3 ? 1 : 4); ++g) {
                    float4 w4[4];
#pragma unroll
                    for (int t = 0; t < 4; ++t) w4[t] = *reinterpret_cast<const float4*>(wb + 32 * t * ldc + 32 * tp + 8 * g);
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        Y[t] = mfma32(w4[t].x, X[tp][4 * g + 0], Y[t]);
                        Y[t] = mfma32(w4[t].y, X[tp][4 * g + 1], Y[t]);
                        Y[t] = mfma32(w4[t].z, X[tp][4 * g + 2], Y[t]);
                        Y[t] = mfma32(w4[t].w, X[tp][4 * g + 3], Y[t]);
                    }
                }
        } else {
            const int i = lane & 31, h = lane >> 5;
            const float* wb = wl + (4 * h) * 128 + i;
#pragma unroll
            for (int k = 0; k < 52; ++k) {
                const float* wrow = wb + (rho(k & 15, 0) + 32 * (k >> 4)) * 128;
#pragma unroll
                for (int t = 0; t < 4; ++t) Y[t] = mfma32(wrow[32 * t], X[k >> 4][k & 15], Y[t]);
            }
        }
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) X[t][r] = relu(Y[t][r] * 0.5f + 0.01f);
    }
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) s += X[t][r];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MODE, int PF>
void run(const char* name, const float* W, float* out, int blocks, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL((k_chain<MODE, PF>), dim3(blocks), dim3(256), 0, 0, W, out, iters);
    hipEventRecord(a);
    hipLaunchKernelGGL((k_chain<MODE, PF>), dim3(blocks), dim3(256), 0, 0, W, out, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double mfma = (double)blocks * 4 * iters * 52 * 4;
    const double tf = mfma * 4096 / (ms * 1e-3) / 1e12;
    printf("%-28s %8.3f ms  %7.1f TF/s  (%.0f%% of 157.3)\n", name, ms, tf, 100 * tf / 157.3);
}

int main() {
    float *W, *out;
    (void)hipMalloc(&W, 128 * 128 * 4);
    (void)hipMalloc(&out, 4096 * 256 * 4);
    std::vector<float> h(128 * 128);
    for (int i = 0; i < 128 * 128; ++i) h[i] = ((i * 7919) % 1000) * 1e-4f - 0.05f;
    (void)hipMemcpy(W, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    const int iters = 200;
    for (int blocks : {512, 2048}) {
        printf("blocks=%d (waves %d)\n", blocks, blocks * 4);
        run<0, 3>("global W, PF=3", W, out, blocks, iters);
        run<0, 6>("global W, PF=6", W, out, blocks, iters);
        run<0, 1>("global W, PF=1", W, out, blocks, iters);
        run<1, 0>("W in registers", W, out, blocks, iters);
        run<2, 0>("W from LDS", W, out, blocks, iters);
        run<3, 0>("global [col][k] dwordx4", W, out, blocks, iters);
        run<4, 0>("LDS [col][k] b128", W, out, blocks, iters);
    }
    return 0;
}
