// Microbenchmark: does the order of the six split-bf16 products matter? The edge kernels issue, per
// k-block, 5 output tiles × mfma32_x6 (6 products chained on ONE accumulator). ORDER 0 is that;
// ORDER 1 issues product p for all 5 tiles before product p+1 (consecutive MFMAs independent).
// Operands live in registers (no memory): the pure matrix-pipe rate of each order at 1 or 2 waves
// per SIMD. Build: hipcc -O3 --offload-arch=gfx950 -I../../spwgnn_amd/csrc x6dep.hip -o x6dep
#include <hip/hip_runtime.h>
#include <cstdio>
#include "device_common.h"
using namespace spw;

template <int ORDER>
__device__ __forceinline__ void kblock(f32x16 (&acc)[5], const bf16x8 (&a)[3], const bf16x8 (&b)[5][3]) {
    if constexpr (ORDER == 0) {
#pragma unroll
        for (int T = 0; T < 5; ++T) acc[T] = mfma32_x6<3>(a, b[T], acc[T]);
    } else {
        constexpr int pa[6] = {2, 0, 1, 1, 0, 0}, pb[6] = {0, 2, 1, 0, 1, 0};
#pragma unroll
        for (int p = 0; p < 6; ++p)
#pragma unroll
            for (int T = 0; T < 5; ++T)
                acc[T] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[pa[p]], b[T][pb[p]], acc[T], 0, 0, 0);
    }
}

// VAR bit 0: a sched_barrier after every k-block (as the edge kernels); bit 1: W2 fragments read
// from an LDS image per (k-block, tile) right before use (as the edge kernels); bit 2: a VALU
// split of a loaded register pair per k-block (4 split2 = 44 VALU, as the G3 side); bit 3: the split's
// inputs are two float4 loaded from global memory two k-blocks ahead (a 2-slot ring, L2-resident rows,
// as the G3 gathers); bit 4: a per-block epilogue (80-register mask + add into a second accumulator
// set, as the dh1pre masking)
template <int ORDER, int WPS, int VAR = 0>
__global__ __launch_bounds__(256 * WPS, 1) void k_dep(float* out, int iters, uint32_t seed, const float4* g3) {
    __shared__ uint4 wl[(VAR & 2) ? 50 * 3 * 64 : 1];
    if (VAR & 2) {
        for (int i = threadIdx.x; i < 50 * 3 * 64; i += blockDim.x) wl[i] = make_uint4(i, seed, i ^ seed, 7u);
        __syncthreads();
    }
    const int lane = threadIdx.x & 63;
    const uint4* wlp = wl + lane;
    bf16x8 a[3], b[5][3];
#pragma unroll
    for (int p = 0; p < 3; ++p) {
        a[p] = as_bf16x8(make_uint4(seed + lane + p, seed ^ lane, 3u * p + 1u, lane * 7u));
#pragma unroll
        for (int T = 0; T < 5; ++T) b[T][p] = as_bf16x8(make_uint4(seed + T + p, lane + 11u * T, p, seed ^ (lane + T)));
    }
    f32x16 acc[5];
#pragma unroll
    for (int T = 0; T < 5; ++T) acc[T] = zero16();
    float xv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) xv[e] = 0.01f * (lane + e);
    // rows of 32 "nodes" × 1 KiB, lane-gathered like G3[receiver] (node = lane & 7 of the block)
    const float4* gp = g3 + ((blockIdx.x * 8 + (lane & 7)) * 64) + (lane >> 5) * 32;
    float4 ring[2][2];
    if (VAR & 8) {
#pragma unroll
        for (int k = 0; k < 2; ++k) { ring[k][0] = gp[2 * k]; ring[k][1] = gp[2 * k + 1]; }
    }
    f32x16 nacc[5];
#pragma unroll
    for (int T = 0; T < 5; ++T) nacc[T] = zero16();
    uint32_t mw = seed ^ lane;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int kb = 0; kb < 10; ++kb) {
            if (VAR & 8) {
                const float4 g0 = ring[kb & 1][0], g1 = ring[kb & 1][1];
                xv[0] = g0.x; xv[1] = g0.y; xv[2] = g0.z; xv[3] = g0.w;
                xv[4] = g1.x; xv[5] = g1.y; xv[6] = g1.z; xv[7] = g1.w;
                const int kn = (kb + 2) % 10;
                ring[kb & 1][0] = gp[2 * kn + 64 * (it & 7)];
                ring[kb & 1][1] = gp[2 * kn + 1 + 64 * (it & 7)];
            }
            if (VAR & 4) {
                uint32_t hw[4], mw[4], lw[4];
#pragma unroll
                for (int m = 0; m < 4; ++m) split2(xv[2 * m] + kb, xv[2 * m + 1], hw[m], mw[m], lw[m]);
                a[0] = as_bf16x8(make_uint4(hw[0], hw[1], hw[2], hw[3]));
                a[1] = as_bf16x8(make_uint4(mw[0], mw[1], mw[2], mw[3]));
                a[2] = as_bf16x8(make_uint4(lw[0], lw[1], lw[2], lw[3]));
            }
            if ((VAR & 2) && ORDER == 2) {   // tiles in groups {0,1}, {2,3,4}: products interleaved in a group
                constexpr int pa[6] = {2, 0, 1, 1, 0, 0}, pb[6] = {0, 2, 1, 0, 1, 0};
#pragma unroll
                for (int g = 0; g < 2; ++g) {
                    const int T0 = g == 0 ? 0 : 2, NT = g == 0 ? 2 : 3;
                    bf16x8 bp[3][3];
#pragma unroll
                    for (int u = 0; u < NT; ++u) {
                        const uint4* wp = wlp + (kb * 5 + T0 + u) * 3 * 64;
                        bp[u][0] = as_bf16x8(wp[0]);
                        bp[u][1] = as_bf16x8(wp[64]);
                        bp[u][2] = as_bf16x8(wp[128]);
                    }
#pragma unroll
                    for (int p = 0; p < 6; ++p)
#pragma unroll
                        for (int u = 0; u < NT; ++u)
                            acc[T0 + u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[pa[p]], bp[u][pb[p]], acc[T0 + u], 0, 0, 0);
                }
            } else if (VAR & 2) {
#pragma unroll
                for (int T = 0; T < 5; ++T) {
                    const uint4* wp = wlp + (kb * 5 + T) * 3 * 64;
                    bf16x8 bp[3];
                    bp[0] = as_bf16x8(wp[0]);
                    bp[1] = as_bf16x8(wp[64]);
                    bp[2] = as_bf16x8(wp[128]);
                    acc[T] = mfma32_x6<3>(a, bp, acc[T]);
                }
            } else {
                kblock<ORDER>(acc, a, b);
            }
            if (VAR & 1) __builtin_amdgcn_sched_barrier(0);
        }
        if (VAR & 16) {
#pragma unroll
            for (int T = 0; T < 5; ++T)
#pragma unroll
                for (int r = 0; r < 16; ++r) nacc[T][r] += ((mw >> ((r & 3) + 8 * (r >> 2))) & 1u) ? acc[T][r] : 0.f;
            mw = mw * 1664525u + 1013904223u;
        }
    }
#pragma unroll
    for (int T = 0; T < 5; ++T) acc[T] += nacc[T];
    float s = 0.f;
#pragma unroll
    for (int T = 0; T < 5; ++T)
#pragma unroll
        for (int r = 0; r < 16; ++r) s += acc[T][r];
    out[(blockIdx.x * blockDim.x + threadIdx.x)] = s;
}

static float4* g3;
template <int ORDER, int WPS, int VAR = 0>
static void run(float* out, int cus) {
    const int iters = 400;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((k_dep<ORDER, WPS, VAR>), dim3(cus), dim3(256 * WPS), 0, 0, out, iters, 12345u + rep, g3);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
    }
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const double mfmas = (double)cus * 4 * WPS * iters * 10 * 30;
    const double flops = mfmas * 2.0 * 32 * 32 * 16;
    printf("order %d waves/SIMD %d var %d: %.3f ms  %.1f TF/s bf16 = %.3f of 2.5 PF (%.1f ns per MFMA per SIMD)\n", ORDER, WPS, VAR, ms,
           flops / ms / 1e9, flops / ms / 1e9 / 2500.0, ms * 1e6 / (mfmas / (cus * 4)));
    (void)VAR;
}

int main() {
    int dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    float* out;
    hipMalloc(&out, (size_t)cus * 512 * sizeof(float));
    hipMalloc(&g3, (size_t)(cus * 8 + 8) * 64 * 16 * 9);
    hipMemset(g3, 0, (size_t)(cus * 8 + 8) * 64 * 16 * 9);
    run<0, 2, 1>(out, cus);
    run<1, 2, 1>(out, cus);
    run<0, 2, 3>(out, cus);
    run<2, 2, 3>(out, cus);
    run<0, 2, 15>(out, cus);
    run<2, 2, 15>(out, cus);
    run<0, 2, 31>(out, cus);
    run<2, 2, 31>(out, cus);
    return 0;
}
