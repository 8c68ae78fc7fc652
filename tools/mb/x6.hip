// Microbenchmark: fp32-accurate GEMM by a 3-way bf16 split (6 bf16 products per fp32 product,
// v_mfma_f32_32x32x16_bf16) vs the native v_mfma_f32_32x32x2_f32, natural orientation
// (rows on the A lanes, W[160][160] as a B-operand image in LDS), one layer Y = X·W over R rows.
// Build: hipcc -O3 --offload-arch=gfx950 -o x6 x6.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
#include <cstring>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int K = 160, NC = 160, NT = 5, NKB = 10;

__device__ __forceinline__ void split8(const float (&x)[8], bf16x8& h, bf16x8& m, bf16x8& l) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const __bf16 hb = (__bf16)x[e];
        const float r = x[e] - (float)hb;
        const __bf16 mb = (__bf16)r;
        const float r2 = r - (float)mb;
        h[e] = hb;
        m[e] = mb;
        l[e] = (__bf16)r2;
    }
}

// image: [T][kb][part][lane][8 bf16] (16 B per lane)
template <int NPROD>
__global__ __launch_bounds__(512, 1) void k_x6(const float* X, const uint4* wimg, float* Y, int nblk) {
    __shared__ uint4 wl[NT * NKB * 3 * 64];
    for (int i = threadIdx.x; i < NT * NKB * 3 * 64; i += blockDim.x) wl[i] = wimg[i];
    __syncthreads();
    const int lane = threadIdx.x & 63, i = lane & 31, h = lane >> 5;
    const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int b = blockIdx.x * nw + wave; b < nblk; b += gridDim.x * nw) {
        f32x16 acc[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
        const float* xr = X + ((size_t)b * 32 + i) * K + 8 * h;
#pragma unroll 2
        for (int kb = 0; kb < NKB; ++kb) {
            const float4 x0 = *reinterpret_cast<const float4*>(xr + 16 * kb);
            const float4 x1 = *reinterpret_cast<const float4*>(xr + 16 * kb + 4);
            const float xv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
            bf16x8 ah, am, al;
            split8(xv, ah, am, al);
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const uint4* wp = wl + ((t * NKB + kb) * 3) * 64 + lane;
                const uint4 uh = wp[0], um = wp[64], ul = wp[128];
                bf16x8 bh, bm, bl;
                memcpy(&bh, &uh, 16);
                memcpy(&bm, &um, 16);
                memcpy(&bl, &ul, 16);
                if (NPROD >= 6) {
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, acc[t], 0, 0, 0);
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc[t], 0, 0, 0);
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc[t], 0, 0, 0);
                }
                if (NPROD >= 3) {
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, acc[t], 0, 0, 0);
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, acc[t], 0, 0, 0);
                }
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc[t], 0, 0, 0);
            }
        }
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
                Y[((size_t)b * 32 + row) * NC + 32 * t + i] = acc[t][r];
            }
    }
}

// fp32: image [T][c (20 chunks of 8 k)][lane][4 floats]: lane (j,h) holds W[8c + 2s + h][32T + j], s=0..3
__global__ __launch_bounds__(512, 1) void k_f32(const float* X, const float4* wimg, float* Y, int nblk) {
    __shared__ float4 wl[NT * 20 * 64];
    for (int i = threadIdx.x; i < NT * 20 * 64; i += blockDim.x) wl[i] = wimg[i];
    __syncthreads();
    const int lane = threadIdx.x & 63, i = lane & 31, h = lane >> 5;
    const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int b = blockIdx.x * nw + wave; b < nblk; b += gridDim.x * nw) {
        f32x16 acc[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
        const float* xr = X + ((size_t)b * 32 + i) * K;
#pragma unroll 2
        for (int c = 0; c < 20; ++c) {
            const float4 x0 = *reinterpret_cast<const float4*>(xr + 8 * c);
            const float4 x1 = *reinterpret_cast<const float4*>(xr + 8 * c + 4);
            const float a0 = h ? x0.y : x0.x, a1 = h ? x0.w : x0.z, a2 = h ? x1.y : x1.x, a3 = h ? x1.w : x1.z;
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const float4 w = wl[(t * 20 + c) * 64 + lane];
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, w.x, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, w.y, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a2, w.z, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a3, w.w, acc[t], 0, 0, 0);
            }
        }
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
                Y[((size_t)b * 32 + row) * NC + 32 * t + i] = acc[t][r];
            }
    }
}

static uint16_t bf16_rne(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}
static float bf16_f(uint16_t b) {
    uint32_t u = (uint32_t)b << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
    const int R = argc > 1 ? atoi(argv[1]) : (1 << 21);
    const int nblk = R / 32;
    std::vector<float> hX((size_t)R * K), hW(K * NC);
    srand(1);
    auto rnd = [] { return (float)rand() / RAND_MAX * 2.f - 1.f; };
    for (auto& v : hW) v = rnd() * 0.1f;
    for (size_t r = 0; r < (size_t)R; ++r)
        for (int k = 0; k < K; ++k) hX[r * K + k] = (k < 150) ? fmaxf(rnd(), 0.f) * (1.f + 3.f * (r % 7)) : 0.f;
    // bf16x3 image
    std::vector<uint16_t> img((size_t)NT * NKB * 3 * 64 * 8);
    for (int t = 0; t < NT; ++t)
        for (int kb = 0; kb < NKB; ++kb)
            for (int l = 0; l < 64; ++l)
                for (int e = 0; e < 8; ++e) {
                    const float w = hW[(16 * kb + 8 * (l >> 5) + e) * NC + 32 * t + (l & 31)];
                    const uint16_t hb = bf16_rne(w);
                    const float r = w - bf16_f(hb);
                    const uint16_t mb = bf16_rne(r);
                    const uint16_t lb = bf16_rne(r - bf16_f(mb));
                    const uint16_t parts[3] = {hb, mb, lb};
                    for (int p = 0; p < 3; ++p) img[((((size_t)(t * NKB + kb) * 3 + p) * 64 + l) * 8) + e] = parts[p];
                }
    std::vector<float> img32((size_t)NT * 20 * 64 * 4);
    for (int t = 0; t < NT; ++t)
        for (int c = 0; c < 20; ++c)
            for (int l = 0; l < 64; ++l)
                for (int s = 0; s < 4; ++s)
                    img32[(((size_t)t * 20 + c) * 64 + l) * 4 + s] = hW[(8 * c + 2 * s + (l >> 5)) * NC + 32 * t + (l & 31)];
    float *dX, *dY, *dW32;
    uint4* dimg;
    CK(hipMalloc(&dX, hX.size() * 4));
    CK(hipMalloc(&dY, (size_t)R * NC * 4));
    CK(hipMalloc(&dimg, img.size() * 2));
    CK(hipMalloc(&dW32, img32.size() * 4));
    CK(hipMemcpy(dX, hX.data(), hX.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dimg, img.data(), img.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dW32, img32.data(), img32.size() * 4, hipMemcpyHostToDevice));
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int NCHK = 4096;
    std::vector<double> ref((size_t)NCHK * NC), mag((size_t)NCHK * NC);
    for (int r = 0; r < NCHK; ++r)
        for (int j = 0; j < NC; ++j) {
            double s = 0, a = 0;
            for (int k = 0; k < K; ++k) {
                s += (double)hX[(size_t)r * K + k] * hW[k * NC + j];
                a += fabs((double)hX[(size_t)r * K + k] * hW[k * NC + j]);
            }
            ref[(size_t)r * NC + j] = s;
            mag[(size_t)r * NC + j] = a;
        }
    std::vector<float> hY((size_t)NCHK * NC);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double flops = 2.0 * R * K * NC;
    for (int variant = 0; variant < 4; ++variant)
        for (int wpc : {4, 8}) {
            auto launch = [&] {
                if (variant == 0) hipLaunchKernelGGL(k_f32, dim3(ncu), dim3(64 * wpc), 0, 0, dX, (const float4*)dW32, dY, nblk);
                if (variant == 1) hipLaunchKernelGGL(k_x6<6>, dim3(ncu), dim3(64 * wpc), 0, 0, dX, dimg, dY, nblk);
                if (variant == 2) hipLaunchKernelGGL(k_x6<3>, dim3(ncu), dim3(64 * wpc), 0, 0, dX, dimg, dY, nblk);
                if (variant == 3) hipLaunchKernelGGL(k_x6<1>, dim3(ncu), dim3(64 * wpc), 0, 0, dX, dimg, dY, nblk);
            };
            launch();
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0));
            const int it = 10;
            for (int q = 0; q < it; ++q) launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ms /= it;
            CK(hipMemcpy(hY.data(), dY, hY.size() * 4, hipMemcpyDeviceToHost));
            double emax = 0, erel = 0;
            for (size_t q = 0; q < hY.size(); ++q) {
                const double e = fabs(hY[q] - ref[q]);
                emax = fmax(emax, e / (mag[q] + 1e-30));
                erel = fmax(erel, e / (fabs(ref[q]) + 1e-3 * mag[q]));
            }
            const char* nm[4] = {"f32 mfma", "bf16x6", "bf16x3", "bf16x1"};
            printf("%-9s waves/CU=%d  %.3f ms  %.1f TF(alg)  %.1f GB/s  err/sum|xw|=%.3g  rel=%.3g\n", nm[variant], wpc, ms,
                   flops / ms / 1e9, (double)R * (K + NC) * 4 / ms / 1e6, emax, erel);
        }
    return 0;
}
