// Accuracy of split-bf16 products on a long, cancelling reduction (a weight-gradient element:
// dW[i][j] = Σ_r X[r][i]·Y[r][j], R rows, random-sign data) vs the f32 MFMA fma chain, against fp64.
// Variants: x6 into one accumulator; x6 with the h·h products in their own accumulator; x9.
// Build: hipcc -O3 --offload-arch=gfx950 -I../../spwgnn_amd/csrc -o x6acc x6acc.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
#include "device_common.h"
using namespace spw;

constexpr int R = 8192, F = 16;

__device__ void split8(const float* v, bf16x8 (&p)[3]) {
    uint32_t hw[4], mw[4], lw[4];
    for (int m = 0; m < 4; ++m) split2(v[2 * m], v[2 * m + 1], hw[m], mw[m], lw[m]);
    p[0] = as_bf16x8(make_uint4(hw[0], hw[1], hw[2], hw[3]));
    p[1] = as_bf16x8(make_uint4(mw[0], mw[1], mw[2], mw[3]));
    p[2] = as_bf16x8(make_uint4(lw[0], lw[1], lw[2], lw[3]));
}

// X, Y: [R][F] row-major; out [F][F]; one wave
template <int MODE>
__global__ void k(const float* X, const float* Y, float* out) {
    const int l = threadIdx.x, i = l & 15, g = l >> 4;
    f32x4 acc = {0, 0, 0, 0}, acc2 = {0, 0, 0, 0};
    for (int r0 = 0; r0 < R; r0 += 32) {
        if (MODE == 3) {   // f32 MFMA 16x16x4: A lane (i, k=g), B lane (k=g, j=i)
            for (int s = 0; s < 8; ++s) {
                const int r = r0 + 4 * s + g;
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(X[r * F + i], Y[r * F + i], acc, 0, 0, 0);
            }
            continue;
        }
        float xv[8], yv[8];
        for (int e = 0; e < 8; ++e) {
            const int r = r0 + 8 * g + e;
            xv[e] = X[r * F + i];
            yv[e] = Y[r * F + i];
        }
        bf16x8 a[3], b[3];
        split8(xv, a);
        split8(yv, b);
        if (MODE == 0) {
            acc = mfma16_x6(a, b, acc);
        } else if (MODE == 1) {
            acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], acc2, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], acc2, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], acc2, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], acc2, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], acc2, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], acc, 0, 0, 0);
        } else {   // x9
            for (int p = 2; p >= 0; --p)
                for (int q = 2; q >= 0; --q) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[p], b[q], acc, 0, 0, 0);
        }
    }
    for (int r = 0; r < 4; ++r) out[(4 * g + r) * F + i] = acc[r] + acc2[r];
}

int main() {
    std::vector<float> X(R * F), Y(R * F);
    srand(7);
    auto nrm = [] { float u1 = (rand() + 1.f) / (RAND_MAX + 2.f), u2 = (rand() + 1.f) / (RAND_MAX + 2.f);
                    return sqrtf(-2.f * logf(u1)) * cosf(6.2831853f * u2); };
    for (int r = 0; r < R; ++r)
        for (int f = 0; f < F; ++f) {
            X[r * F + f] = nrm() * (r % 3 == 0 ? 3.f : 0.1f);            // relu-ish magnitudes
            Y[r * F + f] = nrm() * 1e-3f * (1 + (r % 5));
        }
    std::vector<double> ref(F * F, 0.0), mag(F * F, 0.0);
    for (int r = 0; r < R; ++r)
        for (int i = 0; i < F; ++i)
            for (int j = 0; j < F; ++j) {
                const double p = (double)X[r * F + i] * Y[r * F + j];
                ref[i * F + j] += p;
                mag[i * F + j] += fabs(p);
            }
    float *dX, *dY, *dO;
    hipMalloc(&dX, X.size() * 4); hipMalloc(&dY, Y.size() * 4); hipMalloc(&dO, F * F * 4);
    hipMemcpy(dX, X.data(), X.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dY, Y.data(), Y.size() * 4, hipMemcpyHostToDevice);
    const char* nm[4] = {"x6 one acc", "x6 hh + rest", "x9", "f32 mfma"};
    for (int mode = 0; mode < 4; ++mode) {
        if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, dX, dY, dO);
        if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, dX, dY, dO);
        if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(1), dim3(64), 0, 0, dX, dY, dO);
        if (mode == 3) hipLaunchKernelGGL(k<3>, dim3(1), dim3(64), 0, 0, dX, dY, dO);
        std::vector<float> o(F * F);
        hipMemcpy(o.data(), dO, F * F * 4, hipMemcpyDeviceToHost);
        double emax = 0, erel = 0, emag = 0;
        for (int q = 0; q < F * F; ++q) {
            const double e = fabs(o[q] - ref[q]);
            emax = fmax(emax, e);
            erel = fmax(erel, e / fabs(ref[q]));
            emag = fmax(emag, e / mag[q]);
        }
        printf("%-14s max|err| %.3e  max rel %.3e  max err/Σ|ab| %.3e\n", nm[mode], emax, erel, emag);
    }
    return 0;
}
