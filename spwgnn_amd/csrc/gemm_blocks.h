// Register-level MFMA building blocks (fp32, v_mfma_f32_32x32x2_f32) used by every kernel.
#pragma once
#include "device_common.h"

namespace spw {

// ---- row I/O for the transposed orientation (lane (j, h) owns row j; C reg r of tile t is
//      feature rho(r,h) + 32t, and regs 4q..4q+3 are the 4 consecutive features 8q + 4h + 32t + 0..3).
template <int NT>
__device__ __forceinline__ void store_rho(float* __restrict__ row, const f32x16 (&X)[NT], int h) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float4 v = make_float4(X[t][4 * q], X[t][4 * q + 1], X[t][4 * q + 2], X[t][4 * q + 3]);
            *reinterpret_cast<float4*>(row + 32 * t + 8 * q + 4 * h) = v;
        }
}
template <int NT>
__device__ __forceinline__ void store_rho_masked(float* __restrict__ row, const f32x16 (&X)[NT], int h, bool valid) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float4 v = valid ? make_float4(X[t][4 * q], X[t][4 * q + 1], X[t][4 * q + 2], X[t][4 * q + 3])
                             : make_float4(0.f, 0.f, 0.f, 0.f);
            *reinterpret_cast<float4*>(row + 32 * t + 8 * q + 4 * h) = v;
        }
}
template <int NT>
__device__ __forceinline__ void load_rho(const float* __restrict__ row, f32x16 (&X)[NT], int h) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float4 v = *reinterpret_cast<const float4*>(row + 32 * t + 8 * q + 4 * h);
            X[t][4 * q] = v.x;
            X[t][4 * q + 1] = v.y;
            X[t][4 * q + 2] = v.z;
            X[t][4 * q + 3] = v.w;
        }
}

// ---- split-halves row chunk: lane half h holds features [KH*h, KH*h+KH) of its row.
template <int KH>
__device__ __forceinline__ void load_half(const float* __restrict__ row_plus_khh, float (&x)[KH]) {
    static_assert(KH % 4 == 0, "KH multiple of 4");
    const float4* p = reinterpret_cast<const float4*>(row_plus_khh);
#pragma unroll
    for (int q = 0; q < KH / 4; ++q) {
        float4 v = p[q];
        x[4 * q] = v.x;
        x[4 * q + 1] = v.y;
        x[4 * q + 2] = v.z;
        x[4 * q + 3] = v.w;
    }
}

// ---- transposed orientation: out[t] += Wᵀ·in over register k-steps.
// in: C layout of the previous layer (feature rho(r,h)+32tp on the lane's row); the k-steps are
// (tp, r) for tp < NT_IN, with r < LAST_R in the last input tile (rows beyond are zero padding).
// W: [in][out] row-major with row stride LDW; the A operand of lane (i,h) is W[k(h)][32t + i].
// The weight fragments run PF k-steps ahead in a register ring (hipcc otherwise serialises each
// load with its MFMA under register pressure — see DESIGN.md §3).
template <int NT_OUT, int NT_IN, int LAST_R, int LDW, int PF = 3>
__device__ __forceinline__ void tchain_acc(const f32x16 (&in)[NT_IN], f32x16 (&out)[NT_OUT],
                                           const float* __restrict__ W, int lane) {
    const int i = lane & 31, h = lane >> 5;
    const float* wbase = W + (4 * h) * LDW + i;
    constexpr int NK = (NT_IN - 1) * 16 + LAST_R;
    float w[PF + 1][NT_OUT];
#pragma unroll
    for (int k = 0; k < PF; ++k) {
        if (k >= NK) break;
        const float* wrow = wbase + (rho(k & 15, 0) + 32 * (k >> 4)) * LDW;
#pragma unroll
        for (int t = 0; t < NT_OUT; ++t) w[k][t] = wrow[32 * t];
    }
#pragma unroll
    for (int k = 0; k < NK; ++k) {
        if (k + PF < NK) {
            const int kk = k + PF;
            const float* wrow = wbase + (rho(kk & 15, 0) + 32 * (kk >> 4)) * LDW;
#pragma unroll
            for (int t = 0; t < NT_OUT; ++t) w[kk % (PF + 1)][t] = wrow[32 * t];
        }
        const float b = in[k >> 4][k & 15];
#pragma unroll
        for (int t = 0; t < NT_OUT; ++t) out[t] = mfma32(w[k % (PF + 1)][t], b, out[t]);
    }
}

// ---- transposed orientation, B operand from a split-halves row chunk x (features KH*h + s).
template <int NT_OUT, int KH, int LDW, int PF = 3>
__device__ __forceinline__ void tgemm_half_acc(const float (&x)[KH], f32x16 (&out)[NT_OUT],
                                               const float* __restrict__ W, int lane) {
    const int i = lane & 31, h = lane >> 5;
    const float* wbase = W + (KH * h) * LDW + i;
    float w[PF + 1][NT_OUT];
#pragma unroll
    for (int k = 0; k < PF; ++k)
#pragma unroll
        for (int t = 0; t < NT_OUT; ++t) w[k][t] = wbase[k * LDW + 32 * t];
#pragma unroll
    for (int s = 0; s < KH; ++s) {
        if (s + PF < KH) {
#pragma unroll
            for (int t = 0; t < NT_OUT; ++t) w[(s + PF) % (PF + 1)][t] = wbase[(s + PF) * LDW + 32 * t];
        }
#pragma unroll
        for (int t = 0; t < NT_OUT; ++t) out[t] = mfma32(w[s % (PF + 1)][t], x[s], out[t]);
    }
}

// ---- natural orientation: acc[t] += A·W, A operand = this lane's row chunk a (features KH*h+s),
// W: [k][col] row stride LDW; B operand of lane (j,h) is W[KH*h + s][32t + j].
template <int NT_OUT, int KH, int LDW>
__device__ __forceinline__ void ngemm_acc(const float (&a)[KH], f32x16 (&acc)[NT_OUT],
                                          const float* __restrict__ W, int lane) {
    const int j = lane & 31, h = lane >> 5;
    const float* wbase = W + (KH * h) * LDW + j;
#pragma unroll
    for (int s = 0; s < KH; ++s) {
        const float* wrow = wbase + s * LDW;
#pragma unroll
        for (int t = 0; t < NT_OUT; ++t) acc[t] = mfma32(a[s], wrow[32 * t], acc[t]);
    }
}

// ---- LDS image of a [160][160] (k-major, ld kLdE) packed weight for the natural-orientation edge
// kernels: wl[col * kWlK + k] = W[k][col], k < 152 (the two 76-feature halves). A lane's 4
// consecutive k of one column are one ds_read_b128; kWlK ≡ 28 (mod 32) keeps 8 consecutive
// lanes on distinct 4-bank groups.
constexpr int kWlK = 156;
constexpr int kWlFloats = 160 * kWlK;
constexpr int kEdgeWaves = 8;   // waves per edge workgroup (one workgroup per CU: 97.5 KiB of LDS)
__device__ __forceinline__ void wl_fill(float* wl, const float* __restrict__ W) {
    for (int idx = threadIdx.x; idx < 160 * 2 * kKhE; idx += blockDim.x) {
        const int k = idx / 160, col = idx - k * 160;
        wl[col * kWlK + k] = W[k * kLdE + col];
    }
    __syncthreads();
}

template <int NT>
__device__ __forceinline__ void zero_tiles(f32x16 (&X)[NT]) {
#pragma unroll
    for (int t = 0; t < NT; ++t) X[t] = zero16();
}

// bias (padded vector, feature rho(r,h)+32t) + optional relu, in place (transposed C layout).
template <int NT, bool RELU>
__device__ __forceinline__ void bias_act_rho(f32x16 (&X)[NT], const float* __restrict__ b, int h) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            float v = X[t][r] + b[rho(r, 0) + 4 * h + 32 * t];
            X[t][r] = RELU ? relu(v) : v;
        }
}

}  // namespace spw
