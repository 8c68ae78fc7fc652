// Weight gradients (dW = Σ_rows Xᵀ·Y, deterministic split-row slabs + ordered reduction),
// Keras BCE loss, Keras Adam, sigmoid readout.
#include "kernels.h"

namespace spw {

constexpr int kWgThreads = 320;   // 5 waves: wave w owns output row tile w (32 x-features × all y tiles)
constexpr int kWgLd = 161;        // LDS row stride (odd: conflict-free column reads)

__device__ __forceinline__ int64_t wg_phys(int64_t L, int64_t count, int64_t stride) {
    const int64_t s = L / count, n = L - s * count;
    return (stride ? s * stride : 0) + n;
}

__device__ __forceinline__ float wg_x(const WgradArgs& a, int64_t L, int f) {
    switch (a.xmode) {
        case XM_ROW: {
            if (f < a.x_width) return a.x_ptr[wg_phys(L, a.x_count, a.x_stride) * a.x_ld + f];
            return f == a.x_ones ? 1.f : 0.f;
        }
        case XM_EDGE_D: {
            const int64_t e = L;
            const int sidx = a.esrc[e];
            if (sidx < 0) return 0.f;
            if (f < 2) return a.pos[(int64_t)a.edst[e] * 4 + f] - a.pos[(int64_t)sidx * 4 + f];
            return f == 2 ? 1.f : 0.f;
        }
        case XM_NODE_O: {
            if (f < 2) return a.pos[L * 4 + 1 + f];
            return f == 2 ? 1.f : 0.f;
        }
        default: {  // XM_EDGE_H1, L = s*RE + e
            const int64_t s = L / a.RE, e = L - s * a.RE;
            const int sidx = a.esrc[e];
            if (sidx < 0) return 0.f;
            if (f < kFE) {
                const int didx = a.edst[e];
                const float v = a.A[e * kLdE + f] + a.U[(s * a.RN + sidx) * kLdE + f] + a.V[(s * a.RN + didx) * kLdE + f];
                return relu(v);
            }
            return f == kFE ? 1.f : 0.f;
        }
    }
}

__device__ __forceinline__ float wg_y(const WgradArgs& a, int64_t L, int f) {
    if (a.ymode == YM_ROW) return f < a.y_width ? a.y_ptr[wg_phys(L, a.y_count, a.y_stride) * a.y_ld + f] : 0.f;
    // YM_EDGE_DH2
    const int64_t s = L / a.RE, e = L - s * a.RE;
    const int didx = a.edst[e];
    if (didx < 0 || f >= kFE) return 0.f;
    const uint32_t word = a.mask2[(s * (a.RE / 32) + (e >> 5)) * 160 + (f >> 5) * 32 + (e & 31)];
    return ((word >> (f & 31)) & 1u) ? a.G3[(s * a.RN + didx) * kLdE + f] : 0.f;
}

__global__ __launch_bounds__(kWgThreads) void k_wgrad(WgradArgs a) {
    __shared__ float Xs[32 * kWgLd];
    __shared__ float Ys[32 * kWgLd];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, i = lane & 31;
    const int64_t r_begin = (int64_t)blockIdx.x * a.rows_per_chunk;
    const int64_t r_end = min(a.rows, r_begin + a.rows_per_chunk);
    const int TX = a.kx_pad / 32, TY = a.ny_pad / 32;
    f32x16 acc[5];
    zero_tiles(acc);
    for (int64_t r0 = r_begin; r0 < r_end; r0 += 32) {
        __syncthreads();
        for (int idx = tid; idx < 32 * a.kx_pad; idx += kWgThreads) {
            const int rr = idx / a.kx_pad, f = idx - rr * a.kx_pad;
            const int64_t L = r0 + rr;
            Xs[rr * kWgLd + f] = L < r_end ? wg_x(a, L, f) : 0.f;
        }
        for (int idx = tid; idx < 32 * a.ny_pad; idx += kWgThreads) {
            const int rr = idx / a.ny_pad, f = idx - rr * a.ny_pad;
            const int64_t L = r0 + rr;
            Ys[rr * kWgLd + f] = L < r_end ? wg_y(a, L, f) : 0.f;
        }
        __syncthreads();
        if (wave < TX) {
#pragma unroll 4
            for (int k2 = 0; k2 < 16; ++k2) {
                const int rr = 2 * k2 + h;
                const float av = Xs[rr * kWgLd + 32 * wave + i];
#pragma unroll
                for (int ty = 0; ty < 5; ++ty)
                    if (ty < TY) acc[ty] = mfma32(av, Ys[rr * kWgLd + 32 * ty + i], acc[ty]);
            }
        }
    }
    if (wave < TX) {
        float* out = a.slab + (int64_t)blockIdx.x * a.kx_pad * a.ny_pad;
#pragma unroll
        for (int ty = 0; ty < 5; ++ty) {
            if (ty >= TY) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) out[(int64_t)(32 * wave + rho(r, 0) + 4 * h) * a.ny_pad + 32 * ty + i] = acc[ty][r];
        }
    }
}

__global__ void k_wgrad_reduce(ReduceArgs a) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= a.kx_pad * a.ny_pad) return;
    const int k = idx / a.ny_pad, n = idx - k * a.ny_pad;
    const int64_t stride = (int64_t)a.kx_pad * a.ny_pad;
    float s = 0.f;
    for (int c = 0; c < a.chunks; ++c) s += a.slab[c * stride + idx];
    int col = a.perm ? wo2_perm(n) : n;
    if (col < 0 || col >= a.kernel_cols) return;
    if (a.kernel_off >= 0 && k < a.kernel_rows) a.out[a.kernel_off + (int64_t)(a.kernel_row0 + k) * a.kernel_cols + col] = s;
    if (a.bias_off >= 0 && k == a.bias_row) a.out[a.bias_off + col] = s;
}

// ------------------------------------------------------------------------------------------------
// Keras binary_crossentropy (Networks.py:192): clip(ŷ, 1e-7, 1-1e-7) ≡ clamp(z, ±ln((1-ε)/ε)).
constexpr float kLogitClip = 16.11809565f;

__global__ __launch_bounds__(256) void k_bce_partial(BceArgs a) {
    __shared__ float sl[256], sc[256];
    float ls = 0.f, cs = 0.f;
    const float inv_n = 1.0f / (float)a.n;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < a.n; i += (int64_t)a.blocks * 256) {
        const float z0 = a.logits[i], t = a.targets[i];
        const float z = fminf(fmaxf(z0, -kLogitClip), kLogitClip);
        ls += fmaxf(z, 0.f) - z * t + log1pf(expf(-fabsf(z)));
        const float p = 1.f / (1.f + expf(-z0));
        cs += ((p > 0.5f ? 1.f : 0.f) == t) ? 1.f : 0.f;
        if (a.dlogits) a.dlogits[i] = fabsf(z0) < kLogitClip ? (p - t) * inv_n : 0.f;
    }
    sl[threadIdx.x] = ls;
    sc[threadIdx.x] = cs;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            sl[threadIdx.x] += sl[threadIdx.x + o];
            sc[threadIdx.x] += sc[threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        a.partial[2 * blockIdx.x] = sl[0];
        a.partial[2 * blockIdx.x + 1] = sc[0];
    }
}

__global__ void k_bce_final(BceArgs a) {
    if (threadIdx.x != 0) return;
    double ls = 0.0, cs = 0.0;
    for (int b = 0; b < a.blocks; ++b) {
        ls += a.partial[2 * b];
        cs += a.partial[2 * b + 1];
    }
    a.out3[0] = (float)(ls / (double)a.n);
    a.out3[1] = (float)cs;
    a.out3[2] = (float)a.n;
}

__global__ void k_adam(AdamArgs a) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
        const float p = a.p[i];
        const float g = a.gscale * a.g[i] + 2.f * a.l2 * p;
        const float m = a.b1 * a.m[i] + (1.f - a.b1) * g;
        const float v = a.b2 * a.v[i] + (1.f - a.b2) * g * g;
        a.m[i] = m;
        a.v[i] = v;
        a.p[i] = p - a.lr_t * m / (sqrtf(v) + a.eps);
    }
}

__global__ void k_sigmoid(const float* z, float* p, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = 1.f / (1.f + expf(-z[i]));
}

// ------------------------------------------------------------------------------------------------
hipError_t launch_wgrad(const WgradArgs& a, int chunks, hipStream_t st) {
    hipLaunchKernelGGL(k_wgrad, dim3(chunks), dim3(kWgThreads), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_wgrad_reduce(const ReduceArgs& a, hipStream_t st) {
    const int n = a.kx_pad * a.ny_pad;
    hipLaunchKernelGGL(k_wgrad_reduce, dim3((n + 255) / 256), dim3(256), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_bce(const BceArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(k_bce_partial, dim3(a.blocks), dim3(256), 0, st, a);
    hipLaunchKernelGGL(k_bce_final, dim3(1), dim3(64), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_adam(const AdamArgs& a, hipStream_t st) {
    const int64_t blocks = std::min<int64_t>((a.n + 255) / 256, 2048);
    hipLaunchKernelGGL(k_adam, dim3((unsigned)blocks), dim3(256), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_sigmoid(const float* z, float* p, int64_t n, hipStream_t st) {
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 2048);
    hipLaunchKernelGGL(k_sigmoid, dim3((unsigned)std::max<int64_t>(blocks, 1)), dim3(256), 0, st, z, p, n);
    return hipGetLastError();
}

}  // namespace spw
