// Weight gradients (dW = Σ_rows Xᵀ·Y, deterministic split-row slabs + ordered reduction),
// Keras BCE loss, Keras Adam, sigmoid readout.
#include "kernels.h"

namespace spw {

constexpr int kWgThreads = 320;   // 5 waves: wave w owns output row tile w (32 x-features × all y tiles)

__device__ __forceinline__ int64_t wg_phys(int64_t L, int64_t count, int64_t stride) {
    const int64_t s = L / count, n = L - s * count;
    return (stride ? s * stride : 0) + n;
}
__device__ __forceinline__ float4 f4zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
__device__ __forceinline__ void f4set(float4& v, int k, float x) {
    if (k == 0) v.x = x; else if (k == 1) v.y = x; else if (k == 2) v.z = x; else if (k == 3) v.w = x;
}
__device__ __forceinline__ float4 f4relu(float4 v) {
    return make_float4(relu(v.x), relu(v.y), relu(v.z), relu(v.w));
}
__device__ __forceinline__ float4 f4add3(float4 a, float4 b, float4 c) {
    return make_float4(a.x + b.x + c.x, a.y + b.y + c.y, a.z + b.z + c.z, a.w + b.w + c.w);
}

// 4 consecutive X features [f0, f0+4) of logical row L (all producers write zero padding up to ld)
template <int XM>
__device__ __forceinline__ float4 wg_x4(const WgradArgs& a, int64_t L, int f0) {
    if (XM == XM_ROW) {
        const int64_t r = wg_phys(L, a.x_count, a.x_stride);
        float4 v = f0 < a.x_ld ? *reinterpret_cast<const float4*>(a.x_ptr + r * a.x_ld + f0) : f4zero();
        if (a.x_ones >= f0 && a.x_ones < f0 + 4) f4set(v, a.x_ones - f0, 1.f);
        return v;
    } else if (XM == XM_EDGE_D) {
        const int sidx = a.esrc[L];
        float4 v = f4zero();
        if (sidx >= 0 && f0 == 0) {
            const float4 ps = reinterpret_cast<const float4*>(a.pos)[sidx];
            const float4 pd = reinterpret_cast<const float4*>(a.pos)[a.edst[L]];
            v = make_float4(pd.x - ps.x, pd.y - ps.y, 1.f, 0.f);
        }
        return v;
    } else if (XM == XM_NODE_O) {
        float4 v = f4zero();
        if (f0 == 0) {
            const float4 p = reinterpret_cast<const float4*>(a.pos)[L];
            v = make_float4(p.y, p.z, 1.f, 0.f);
        }
        return v;
    } else {  // XM_EDGE_H1
        const int64_t s = L / a.RE, e = L - s * a.RE;
        const int sidx = a.esrc[e];
        if (sidx < 0) return f4zero();
        const int didx = a.edst[e];
        const float4 x = *reinterpret_cast<const float4*>(a.A + e * kLdE + f0);
        const float4 u = *reinterpret_cast<const float4*>(a.U + (s * a.RN + sidx) * kLdE + f0);
        const float4 w = *reinterpret_cast<const float4*>(a.V + (s * a.RN + didx) * kLdE + f0);
        float4 v = f4relu(f4add3(x, u, w));
        if (f0 == 148) { v.z = 1.f; v.w = 0.f; }        // feature 150 = ones (b2), 151 = 0
        else if (f0 >= 152) v = f4zero();
        return v;
    }
}

template <int YM>
__device__ __forceinline__ float4 wg_y4(const WgradArgs& a, int64_t L, int f0) {
    if (YM == YM_ROW) {
        const int64_t r = wg_phys(L, a.y_count, a.y_stride);
        return f0 < a.y_ld ? *reinterpret_cast<const float4*>(a.y_ptr + r * a.y_ld + f0) : f4zero();
    } else {  // YM_EDGE_DH2
        const int64_t s = L / a.RE, e = L - s * a.RE;
        const int didx = a.edst[e];
        if (didx < 0 || f0 >= 152) return f4zero();
        const uint32_t word = a.mask2[(s * (a.RE / 32) + (e >> 5)) * 160 + (f0 >> 5) * 32 + (e & 31)];
        const uint32_t bits = word >> (f0 & 31);
        const float4 g = *reinterpret_cast<const float4*>(a.G3 + (s * a.RN + didx) * kLdE + f0);
        return make_float4((bits & 1u) ? g.x : 0.f, (bits & 2u) ? g.y : 0.f, (bits & 4u) ? g.z : 0.f,
                           (bits & 8u) ? g.w : 0.f);
    }
}

// dW[k][n] (slab per chunk) = Σ_{rows of the chunk} X[row][k] · Y[row][n]
template <int XM, int YM, int KXP, int NYP>
__global__ __launch_bounds__(kWgThreads) void k_wgrad_t(WgradArgs a) {
    constexpr int TX = KXP / 32, TY = NYP / 32;
    constexpr int LDX = KXP + 4, LDY = NYP + 4;   // 16-B aligned rows; MFMA reads are conflict-free
    constexpr int GX = KXP / 4, GY = NYP / 4;
    __shared__ __attribute__((aligned(16))) float Xs[32 * LDX];
    __shared__ __attribute__((aligned(16))) float Ys[32 * LDY];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, i = lane & 31;
    const int64_t r_begin = (int64_t)blockIdx.x * a.rows_per_chunk;
    const int64_t r_end = min(a.rows, r_begin + a.rows_per_chunk);
    f32x16 acc[TY];
#pragma unroll
    for (int t = 0; t < TY; ++t) acc[t] = zero16();
    for (int64_t r0 = r_begin; r0 < r_end; r0 += 32) {
        __syncthreads();
#pragma unroll
        for (int g = tid; g < 32 * GX; g += kWgThreads) {
            const int rr = g / GX, c4 = g - rr * GX;
            const int64_t L = r0 + rr;
            const float4 v = L < r_end ? wg_x4<XM>(a, L, 4 * c4) : f4zero();
            *reinterpret_cast<float4*>(&Xs[rr * LDX + 4 * c4]) = v;
        }
#pragma unroll
        for (int g = tid; g < 32 * GY; g += kWgThreads) {
            const int rr = g / GY, c4 = g - rr * GY;
            const int64_t L = r0 + rr;
            const float4 v = L < r_end ? wg_y4<YM>(a, L, 4 * c4) : f4zero();
            *reinterpret_cast<float4*>(&Ys[rr * LDY + 4 * c4]) = v;
        }
        __syncthreads();
        if (wave < TX) {
#pragma unroll
            for (int k2 = 0; k2 < 16; ++k2) {
                const int rr = 2 * k2 + h;
                const float av = Xs[rr * LDX + 32 * wave + i];
#pragma unroll
                for (int ty = 0; ty < TY; ++ty) acc[ty] = mfma32(av, Ys[rr * LDY + 32 * ty + i], acc[ty]);
            }
        }
    }
    if (wave < TX) {
        float* out = a.slab + (int64_t)blockIdx.x * KXP * NYP;
#pragma unroll
        for (int ty = 0; ty < TY; ++ty)
#pragma unroll
            for (int r = 0; r < 16; ++r) out[(int64_t)(32 * wave + rho(r, 0) + 4 * h) * NYP + 32 * ty + i] = acc[ty][r];
    }
}

// stage 1: partial[g][idx] = Σ_{c in group g} slab[c][idx] (contiguous chunk ranges, fixed order)
__global__ void k_wgrad_reduce1(ReduceArgs a, float* partial, int groups) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const int n = a.kx_pad * a.ny_pad;
    if (idx >= n) return;
    const int g = blockIdx.y;
    const int per = (a.chunks + groups - 1) / groups;
    const int c0 = g * per, c1 = min(a.chunks, c0 + per);
    float s = 0.f;
    for (int c = c0; c < c1; ++c) s += a.slab[(int64_t)c * n + idx];
    partial[(int64_t)g * n + idx] = s;
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
    const dim3 g(chunks), b(kWgThreads);
#define SPW_WG(XM, YM, KX, NY)                                                               \
    if (a.xmode == XM && a.ymode == YM && a.kx_pad == KX && a.ny_pad == NY) {                 \
        hipLaunchKernelGGL((k_wgrad_t<XM, YM, KX, NY>), g, b, 0, st, a);                      \
        return hipGetLastError();                                                             \
    }
    SPW_WG(XM_ROW, YM_ROW, 160, 160)
    SPW_WG(XM_ROW, YM_ROW, 128, 160)
    SPW_WG(XM_ROW, YM_ROW, 160, 128)
    SPW_WG(XM_ROW, YM_ROW, 128, 128)
    SPW_WG(XM_EDGE_D, YM_ROW, 32, 160)
    SPW_WG(XM_NODE_O, YM_ROW, 32, 128)
    SPW_WG(XM_EDGE_H1, YM_EDGE_DH2, 160, 160)
#undef SPW_WG
    return hipErrorInvalidValue;
}
hipError_t launch_wgrad_reduce(const ReduceArgs& a, float* partial, int groups, hipStream_t st) {
    const int n = a.kx_pad * a.ny_pad;
    if (groups > 1 && a.chunks > groups) {
        hipLaunchKernelGGL(k_wgrad_reduce1, dim3((n + 255) / 256, groups), dim3(256), 0, st, a, partial, groups);
        ReduceArgs b = a;
        b.slab = partial;
        b.chunks = groups;
        hipLaunchKernelGGL(k_wgrad_reduce, dim3((n + 255) / 256), dim3(256), 0, st, b);
    } else {
        hipLaunchKernelGGL(k_wgrad_reduce, dim3((n + 255) / 256), dim3(256), 0, st, a);
    }
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
