// FETCH_SIZE calibration per load width (MI355X_MICROARCH.md: only 16-B/lane streaming reads are
// calibrated, FETCH_SIZE = ½ of their bytes). Each kernel reads the same 1 GiB buffer once with
// W-byte loads per lane (coalesced, grid-stride) and writes one float per workgroup.
// build: hipcc -O3 --offload-arch=gfx950 tools/fetchcal.hip -o tools/bin/fetchcal
// run:   rocprofv3 --kernel-trace --pmc FETCH_SIZE -d DIR -o run --output-format csv -- tools/bin/fetchcal
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <class T>
__device__ __forceinline__ float fold(T v);
template <> __device__ __forceinline__ float fold(float4 v) { return v.x + v.y + v.z + v.w; }
template <> __device__ __forceinline__ float fold(uint2 v) { return __uint_as_float(v.x) + __uint_as_float(v.y); }
template <> __device__ __forceinline__ float fold(float v) { return v; }
template <> __device__ __forceinline__ float fold(unsigned short v) { return (float)v; }

template <class T>
__global__ __launch_bounds__(256) void k_read(const T* __restrict__ p, int64_t n, float* out) {
    float s = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) s += fold(p[i]);
    __shared__ float r[256];
    r[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = 0.f;
        for (int k = 0; k < 256; ++k) t += r[k];
        out[blockIdx.x] = t;
    }
}

// 16-B loads of a chunk-major gather pattern: lane i of a half-wave reads row (perm(i)) of a 32-row
// block, 4 floats, like the edge kernels' U/V gathers (rows scattered inside 1 KiB chunks)
__global__ __launch_bounds__(256) void k_gather16(const float4* __restrict__ p, int64_t nblk, float* out) {
    float s = 0.f;
    for (int64_t b = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5); b < nblk; b += (int64_t)gridDim.x * 8) {
        const int i = threadIdx.x & 31;
        const int row = (i * 7 + 3) & 31;
        for (int q = 0; q < 38; ++q) s += fold(p[b * 32 * 38 + q * 32 + row]);
    }
    __shared__ float r[256];
    r[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = 0.f;
        for (int k = 0; k < 256; ++k) t += r[k];
        out[blockIdx.x] = t;
    }
}

int main() {
    const int64_t bytes = 1ll << 30;
    void* buf;
    float* out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess) return 1;
    hipMemset(buf, 0, bytes);
    const int grid = 2048;
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_read<float4>, dim3(grid), dim3(256), 0, 0, (const float4*)buf, bytes / 16, out);
        hipLaunchKernelGGL(k_read<uint2>, dim3(grid), dim3(256), 0, 0, (const uint2*)buf, bytes / 8, out);
        hipLaunchKernelGGL(k_read<float>, dim3(grid), dim3(256), 0, 0, (const float*)buf, bytes / 4, out);
        hipLaunchKernelGGL(k_read<unsigned short>, dim3(grid), dim3(256), 0, 0, (const unsigned short*)buf, bytes / 2, out);
        hipLaunchKernelGGL(k_gather16, dim3(grid), dim3(256), 0, 0, (const float4*)buf, bytes / (32 * 38 * 16), out);
    }
    hipDeviceSynchronize();
    printf("read 1 GiB per kernel (gather: %lld B)\n", (long long)((bytes / (32 * 38 * 16)) * 32 * 38 * 16));
    return 0;
}
