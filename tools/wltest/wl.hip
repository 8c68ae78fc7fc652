#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
__device__ __forceinline__ uint32_t wimm(uint32_t val, int ln, uint32_t old) {
    uint32_t r;
    asm volatile("v_writelane_b32 %0, %1, %2" : "=v"(r) : "s"(val), "i"(ln), "0"(old));
    return r;
}
__device__ __forceinline__ uint32_t wsel(uint32_t val, int ln, uint32_t old) {
    return ((int)(threadIdx.x & 63) == ln) ? val : old;
}
template <bool IMM>
__global__ void k(const float* x, uint32_t* out) {
    const int lane = threadIdx.x;
    float v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = x[r * 64 + lane];
    uint32_t mw = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const uint64_t bal = __ballot(v[r] > 0.f);
        if (IMM) { mw = wimm((uint32_t)bal, r, mw); mw = wimm((uint32_t)(bal >> 32), 32 + r, mw); }
        else { mw = wsel((uint32_t)bal, r, mw); mw = wsel((uint32_t)(bal >> 32), 32 + r, mw); }
    }
    out[lane] = mw;
}
int main() {
    std::vector<float> hx(1024);
    for (int i = 0; i < 1024; ++i) hx[i] = ((i * 2654435761u) >> 7) % 3 == 0 ? 1.f : -1.f;
    float* dx; uint32_t* d1; uint32_t* d2;
    hipMalloc(&dx, 4096); hipMalloc(&d1, 256); hipMalloc(&d2, 256);
    hipMemcpy(dx, hx.data(), 4096, hipMemcpyHostToDevice);
    hipMemset(d1, 0, 256); hipMemset(d2, 0, 256);
    hipLaunchKernelGGL(k<true>, 1, 64, 0, 0, dx, d1);
    hipLaunchKernelGGL(k<false>, 1, 64, 0, 0, dx, d2);
    uint32_t a[64], b[64];
    hipMemcpy(a, d1, 256, hipMemcpyDeviceToHost); hipMemcpy(b, d2, 256, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l) if (a[l] != b[l]) { if (bad < 8) printf("lane %d imm %08x sel %08x\n", l, a[l], b[l]); ++bad; }
    printf("mismatches %d\n", bad);
    return 0;
}
