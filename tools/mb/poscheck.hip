// Does v_mfma_f32_32x32x16_bf16 give bit-identical results for identical B columns / A rows?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cstdlib>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
__global__ void k(const uint16_t* A, const uint16_t* B, const float* C0, float* D, int mode) {
    const int l = threadIdx.x, i = l & 31, h = l >> 5;
    bf16x8 a, b;
    for (int e = 0; e < 8; ++e) {
        uint16_t av = mode == 0 ? A[i * 16 + 8 * h + e] : A[0 * 16 + 8 * h + e];       // mode1: all rows = row 0
        uint16_t bv = mode == 0 ? B[(8 * h + e) * 32 + 0] : B[(8 * h + e) * 32 + i];   // mode0: all cols = col 0
        a[e] = __builtin_bit_cast(__bf16, av);
        b[e] = __builtin_bit_cast(__bf16, bv);
    }
    f32x16 c;
    for (int r = 0; r < 16; ++r) c[r] = C0[r];
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    for (int r = 0; r < 16; ++r) D[l * 16 + r] = c[r];
}
int main() {
    uint16_t hA[32 * 16], hB[16 * 32];
    float hC[16], hD[64 * 16];
    srand(3);
    int bad0 = 0, bad1 = 0;
    uint16_t *dA, *dB; float *dC, *dD;
    hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dC, sizeof hC); hipMalloc(&dD, sizeof hD);
    for (int trial = 0; trial < 200; ++trial) {
        for (auto& v : hA) { float f = ((rand() & 0xffff) / 65536.f - 0.5f) * (1 << (rand() % 20)) ; uint32_t u; memcpy(&u, &f, 4); v = u >> 16; }
        for (auto& v : hB) { float f = ((rand() & 0xffff) / 65536.f - 0.5f) * (1 << (rand() % 20)); uint32_t u; memcpy(&u, &f, 4); v = u >> 16; }
        for (auto& v : hC) v = ((rand() & 0xffff) / 65536.f - 0.5f) * 1000.f;
        hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice); hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
        hipMemcpy(dC, hC, sizeof hC, hipMemcpyHostToDevice);
        for (int mode = 0; mode < 2; ++mode) {
            hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD, mode);
            hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
            // D of lane l reg r: row rho(r, l>>5), col l&31
            if (mode == 0) {  // identical columns: compare each (row) across cols
                for (int l = 0; l < 64; ++l) for (int r = 0; r < 16; ++r) {
                    float ref = hD[(l & 32) * 16 + r];   // col 0 of the same half
                    if (memcmp(&ref, &hD[l * 16 + r], 4)) ++bad0;
                }
            } else {  // identical rows (row 0 everywhere): compare across rows within a column
                for (int l = 0; l < 64; ++l) for (int r = 0; r < 16; ++r) {
                    float ref = hD[(l & 31) * 16 + 0];  // row rho(0,0)=0 of col l&31
                    // C differs per row r (C0[r]) → only compare rows with equal C: none; skip
                    (void)ref;
                }
            }
        }
    }
    printf("column-position mismatches: %d\n", bad0);
    return 0;
}
