// Does column j of v_mfma_f32_32x32x16_bf16 depend on the OTHER columns of B (or rows of A)?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cstdlib>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
__global__ void k(const uint16_t* A, const uint16_t* B, const float* C, float* D, int use16) {
    const int l = threadIdx.x, i = l & 31, h = l >> 5;
    bf16x8 a, b;
    for (int e = 0; e < 8; ++e) {
        a[e] = __builtin_bit_cast(__bf16, A[i * 16 + 8 * h + e]);
        b[e] = __builtin_bit_cast(__bf16, B[(8 * h + e) * 32 + i]);
    }
    f32x16 c;
    for (int r = 0; r < 16; ++r) c[r] = C[l * 16 + r];
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    for (int r = 0; r < 16; ++r) D[l * 16 + r] = c[r];
}
static uint16_t rb(int sc) { float f = ((rand() & 0xffff) / 65536.f - 0.5f) * (float)(1 << (rand() % sc)); uint32_t u; memcpy(&u, &f, 4); return u >> 16; }
int main() {
    uint16_t hA[32 * 16], hB[16 * 32];
    float hC[64 * 16], hD[64 * 16], ref[64 * 16];
    uint16_t *dA, *dB; float *dC, *dD;
    hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dC, sizeof hC); hipMalloc(&dD, sizeof hD);
    srand(5);
    int badcol = 0, badrow = 0, trials = 0;
    for (int base = 0; base < 50; ++base) {
        for (auto& v : hA) v = rb(24);
        for (auto& v : hB) v = rb(24);
        for (auto& v : hC) v = ((rand() & 0xffff) / 65536.f - 0.5f) * 100.f;
        auto run = [&](float* out) {
            hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice); hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
            hipMemcpy(dC, hC, sizeof hC, hipMemcpyHostToDevice);
            hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD, 0);
            hipMemcpy(out, dD, sizeof hD, hipMemcpyDeviceToHost);
        };
        run(ref);
        for (int v = 0; v < 20; ++v) {
            // perturb every B column except column 0 and every A row except row 0
            for (int k = 0; k < 16; ++k) for (int j = 1; j < 32; ++j) hB[k * 32 + j] = rb(24);
            for (int i = 1; i < 32; ++i) for (int k = 0; k < 16; ++k) hA[i * 16 + k] = rb(24);
            run(hD);
            ++trials;
            // column 0 = lanes 0 and 32 (all regs); row 0 = reg 0 of lanes 0..31
            for (int l : {0, 32}) for (int r = 0; r < 16; ++r) if (memcmp(&ref[l * 16 + r], &hD[l * 16 + r], 4)) ++badcol;
            for (int l = 0; l < 32; ++l) if (memcmp(&ref[l * 16], &hD[l * 16], 4)) ++badrow;
        }
    }
    printf("trials %d: column-0 changes %d, row-0 changes %d\n", trials, badcol, badrow);
    return 0;
}
