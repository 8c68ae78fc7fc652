// Device helpers shared by the gfx950 kernels of libspwgnn_hip.
//
// MFMA: v_mfma_f32_32x32x2_f32 (exact fp32, one rounding per product, fmaf-chain order).
//   A operand, lane l: A[i = l&31][k = l>>5];  B operand: B[k = l>>5][j = l&31]
//   C/D: 16 regs, reg r of lane l holds C[row = rho(r, l>>5)][col = l&31],
//        rho(r,h) = (r&3) + 8(r>>2) + 4h.
// Two orientations are used:
//   natural     rows (edges/nodes) on the A lanes, features on the C lanes — segment sums run
//               over the C registers;
//   transposed  features on the A lanes (weights), rows on the B/C lanes — an MLP chains layer to
//               layer in registers (C of layer n is the B operand of layer n+1, k-step = C reg).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "spwgnn_layout.h"

namespace spw {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
typedef float f32x4 __attribute__((ext_vector_type(4)));
// v_mfma_f32_16x16x4_f32: A lane l = A[l&15][k=l>>4], B lane l = B[k=l>>4][l&15];
// C reg r of lane l = C[row 4(l>>4) + r][col l&15].
__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ constexpr int rho(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// Start of a replayable training step (one thread): the optimizer step count moves on and the
// dropout key is derived for the new step — mode 0: key + 1 (the Keras front end's per-step seed
// counter); mode 1: splitmix64 chain of (seed, iteration, rank, micro 0), Trainer.run_config's key.
__device__ __forceinline__ uint64_t splitmix64_dev(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
__device__ __forceinline__ void step_advance_dev(uint64_t* key, int32_t* step, int mode, uint64_t seed, int32_t rank) {
    const int32_t it = *step;
    uint64_t k;
    if (mode == 0) {
        k = *key + 1ull;
    } else {
        k = splitmix64_dev(seed);
        k = splitmix64_dev(k ^ (uint64_t)(int64_t)it);
        k = splitmix64_dev(k ^ (uint64_t)(int64_t)rank);
        k = splitmix64_dev(k ^ 0ull);
    }
    *key = k;
    *step = it + 1;
}

// ---------------------------------------------------------------------------------------------
// Split-bf16 products ("x6" math). gfx950's bf16 MFMA runs 16× the f32 MFMA rate;
// an fp32 operand x is split (round-to-nearest at each stage) into x = h + m + l + O(2^-25·|x|)
// with h, m, l bf16, and x·y ≈ hh + hm + mh + mm + hl + lh (the dropped ml, lm, ll terms are
// O(2^-26)): six bf16 products with exact fp32 accumulation = fp32-class results at 6/16 of the
// f32 MFMA cost.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
    typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
    const bf2 r = {(__bf16)a, (__bf16)b};
    return __builtin_bit_cast(uint32_t, r);
}
__device__ __forceinline__ float bf16_lo(uint32_t p) { return __uint_as_float(p << 16); }
// Streaming loads (non-temporal: the lines are the caches' first victims) for arrays read once per
// launch beside gathered rows that are reused — the edge kernels' A rows and h2>0 words stream while
// the node rows U, V, G3 are gathered many times per tower (config 3's bf16 edge forward: 7.26 → 5.87
// GB of L2 misses per launch). SPWGNN_NO_NT (A/B builds): plain loads.
__device__ __forceinline__ uint2 ld_nt_u2(const void* p) {
#ifdef SPWGNN_NO_NT
    return *reinterpret_cast<const uint2*>(p);
#else
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 v = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p));
    return make_uint2(v[0], v[1]);
#endif
}
__device__ __forceinline__ float4 ld_nt_f4(const void* p) {
#ifdef SPWGNN_NO_NT
    return *reinterpret_cast<const float4*>(p);
#else
    const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
    return make_float4(v[0], v[1], v[2], v[3]);
#endif
}
__device__ __forceinline__ uint4 ld_nt_u4(const void* p) {
#ifdef SPWGNN_NO_NT
    return *reinterpret_cast<const uint4*>(p);
#else
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v[0], v[1], v[2], v[3]);
#endif
}
// 16 bytes of pinned, device-mapped HOST memory that the host rewrites between launches (a replayed
// step's upload slot): two system-scope relaxed atomic loads, which the compiler issues as global loads
// with the system-coherence cache bits — never a stale L2 line from an earlier read of the same slot,
// whether or not the allocation is fine-grained and whatever acquire the launch began with.
__device__ __forceinline__ uint4 ld_sys_u4(const uint4* p) {
    const uint64_t* q = reinterpret_cast<const uint64_t*>(p);
    const uint64_t lo = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t hi = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}
__device__ __forceinline__ uint32_t ld_nt_u1(const uint32_t* p) {
#ifdef SPWGNN_NO_NT
    return *p;
#else
    return __builtin_nontemporal_load(p);
#endif
}
// x rounded to bf16 (RNE), as an fp32 value
__device__ __forceinline__ float bf16_round(float x) { return __uint_as_float(pk_bf16(x, 0.f) << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t p) { return __uint_as_float(p & 0xffff0000u); }
// (a, b) → three packed bf16 pairs h, m, l (element 0 = a in the low half)
// bf16_lo of h and m as a v_perm_b32: written as a shift, the compiler rebuilds it as a second
// v_cvt_pk_bf16_f32 of `a` alone plus the shift (13 VALU per pair instead of 11); an empty asm
// barrier on h and m also prevents that but costs a hazard s_nop per barrier.
__device__ __forceinline__ float bf16_lo_perm(uint32_t p) {
    return __uint_as_float(__builtin_amdgcn_perm(p, p, 0x01000C0Cu));   // bytes [0, 0, p0, p1]
}
__device__ __forceinline__ void split2(float a, float b, uint32_t& h, uint32_t& m, uint32_t& l) {
    h = pk_bf16(a, b);
    const float ra = a - bf16_lo_perm(h), rb = b - bf16_hi(h);
    m = pk_bf16(ra, rb);
    l = pk_bf16(ra - bf16_lo_perm(m), rb - bf16_hi(m));
}
__device__ __forceinline__ bf16x8 as_bf16x8(i16x4 lo, i16x4 hi) {
    const i16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, v);
}
__device__ __forceinline__ bf16x8 as_bf16x8(uint4 v) { return __builtin_bit_cast(bf16x8, v); }
// acc += a·b over the six split products (a[p], b[p]: parts h, m, l); small terms first.
// NP = 1 is the bf16 math (SPWGNN_MATH_BF16): the h parts alone, one product.
template <int NP = 3>
__device__ __forceinline__ f32x4 mfma16_x6(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x4 c) {
    if constexpr (NP == 1) return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], c, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], c, 0, 0, 0);
}
template <int NP = 3>
__device__ __forceinline__ f32x16 mfma32_x6(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x16 c) {
    if constexpr (NP == 1) return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], c, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], c, 0, 0, 0);
}
// The six products of NT output tiles interleaved (product p for every tile before product p+1):
// consecutive MFMAs write different accumulators, which the matrix pipe overlaps better than one
// tile's chain of six (measured, tools/mb/x6dep.hip: 0.77 -> 0.80 of the bf16 peak at two waves per
// SIMD with LDS-fed fragments). Same products and per-accumulator order as mfma32_x6: bit-identical.
template <int NP, int NT>
__device__ __forceinline__ void mfma32_x6_group(const bf16x8 (&a)[3], const bf16x8 (&b)[NT][3], f32x16* acc) {
    if constexpr (NP == 1) {
#pragma unroll
        for (int u = 0; u < NT; ++u) acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[u][0], acc[u], 0, 0, 0);
    } else {
        constexpr int pa[6] = {2, 0, 1, 1, 0, 0}, pb[6] = {0, 2, 1, 0, 1, 0};
#pragma unroll
        for (int p = 0; p < 6; ++p)
#pragma unroll
            for (int u = 0; u < NT; ++u)
                acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[pa[p]], b[u][pb[p]], acc[u], 0, 0, 0);
    }
}
// ds_read_b64_tr_b16: lane 4q+p of each 16-lane group addresses row q, 16-bit columns 4p..4p+3 of a
// 4×16 block; lane i of the group receives column i of the 4 rows (row q in element q)
__device__ __forceinline__ i16x4 lds_tr16(const char* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(p));
}

__device__ __forceinline__ f32x16 zero16() {
    f32x16 z;
#pragma unroll
    for (int i = 0; i < 16; ++i) z[i] = 0.f;
    return z;
}

// Orders this wave's LDS writes before its later LDS reads (single wavefront, no WG barrier:
// waves of a workgroup run independent tiles).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float relu(float x) { return x > 0.f ? x : 0.f; }
// relu(x) on a real edge (cap = +inf), 0 on a padding edge (cap = 0): one v_med3_f32 where
// relu(x) · valid was a v_max_f32 and a v_mul_f32 (the same values)
__device__ __forceinline__ float relu_valid(float x, float cap) { return __builtin_amdgcn_fmed3f(x, 0.f, cap); }
// g if bit f of bits is set, else +0: a sign-extended one-bit field as an AND mask (v_bfe_i32 +
// v_and_b32; written as a select the compiler emits and + compare + cndmask)
__device__ __forceinline__ float mask_bit(float g, uint32_t bits, int f) {
    return __uint_as_float(__float_as_uint(g) & (uint32_t)__builtin_amdgcn_sbfe((int)bits, f, 1));
}
// tanh in fp32 for the split-bf16 node kernels, ≤ 1 ulp below |x| = 0.625 and ≤ 2 ulp above (libm
// tanhf: ≤ 1). Above 0.625: 1 − 2/(2^(2x·log2 e) + 1) on the transcendental unit (v_exp_f32,
// v_rcp_f32), exact in the limits (±1 at ±∞, NaN propagates). Below: x + x³·p(x²), p a degree-4 fit of
// (tanh x − x)/x³ on [0, 0.625] (max 0.72 ulp in fp32) — the exp form cancels there (1 − 0.999…) and
// loses up to 4·10⁵ ulp of relative accuracy near 0, which bf16 math then rounds into its operands
// (it was the engine's offset from the bf16 emulator). 14 VALU instead of libm's ≈ 22.
__device__ __forceinline__ float acc_tanh(float x) {
    const float u = x * x;
    float p = __builtin_fmaf(-0.005700227044831583f, u, 0.020631621187850974f);
    p = __builtin_fmaf(p, u, -0.053736200685166706f);
    p = __builtin_fmaf(p, u, 0.13331381511777754f);
    p = __builtin_fmaf(p, u, -0.333332788328783f);
    const float small = __builtin_fmaf(x * u, p, x);
    const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);
    const float big = __builtin_fmaf(-2.f, __builtin_amdgcn_rcpf(e + 1.f), 1.f);
#ifdef SPWGNN_TANH_EXP_ONLY   // diagnosis A/B: the exp form everywhere (rounds 1-4's fast_tanh)
    return big + 0.f * small;
#else
    return __builtin_fabsf(x) < 0.625f ? small : big;
#endif
}
// The 2-input first Dense of the encoders with one explicit rounding order: left to the compiler,
// unrolled copies of x0·w0 + x1·w1 + b were contracted / paired differently, so an edge's value
// depended on which copy (column tile) processed it.
__device__ __forceinline__ float dense2(float x0, float x1, float w0, float w1, float b) {
    return __builtin_fmaf(x1, w1, __builtin_fmaf(x0, w0, b));
}

// Put a wave-uniform 32-bit value into lane `ln` of `old` (v_cmp + v_cndmask; no exec branch).
__device__ __forceinline__ uint32_t writelane(uint32_t val, int ln, uint32_t old) {
    return ((int)(threadIdx.x & 63) == ln) ? val : old;
}
// v_writelane_b32 with a compile-time lane (ln must fold to a constant after unrolling; a uniform
// SGPR value goes straight into one lane: 1 VALU instead of a compare + select). The compiler does
// not see the SGPR read inside the asm: a v_cmp writing the SGPR right before it is read stale
// without a wait state (measured on gfx950: tools/wltest), hence the s_nop.
__device__ __forceinline__ uint32_t writelane_imm(uint32_t val, int ln, uint32_t old) {
    uint32_t r;
    asm volatile("s_nop 1\n\tv_writelane_b32 %0, %1, %2" : "=v"(r) : "s"(val), "i"(ln), "0"(old));
    return r;
}

// The same without the wait state, for batches: every SGPR it reads must have been written several
// instructions earlier (a group of ballots, a sched_barrier, then the group's writelanes).
// Eight of them into one register in one statement: the compiler pads each inline asm with a
// hazard s_nop; one pad per eight writelanes instead of one per writelane.
__device__ __forceinline__ uint32_t writelane8_batched(uint32_t old, const uint32_t (&v)[8], const int (&ln)[8]) {
    asm volatile(
        "v_writelane_b32 %0, %1, %9\n\tv_writelane_b32 %0, %2, %10\n\t"
        "v_writelane_b32 %0, %3, %11\n\tv_writelane_b32 %0, %4, %12\n\t"
        "v_writelane_b32 %0, %5, %13\n\tv_writelane_b32 %0, %6, %14\n\t"
        "v_writelane_b32 %0, %7, %15\n\tv_writelane_b32 %0, %8, %16"
        : "+v"(old)
        : "s"(v[0]), "s"(v[1]), "s"(v[2]), "s"(v[3]), "s"(v[4]), "s"(v[5]), "s"(v[6]), "s"(v[7]),
          "i"(ln[0]), "i"(ln[1]), "i"(ln[2]), "i"(ln[3]), "i"(ln[4]), "i"(ln[5]), "i"(ln[6]), "i"(ln[7]));
    return old;
}
__device__ __forceinline__ uint32_t writelane_imm_batched(uint32_t val, int ln, uint32_t old) {
    uint32_t r;
    asm volatile("v_writelane_b32 %0, %1, %2" : "=v"(r) : "s"(val), "i"(ln), "0"(old));
    return r;
}

// ---------------------------------------------------------------------------------------------
// Dropout key (our own counter-based RNG; Keras' TF draws cannot be reproduced — DESIGN.md §6).
// keep(seed, kind, tower, a, b, feature) = mix(...) >= rate·2^32.  Restated bit-exactly in
// tests (oracle helper) to build the oracle's multiplicative masks.
__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}
__host__ __device__ __forceinline__ uint32_t drop_row_key(uint64_t seed, uint32_t kind, uint32_t tower,
                                                          uint32_t a, uint32_t b) {
    uint32_t h = mix32((uint32_t)seed ^ mix32((uint32_t)(seed >> 32) + kind));
    h = mix32(h ^ tower);
    h = mix32(h ^ ((a << 16) | (b & 0xffffu)));
    return h;
}
__host__ __device__ __forceinline__ bool drop_keep(uint32_t rowkey, uint32_t feature, uint32_t thresh) {
    return mix32(rowkey ^ feature) >= thresh;
}

// ---------------------------------------------------------------------------------------------
// Packed (zero-padded) weight copies built by k_prep at the start of every call.
enum PackId : int {
    PK_RM1 = 0, PK_RM2, PK_RM3, PK_W1A,       // [160][160] [in][out]
    PK_OM1,                                    // [128][128]
    PK_W1B, PK_W1C,                            // [128][160] [P feature][U/V feature]
    PK_W2,                                     // [160][160] rmp.1 [in][out]
    PK_W3A,                                    // [160][128] rmp.2 rows 0..149, row 150 = rmp.2 bias
    PK_WO1C, PK_WO1A, PK_WO1P,                 // [128][128] omp.0 rows 0-99 / 100-199 / 200-299
    PK_WO2,                                    // [128][128] omp.1 with permuted columns (x' order)
    PK_W2T,                                    // [160][160] W2T[k][j] = W2[j][k]
    PK_W1BT, PK_W1CT,                          // [160][128] W1bT[k][p] = W1b[p][k]
    PK_WO2T,                                   // [128][128] Wo2pT[k][i] = Wo2p[i][k]
    PK_WO1CT, PK_WO1AT, PK_WO1PT,              // [128][128] Wo1T_p[k][i] = Wo1[off_p+i][k]
    PK_W3T,                                    // [128][160] W3T[k][i] = W3[i][k]
    PK_W1AT, PK_RM3T, PK_RM2T, PK_RM1T,        // [160][160] transposes
    PK_OM1T,                                   // [128][128]
    // biases, padded vectors
    PB_RM1, PB_RM2, PB_RM3, PB_W1A, PB_W2,     // [160]
    PB_OM1, PB_O1, PB_O2P,                     // [128]  (PB_O2P permuted like PK_WO2)
    PK_RM0,                                    // [2][160] rm.0 kernel
    PK_OM0,                                    // [2][128] om.0 kernel
    PB_RM0, PB_OM0,                            // [160], [128]
    PK_COUNT
};

struct PackSlots {
    int64_t off[PK_COUNT];
    int64_t total;
};

__host__ __device__ inline int pack_rows(int id) {
    switch (id) {
        case PK_RM1: case PK_RM2: case PK_RM3: case PK_W1A: case PK_W2: case PK_W2T:
        case PK_W1AT: case PK_RM3T: case PK_RM2T: case PK_RM1T: case PK_W3A: case PK_W1BT: case PK_W1CT:
            return 160;
        case PB_RM1: case PB_RM2: case PB_RM3: case PB_W1A: case PB_W2: case PB_OM1: case PB_O1: case PB_O2P:
        case PB_RM0: case PB_OM0:
            return 1;
        case PK_RM0: case PK_OM0:
            return 2;
        default:
            return 128;
    }
}
__host__ __device__ inline int pack_cols(int id) {
    switch (id) {
        case PK_RM1: case PK_RM2: case PK_RM3: case PK_W1A: case PK_W2: case PK_W2T:
        case PK_W1AT: case PK_RM3T: case PK_RM2T: case PK_RM1T: case PK_W1B: case PK_W1C: case PK_W3T:
        case PB_RM1: case PB_RM2: case PB_RM3: case PB_W1A: case PB_W2:
        case PK_RM0: case PB_RM0:
            return 160;
        default:
            return 128;
    }
}

// x' (permuted omp.1 output) column f' ↔ Keras column: state f' < 100 ↔ col f'+1, logit ↔ col 0.
__host__ __device__ __forceinline__ int wo2_perm(int fp) { return fp < 100 ? fp + 1 : (fp == 100 ? 0 : -1); }

}  // namespace spw
