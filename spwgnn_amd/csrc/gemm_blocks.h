// Register-level MFMA building blocks (fp32, v_mfma_f32_32x32x2_f32) used by every kernel.
#pragma once
#include <type_traits>
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

// ---- chunk-major block rows (transposed orientation, lane (j, h) = row j of the 32-row block):
// regs 4q..4q+3 of tile t are features f0 = 32t + 8q + 4h .. +3, one 16-byte piece; NT = 5 tiles
// ↔ 152-feature blocks (KH 76), NT = 4 ↔ 104-feature blocks (KH 52).
template <int NT>
__device__ __forceinline__ void store_cm(float* __restrict__ blk, const f32x16 (&X)[NT], int lane, bool valid) {
    constexpr int KH = NT == 5 ? kKhE : kKhN;
    const int j = lane & 31, h = lane >> 5;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int f0 = 32 * t + 8 * q + 4 * h;
            if (32 * t + 8 * q + 4 < 2 * KH) {   // f0 < 2·KH on both halves
                float4 v = valid ? make_float4(X[t][4 * q], X[t][4 * q + 1], X[t][4 * q + 2], X[t][4 * q + 3])
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
                *reinterpret_cast<float4*>(blk + cm_offk<KH>(j, f0)) = v;
            }
        }
}
// one 16-byte piece p = 4t + q of store_cm (pieces with f0 ≥ 2·KH do not exist: NT = 5 has 19,
// NT = 4 has 13 — exactly the group count of a chain whose input is X)
template <int NT>
__device__ __forceinline__ void store_cm_piece(float* __restrict__ blk, const f32x16 (&X)[NT], int lane, int p) {
    constexpr int KH = NT == 5 ? kKhE : kKhN;
    const int j = lane & 31, h = lane >> 5, t = p >> 2, q = p & 3;
    if (32 * t + 8 * q + 4 < 2 * KH)
        *reinterpret_cast<float4*>(blk + cm_offk<KH>(j, 32 * t + 8 * q + 4 * h)) =
            make_float4(X[t][4 * q], X[t][4 * q + 1], X[t][4 * q + 2], X[t][4 * q + 3]);
}
template <int NT>
__device__ __forceinline__ void load_cm(const float* __restrict__ blk, f32x16 (&X)[NT], int lane) {
    constexpr int KH = NT == 5 ? kKhE : kKhN;
    const int j = lane & 31, h = lane >> 5;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int f0 = 32 * t + 8 * q + 4 * h;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (32 * t + 8 * q + 4 < 2 * KH) v = *reinterpret_cast<const float4*>(blk + cm_offk<KH>(j, f0));
            X[t][4 * q] = v.x;
            X[t][4 * q + 1] = v.y;
            X[t][4 * q + 2] = v.z;
            X[t][4 * q + 3] = v.w;
        }
}
// ---- bf16 storage (bf16 math): an array that only ever feeds MFMA operands is stored
// as bf16 with the element index of its fp32 layout (a 16-byte float4 piece becomes an 8-byte uint2
// at the same element offset). The bf16 math rounds every operand to bf16 (RNE) anyway, so storing
// the rounded value is exact: the products see the same bits.
__device__ __forceinline__ uint2 pack4_bf16(float4 v) { return make_uint2(pk_bf16(v.x, v.y), pk_bf16(v.z, v.w)); }
__device__ __forceinline__ float4 unpack4_bf16(uint2 u) {
    return make_float4(bf16_lo(u.x), bf16_hi(u.x), bf16_lo(u.y), bf16_hi(u.y));
}
template <int NT>
__device__ __forceinline__ void store_cm_b16(uint16_t* __restrict__ blk, const f32x16 (&X)[NT], int lane, bool valid) {
    constexpr int KH = NT == 5 ? kKhE : kKhN;
    const int j = lane & 31, h = lane >> 5;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int f0 = 32 * t + 8 * q + 4 * h;
            if (32 * t + 8 * q + 4 < 2 * KH) {
                const float4 v = valid ? make_float4(X[t][4 * q], X[t][4 * q + 1], X[t][4 * q + 2], X[t][4 * q + 3])
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
                *reinterpret_cast<uint2*>(blk + cm_offk<KH>(j, f0)) = pack4_bf16(v);
            }
        }
}

template <int NT>
__device__ __forceinline__ void load_cm_b16(const uint16_t* __restrict__ blk, f32x16 (&X)[NT], int lane) {
    constexpr int KH = NT == 5 ? kKhE : kKhN;
    const int j = lane & 31, h = lane >> 5;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int f0 = 32 * t + 8 * q + 4 * h;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (32 * t + 8 * q + 4 < 2 * KH) v = unpack4_bf16(*reinterpret_cast<const uint2*>(blk + cm_offk<KH>(j, f0)));
            X[t][4 * q] = v.x;
            X[t][4 * q + 1] = v.y;
            X[t][4 * q + 2] = v.z;
            X[t][4 * q + 3] = v.w;
        }
}
// ---- U = P·W1b and V = P·W1c in bf16 math (training): rounded to bf16 once where
// they are stored, like A (§3g) — h1 = relu(A + U[s] + V[r]) adds three bf16 values in fp32 — and
// stored as bf16 (half the bytes of the edge forward's gathers) where every reader is a wide kernel.
enum : int { kUvF32 = 0, kUvRound = 1, kUvB16 = 2 };
template <int NT>
__device__ __forceinline__ void store_cm_uv(float* base, int64_t off, f32x16 (&X)[NT], int lane, bool valid, int uv16) {
    if (uv16 == kUvB16) {
        store_cm_b16<NT>(reinterpret_cast<uint16_t*>(base) + off, X, lane, valid);   // element index of fp32
        return;
    }
    if (uv16 == kUvRound)   // X is rounded in place
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) X[t][r] = bf16_round(X[t][r]);
    store_cm<NT>(base + off, X, lane, valid);
}
// the team kernels' form (fp32 storage only): one output tile, rounded in place when uv16 asks
__device__ __forceinline__ void round_uv_tile(f32x16& X, int uv16) {
    if (uv16 == kUvRound)
#pragma unroll
        for (int r = 0; r < 16; ++r) X[r] = bf16_round(X[r]);
}
__device__ __forceinline__ float4 unpack_uv(float4 v) { return v; }
__device__ __forceinline__ float4 unpack_uv(uint2 v) { return unpack4_bf16(v); }

// one element of a bf16-stored array (RNE; the element index of the fp32 layout)
__device__ __forceinline__ void store_b16(float* base, int64_t idx, float v) {
    reinterpret_cast<uint16_t*>(base)[idx] = (uint16_t)(pk_bf16(v, 0.f) & 0xffffu);
}

// ---- h2 > 0 bits (mask2) of one 32-edge block: kM2Blk words, [edge][8]; word t < 5 holds the bits
// of features 32t .. 32t+31 (bit = feature within the tile), words 5..7 are zero padding — an edge's
// five words are one 16-byte + one 4-byte load.
constexpr int kM2Blk = 256;
__device__ __forceinline__ void load_m2(const uint32_t* __restrict__ blk_words, int edge, uint32_t (&w)[5]) {
    const uint32_t* p = blk_words + edge * 8;
    const uint4 v = ld_nt_u4(p);   // streamed: each step's words are read once per kernel
    w[0] = v.x;
    w[1] = v.y;
    w[2] = v.z;
    w[3] = v.w;
    w[4] = ld_nt_u1(p + 4);
}
// writer side: word (edge, t) lives in register (8·edge + t) >> 6, lane (8·edge + t) & 63 of the
// four-register image that k_edge_fwd stores with one full-wave store per register
__host__ __device__ __forceinline__ constexpr int m2_pos(int edge, int t) { return 8 * edge + t; }

// split-halves chunk of a chunk-major row: x[s] = feature KH·h + s of row j
template <int KH>
__device__ __forceinline__ void load_half_cm(const float* __restrict__ blk, int lane, float (&x)[KH]) {
    const float* p = blk + ((lane >> 5) * 32 + (lane & 31)) * 4;
#pragma unroll
    for (int q = 0; q < KH / 4; ++q) {
        const float4 v = *reinterpret_cast<const float4*>(p + 256 * q);
        x[4 * q] = v.x;
        x[4 * q + 1] = v.y;
        x[4 * q + 2] = v.z;
        x[4 * q + 3] = v.w;
    }
}
// feature f of row `row` in a chunk-major array (block size KH·64 floats)
template <int KH>
__device__ __forceinline__ int64_t cm_index(int64_t row, int f) {
    return (row >> 5) * (KH * 64) + cm_offk<KH>((int)(row & 31), f);
}

// ---- per-lane activation-sign bits of NT C-layout tiles (bit 16t + r of the lane's words), so a
// backward pass in the same orientation reads 3 words per lane instead of the activations.
// X must be ≥ +0 (post-relu): then X > 0 ⟺ its bit pattern is non-zero, min(bits, 1) is the bit.
// Two VALU per bit, no compare: bits(X) + 0x7fffffff has bit 31 set ⟺ bits(X) ≠ 0, and
// v_alignbit_b32(w, b, 31) = (w << 1) | (b >> 31) shifts it in (a word's bits walked from the top
// index down). Written as a compare, the compiler emits v_cmp + s_nop + v_cndmask + v_or per bit.
template <int NT>
__device__ __forceinline__ void store_pos_bits(uint32_t* __restrict__ words, const f32x16 (&X)[NT], int lane) {
    constexpr int NB = NT * 16;
#pragma unroll
    for (int k = 0; k < (NB + 31) / 32; ++k) {
        uint32_t w = 0u;
#pragma unroll
        for (int idx = (32 * k + 31 < NB ? 32 * k + 31 : NB - 1); idx >= 32 * k; --idx)
            w = __builtin_amdgcn_alignbit(w, __float_as_uint(X[idx >> 4][idx & 15]) + 0x7fffffffu, 31);
        words[64 * k + lane] = w;
    }
}
template <int NT>
__device__ __forceinline__ void apply_pos_bits(const uint32_t* __restrict__ words, f32x16 (&X)[NT], int lane, float scale) {
    uint32_t w[(NT * 16 + 31) / 32];
#pragma unroll
    for (int k = 0; k < (NT * 16 + 31) / 32; ++k) w[k] = words[64 * k + lane];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r)
            X[t][r] = mask_bit(X[t][r] * scale, w[(16 * t + r) >> 5], (16 * t + r) & 31);
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

// ---- transposed orientation: out[t] += Wᵀ·in with the [K][N] weight as a k4-blocked image
// W4[((k>>2)·N + col)·4 + (k&3)] (built by k_prep). The A operand of lane (i, h) at
// k-step kk of input tile tp is W[rho(kk,h) + 32tp][32t + i]; k-steps 4g..4g+3 are the 4
// consecutive features 8g + 4h + 0..3 — one 16-byte load per tile per 4 MFMAs, and the 32 lanes
// of a half read 512 contiguous bytes. (One dword load per MFMA caps the matrix pipe near 50 %;
// tools/mb/chain.hip.) The next group's fragments load while this group's MFMAs issue.
// in: C layout of the previous layer; k-steps (tp, r) for tp < NT_IN, r < LAST_R in the last
// input tile (LAST_R % 4 == 0; rows beyond are zero padding).
// `side(gi)` runs after group gi's MFMAs: independent work (e.g. the previous layer's stores,
// store_cm_piece) issued beside the matrix pipe instead of before the chain.
struct NoSide {
    __device__ __forceinline__ void operator()(int) const {}
};
template <int NT_OUT, int NT_IN, int LAST_R, int N, class Side = NoSide>
__device__ __forceinline__ void tchain_acc(const f32x16 (&in)[NT_IN], f32x16 (&out)[NT_OUT],
                                           const float* __restrict__ W4, int lane, Side side = Side()) {
    static_assert(LAST_R % 4 == 0, "16-byte fragments");
    const float* wb = W4 + ((lane >> 5) * N + (lane & 31)) * 4;   // k-block h, column i
    constexpr int NG = (NT_IN - 1) * 4 + LAST_R / 4;   // groups of 4 k-steps: k-block 2gi + h
    float4 cur[NT_OUT], nxt[NT_OUT];
#pragma unroll
    for (int t = 0; t < NT_OUT; ++t) cur[t] = *reinterpret_cast<const float4*>(wb + 128 * t);
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
        if (gi + 1 < NG) {
#pragma unroll
            for (int t = 0; t < NT_OUT; ++t) nxt[t] = *reinterpret_cast<const float4*>(wb + 8 * N * (gi + 1) + 128 * t);
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of this group's MFMAs
        const int tp = gi >> 2, r0 = 4 * (gi & 3);
#pragma unroll
        for (int t = 0; t < NT_OUT; ++t) {
            out[t] = mfma32(cur[t].x, in[tp][r0], out[t]);
            out[t] = mfma32(cur[t].y, in[tp][r0 + 1], out[t]);
            out[t] = mfma32(cur[t].z, in[tp][r0 + 2], out[t]);
            out[t] = mfma32(cur[t].w, in[tp][r0 + 3], out[t]);
        }
        side(gi);
        if (gi + 1 < NG) {
#pragma unroll
            for (int t = 0; t < NT_OUT; ++t) cur[t] = nxt[t];
        }
    }
}

// ---- transposed orientation, B operand from a split-halves row chunk x (features KH*h + s),
// k4-blocked weight: k-steps 4q..4q+3 of half h are k-block KH/4·h + q.
template <int NT_OUT, int KH, int N>
__device__ __forceinline__ void tgemm_half_acc(const float (&x)[KH], f32x16 (&out)[NT_OUT],
                                               const float* __restrict__ W4, int lane) {
    static_assert(KH % 4 == 0, "16-byte fragments");
    const float* wb = W4 + ((KH / 4) * (lane >> 5) * N + (lane & 31)) * 4;
    float4 cur[NT_OUT], nxt[NT_OUT];
#pragma unroll
    for (int t = 0; t < NT_OUT; ++t) cur[t] = *reinterpret_cast<const float4*>(wb + 128 * t);
#pragma unroll
    for (int q = 0; q < KH / 4; ++q) {
        if (q + 1 < KH / 4) {
#pragma unroll
            for (int t = 0; t < NT_OUT; ++t) nxt[t] = *reinterpret_cast<const float4*>(wb + 4 * N * (q + 1) + 128 * t);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < NT_OUT; ++t) {
            out[t] = mfma32(cur[t].x, x[4 * q], out[t]);
            out[t] = mfma32(cur[t].y, x[4 * q + 1], out[t]);
            out[t] = mfma32(cur[t].z, x[4 * q + 2], out[t]);
            out[t] = mfma32(cur[t].w, x[4 * q + 3], out[t]);
        }
        if (q + 1 < KH / 4) {
#pragma unroll
            for (int t = 0; t < NT_OUT; ++t) cur[t] = nxt[t];
        }
    }
}

// ---- transposed orientation, B operand streamed from a split-halves global row (features
// KH*h + s, 16 bytes at a time), k4-blocked weight. Rolled loop (bounded registers).
// XS = float4 stride between consecutive 4-feature chunks of the row: 1 for row-major rows,
// 64 for chunk-major blocks (row_khh then points at the lane's (h, j) piece of chunk 0).
template <int NT_OUT, int KH, int N, int XS = 1>
__device__ __forceinline__ void tgemm_stream_acc(const float* __restrict__ row_khh, f32x16 (&out)[NT_OUT],
                                                 const float* __restrict__ W4, int lane) {
    static_assert(KH % 4 == 0, "16-byte fragments");
    const float4* x4 = reinterpret_cast<const float4*>(row_khh);
    const float* wb = W4 + ((KH / 4) * (lane >> 5) * N + (lane & 31)) * 4;
    static_assert((KH / 4) % 2 == 1, "ring schedule below: odd chunk count");
    float4 w0[NT_OUT], w1[NT_OUT];
    float4 x0 = x4[0], x1;  // chunk q at x4[XS·q]
#pragma unroll
    for (int t = 0; t < NT_OUT; ++t) w0[t] = *reinterpret_cast<const float4*>(wb + 128 * t);
    // two register slots with static names (loop unrolled by 2): the prefetch of chunk q+1 is
    // never copied, so the wait before chunk q covers chunk q's loads only
    auto chunk = [&](int q, const float4 (&cw)[NT_OUT], const float4& cx, float4 (&nw)[NT_OUT], float4& nx) {
        const int qn = min(q + 1, KH / 4 - 1);   // unconditional (clamped) prefetch
#pragma unroll
        for (int t = 0; t < NT_OUT; ++t) nw[t] = *reinterpret_cast<const float4*>(wb + 4 * N * qn + 128 * t);
        nx = x4[XS * qn];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < NT_OUT; ++t) {
            out[t] = mfma32(cw[t].x, cx.x, out[t]);
            out[t] = mfma32(cw[t].y, cx.y, out[t]);
            out[t] = mfma32(cw[t].z, cx.z, out[t]);
            out[t] = mfma32(cw[t].w, cx.w, out[t]);
        }
    };
#pragma unroll 1
    for (int q = 0; q + 1 < KH / 4; q += 2) {
        chunk(q, w0, x0, w1, x1);
        chunk(q + 1, w1, x1, w0, x0);
    }
    chunk(KH / 4 - 1, w0, x0, w1, x1);
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
// The x6 W2 / W2ᵀ LDS images (50 steps × 3 parts × 64 lanes uint4 = 150 KB) reach past ds_read's
// 16-bit byte offset. Fragment idx (uint4 units, lane included in the base) is read from one of three
// bases 64 KB apart, each in its own register: the opaque offsets keep the compiler from rebuilding
// every address beyond 64 KB with a v_or (≈ 10 VALU per k-block).
struct WlBases {
    const uint4* b[3];
    __device__ __forceinline__ explicit WlBases(const uint4* wlp) {
        int o1 = 4096, o2 = 8192;
        asm("" : "+v"(o1));
        asm("" : "+v"(o2));
        b[0] = wlp;
        b[1] = wlp + o1;
        b[2] = wlp + o2;
    }
    __device__ __forceinline__ uint4 at(int idx) const { return b[idx >> 12][idx & 4095]; }
};
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

constexpr int kX6Ring = 3;
// SPWGNN_PAD_DBG (diagnosis builds, wrong results): 1 skips the MFMAs of the last output tile of every
// 4-tile (100-wide) transposed product — the time the padding rows 100..127 cost
#ifndef SPWGNN_PAD_DBG
#define SPWGNN_PAD_DBG 0
#endif
// (the x6 edge kernels pick their wave counts per variant: kernels_fwd.hip / kernels_bwd.hip)

// ---- half tile (HT): a 4-tile product's last tile (output rows 96..127, of which a
// 100-wide layer uses 96..99) runs as two 16x16x32 MFMAs per k-block PAIR over rows 96..111 — one per
// 16-node half of the column tile — instead of one 32x32x16 MFMA per k-block over 32 rows: half the
// matrix cycles of that tile. B operands: one v_permlane16_swap per register of the pair's split
// parts (lane group g = (k-block 2P + (g&1), lane half g>>1), the image's ht slot order). The two
// 16x16 accumulators convert to and from rows 0..15 of the 32x32 C tile with permlane16 + permlane32
// swaps (both involutions), so every caller keeps the 32x32 C layout; rows 16..31 stay untouched.
template <int NC, int NT>
__device__ __forceinline__ void ht_enter(const f32x16 (&out)[NC][NT], f32x4 (&q)[NC][2]) {
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const auto x = __builtin_amdgcn_permlane32_swap(__float_as_uint(out[c][3][r]), __float_as_uint(out[c][3][4 + r]), false, false);
            const auto y = __builtin_amdgcn_permlane16_swap(x[0], x[1], false, false);
            q[c][0][r] = __uint_as_float(y[0]);
            q[c][1][r] = __uint_as_float(y[1]);
        }
}
template <int NC, int NT>
__device__ __forceinline__ void ht_leave(const f32x4 (&q)[NC][2], f32x16 (&out)[NC][NT]) {
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const auto x = __builtin_amdgcn_permlane16_swap(__float_as_uint(q[c][0][r]), __float_as_uint(q[c][1][r]), false, false);
            const auto y = __builtin_amdgcn_permlane32_swap(x[0], x[1], false, false);
            out[c][3][r] = __uint_as_float(y[0]);
            out[c][3][4 + r] = __uint_as_float(y[1]);
        }
}
// k-block pair (x0 = k-block 2P, x1 = 2P + 1 or absent) of column tile c into its two half accumulators
template <int PARTS, int NC>
__device__ __forceinline__ void ht_mfma(const bf16x8 (&a)[3], const uint32_t (&x0)[NC][3][4], const uint32_t (&x1)[NC][3][4],
                                        bool has1, f32x4 (&q)[NC][2]) {
    constexpr int LP = PARTS == 1 ? 1 : 3;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        bf16x8 b0[3], b1[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            uint32_t u0[4] = {0u, 0u, 0u, 0u}, u1[4] = {0u, 0u, 0u, 0u};
            if (p < LP) {
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const auto r = __builtin_amdgcn_permlane16_swap(x0[c][p][m], has1 ? x1[c][p][m] : 0u, false, false);
                    u0[m] = r[0];
                    u1[m] = r[1];
                }
            }
            b0[p] = as_bf16x8(make_uint4(u0[0], u0[1], u0[2], u0[3]));
            b1[p] = as_bf16x8(make_uint4(u1[0], u1[1], u1[2], u1[3]));
        }
        q[c][0] = mfma16_x6<PARTS>(a, b0, q[c][0]);
        q[c][1] = mfma16_x6<PARTS>(a, b1, q[c][1]);
    }
}

// B sources that hand over a k-block's element pair m as stored bf16 bits (a `word(c, kb, m)`
// member): in bf16 math (one part) that word already is the operand — no unpack and re-pack per pair
template <class T, class = void>
struct has_b16_words : std::false_type {};
template <class T>
struct has_b16_words<T, std::void_t<decltype(std::declval<const std::decay_t<T>&>().word(0, 0, 0))>> : std::true_type {};

// ---- transposed orientation in split-bf16 math (x6), NC column tiles of 32 rows per wave:
// out[c][T] += Wᵀ·B[c] over NKB k-blocks of 16. getb(c, kb, v) supplies the 8 fp32 B values of
// lane (j, h) for k-block kb (split into three bf16 parts here, once per k-block); the weight image
// (k_prep) holds, per step u = kb·NT_OUT + T, the three matching A-operand parts of lane (i, h),
// 16 bytes each: [u][part][lane] uint4. Steps stream through a D-deep ring of static slots (fully
// unrolled; the loads of step u + D issue before step u's MFMAs).
template <int NT_OUT, int NKB, int NC, int D = kX6Ring, int PARTS = 3, bool HT = false, class GetB>
__device__ __forceinline__ void tgemm_x6(GetB&& getb, f32x16 (&out)[NC][NT_OUT], const uint4* __restrict__ img,
                                         int lane) {
    static_assert(!HT || NT_OUT == 4, "half tile: 4-tile products");
    constexpr int NS = NKB * NT_OUT, NP = 4 * NC;   // pair-splits per k-block
    constexpr int SPD = HT ? 3 : 2;                 // split slots (HT: a pair's first k-block stays live)
    const uint4* wb = img + lane;
    uint4 ring[D][3];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int p = 0; p < 3; ++p) ring[d][p] = wb[(d * 3 + p) * 64];
    // split parts of k-block kb in slot kb % SPD; the next k-block's pair-splits are spread over
    // this k-block's steps, so the VALU work interleaves with the MFMAs
    uint32_t sp[SPD][NC][3][4];
    f32x4 hq[NC][2];
    if constexpr (HT) ht_enter(out, hq);
    auto split_pair = [&](int kb, int q) {
        const int c = q >> 2, m = q & 3;
        if constexpr (PARTS == 1 && has_b16_words<GetB>::value) {   // bf16 math: the stored pair is the h part
            sp[kb % SPD][c][0][m] = getb.word(c, kb, m);
            sp[kb % SPD][c][1][m] = sp[kb % SPD][c][2][m] = 0u;
        } else {
            float v[8];
            getb(c, kb, v);
            split2(v[2 * m], v[2 * m + 1], sp[kb % SPD][c][0][m], sp[kb % SPD][c][1][m], sp[kb % SPD][c][2][m]);
        }
    };
#pragma unroll
    for (int q = 0; q < NP; ++q) split_pair(0, q);
#pragma unroll
    for (int u = 0; u < NS; ++u) {
        const int kb = u / NT_OUT, T = u - kb * NT_OUT;
        bf16x8 bq[NC][3];
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int p = 0; p < 3; ++p)
                bq[c][p] = as_bf16x8(make_uint4(sp[kb % SPD][c][p][0], sp[kb % SPD][c][p][1], sp[kb % SPD][c][p][2], sp[kb % SPD][c][p][3]));
        bf16x8 a[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) a[p] = as_bf16x8(ring[u % D][p]);
        if (u + D < NS) {
#pragma unroll
            for (int p = 0; p < 3; ++p) ring[u % D][p] = wb[((u + D) * 3 + p) * 64];
        }
        if (kb + 1 < NKB) {
#pragma unroll
            for (int q = NP * T / NT_OUT; q < NP * (T + 1) / NT_OUT; ++q) split_pair(kb + 1, q);
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (HT) {
            if (T == 3) {
                if ((kb & 1) || kb == NKB - 1) ht_mfma<PARTS>(a, sp[(kb & ~1) % SPD], sp[kb % SPD], (kb & 1) != 0, hq);
                continue;
            }
        }
        if (SPWGNN_PAD_DBG && NT_OUT == 4 && T == 3) continue;   // diagnosis: the 100-wide layers' padding tile
#pragma unroll
        for (int c = 0; c < NC; ++c) out[c][T] = mfma32_x6<PARTS>(a, bq[c], out[c][T]);
    }
    if constexpr (HT) ht_leave(hq, out);
}
// ---- the same product with the weight image shared by the NW waves of a workgroup through LDS.
// Every wave of the workgroup calls the same tgemm_x6_wg sequence (no early exit: a wave with no
// rows of its own runs on clamped rows and stores nothing), so the image streams from L2 once per
// workgroup instead of once per wave. The image is cut into slices of KPS k-blocks (all NT_OUT steps,
// the parts the math uses: x6 one k-block × 3 parts, bf16 three k-blocks × the h part — ≤ 15 KiB
// either way), DMA'd (global_load_lds, 1 KiB per wave-instruction, the NW waves' pieces interleaved)
// into a ring of kWgRing LDS slots kWgRing − 2 slices ahead of use. One barrier per slice, at its
// last step: it certifies that slice sl+1 has landed (each wave waits for its own DMAs with a vmcnt
// that leaves the newer slices in flight) and that no wave still reads slot (sl−1) mod kWgRing, which
// then receives slice sl + kWgRing − 1. Fragments are read one step ahead with ds_read_b128.
// lds: kWgRing · kWgSlot uint4.
constexpr int kWgSlot = 15 * 64;   // uint4 per slot
constexpr int kWgRing = 4;         // slots (4 × 15 KiB per workgroup; two workgroups per CU)
template <int NW>
struct WgRing {
    uint4* lds;
    int wid;   // wave index in the workgroup (wave-uniform)
};
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int NT_OUT, int NKB, int NC, int NW, int PARTS = 3, bool HT = false, class GetB>
__device__ __forceinline__ void tgemm_x6_wg(GetB&& getb, f32x16 (&out)[NC][NT_OUT], const uint4* __restrict__ img,
                                            int lane, const WgRing<NW>& wr) {
    static_assert(!HT || NT_OUT == 4, "half tile: 4-tile products");
    constexpr int SPD = HT ? 3 : 2;
    constexpr int LP = PARTS == 1 ? 1 : 3;    // parts held in LDS
    constexpr int KPS = PARTS == 1 ? 3 : 1;   // k-blocks per slice
    static_assert(KPS * NT_OUT * LP * 64 <= kWgSlot, "slot size");
    constexpr int NS = NKB * NT_OUT, NP = 4 * NC, SST = KPS * NT_OUT;   // steps, pair-splits, steps per slice
    constexpr int NSL = (NKB + KPS - 1) / KPS, R = kWgRing;
    constexpr int PPW = (SST * LP + NW - 1) / NW;   // DMAs per wave per slice (short slices repeat pieces)
    auto issue = [&](int sl) {
        const int pc = (min(KPS, NKB - sl * KPS) * NT_OUT) * LP;   // pieces of this slice
#pragma unroll
        for (int q = 0; q < PPW; ++q) {
            const int i = min(wr.wid + NW * q, pc - 1);   // the last pieces may be loaded twice (same bytes)
            const int js = i / LP, p = i - js * LP;       // step within the slice, part
            __builtin_amdgcn_global_load_lds(img + ((sl * SST + js) * 3 + p) * 64 + lane,
                                             wr.lds + ((sl % R) * kWgSlot + i * 64), 16, 0, 0);
        }
    };
    const uint4* rl = wr.lds + lane;
    auto frag = [&](int u, uint4 (&f)[3]) {
        const int sl = u / SST, js = u - sl * SST;
#pragma unroll
        for (int p = 0; p < 3; ++p) f[p] = p < LP ? rl[(sl % R) * kWgSlot + (js * LP + p) * 64] : make_uint4(0u, 0u, 0u, 0u);
    };
    __builtin_amdgcn_s_barrier();   // every wave is done with the previous call's slots
    asm volatile("" ::: "memory");  // no memory op moves below: the vmcnt counts below see only DMAs
#pragma unroll
    for (int sl = 0; sl < R - 1 && sl < NSL; ++sl) issue(sl);
    uint32_t sp[SPD][NC][3][4];
    f32x4 hq[NC][2];
    if constexpr (HT) ht_enter(out, hq);
    auto split_pair = [&](int kb, int q) {
        const int c = q >> 2, m = q & 3;
        if constexpr (PARTS == 1 && has_b16_words<GetB>::value) {   // bf16 math: the stored pair is the h part
            sp[kb % SPD][c][0][m] = getb.word(c, kb, m);
            sp[kb % SPD][c][1][m] = sp[kb % SPD][c][2][m] = 0u;
        } else {
            float v[8];
            getb(c, kb, v);
            split2(v[2 * m], v[2 * m + 1], sp[kb % SPD][c][0][m], sp[kb % SPD][c][1][m], sp[kb % SPD][c][2][m]);
        }
    };
#pragma unroll
    for (int q = 0; q < NP; ++q) split_pair(0, q);
    wait_vmcnt<PPW * ((R - 2 < NSL - 1) ? R - 2 : NSL - 1)>();   // slice 0 landed (this wave's part)
    __builtin_amdgcn_s_barrier();
    uint4 fr[2][3];
    frag(0, fr[0]);
#pragma unroll
    for (int u = 0; u < NS; ++u) {
        const int kb = u / NT_OUT, T = u - kb * NT_OUT;
        bf16x8 bq[NC][3];
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int p = 0; p < 3; ++p)
                bq[c][p] = as_bf16x8(make_uint4(sp[kb % SPD][c][p][0], sp[kb % SPD][c][p][1], sp[kb % SPD][c][p][2], sp[kb % SPD][c][p][3]));
        bf16x8 a[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) a[p] = as_bf16x8(fr[u & 1][p]);
        if (u + 1 < NS) {
            if ((u + 1) % SST == 0) {   // slice sl+1 landed, slot (sl−1) % R free on every wave
                const int sl = u / SST;
                // slices issued after sl+1 so far: up to min(sl + R − 2, NSL − 1)
                const int ahead = min(sl + R - 2, NSL - 1) - (sl + 1);
                if (ahead >= 2) wait_vmcnt<2 * PPW>();
                else if (ahead == 1) wait_vmcnt<PPW>();
                else wait_vmcnt<0>();
                __builtin_amdgcn_s_barrier();
                if (sl + R - 1 < NSL) issue(sl + R - 1);
            }
            frag(u + 1, fr[(u + 1) & 1]);
        }
        if (kb + 1 < NKB) {
#pragma unroll
            for (int q = NP * T / NT_OUT; q < NP * (T + 1) / NT_OUT; ++q) split_pair(kb + 1, q);
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (HT) {
            if (T == 3) {
                if ((kb & 1) || kb == NKB - 1) ht_mfma<PARTS>(a, sp[(kb & ~1) % SPD], sp[kb % SPD], (kb & 1) != 0, hq);
                continue;
            }
        }
        if (SPWGNN_PAD_DBG && NT_OUT == 4 && T == 3) continue;
#pragma unroll
        for (int c = 0; c < NC; ++c) out[c][T] = mfma32_x6<PARTS>(a, bq[c], out[c][T]);
    }
    if constexpr (HT) ht_leave(hq, out);
}
template <int NT_OUT, int NKB, int NT_IN, int NC, int NW, int PARTS = 3, bool HT = false>
__device__ __forceinline__ void tchain_x6_wg(const f32x16 (&in)[NC][NT_IN], f32x16 (&out)[NC][NT_OUT],
                                             const uint4* __restrict__ img, int lane, const WgRing<NW>& wr) {
    static_assert(NKB <= 2 * NT_IN, "k-blocks beyond the input tiles");
    tgemm_x6_wg<NT_OUT, NKB, NC, NW, PARTS, HT>(
        [&](int c, int kb, float (&v)[8]) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = in[c][kb >> 1][8 * (kb & 1) + e];
        },
        out, img, lane, wr);
}

// Chain layer: B = the C layout of the previous layer; k-block kb of tile t = kb>>1 is registers
// 8(kb&1) .. +7 of in[c][t] (element e of lane half h = feature 16kb + 8(e>>2) + 4h + (e&3): image
// kind X6_CHAIN).
template <int NT_OUT, int NKB, int NT_IN, int NC, int D = kX6Ring, int PARTS = 3, bool HT = false>
__device__ __forceinline__ void tchain_x6(const f32x16 (&in)[NC][NT_IN], f32x16 (&out)[NC][NT_OUT],
                                          const uint4* __restrict__ img, int lane) {
    static_assert(NKB <= 2 * NT_IN, "k-blocks beyond the input tiles");
    tgemm_x6<NT_OUT, NKB, NC, D, PARTS, HT>(
        [&](int c, int kb, float (&v)[8]) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = in[c][kb >> 1][8 * (kb & 1) + e];
        },
        out, img, lane);
}

// Kernels templated on the weight source: NW = 0 → each wave streams the image itself (tgemm_x6's
// register ring, depth D), NW > 0 → the workgroup's shared LDS ring (tgemm_x6_wg).
// HT: the half-tile form (4-tile products on the ht images, kernels.h X6Desc)
template <int NT_OUT, int NKB, int NC, int D, int PARTS, int NW, bool HT = false, class GetB>
__device__ __forceinline__ void tgemm_x6s(GetB&& getb, f32x16 (&out)[NC][NT_OUT], const uint4* __restrict__ img, int lane,
                                          const WgRing<NW>& wr) {
    if constexpr (NW > 0) tgemm_x6_wg<NT_OUT, NKB, NC, NW, PARTS, HT>(getb, out, img, lane, wr);
    else tgemm_x6<NT_OUT, NKB, NC, D, PARTS, HT>(getb, out, img, lane);
}
template <int NT_OUT, int NKB, int NT_IN, int NC, int D, int PARTS, int NW, bool HT = false>
__device__ __forceinline__ void tchain_x6s(const f32x16 (&in)[NC][NT_IN], f32x16 (&out)[NC][NT_OUT],
                                           const uint4* __restrict__ img, int lane, const WgRing<NW>& wr) {
    if constexpr (NW > 0) tchain_x6_wg<NT_OUT, NKB, NT_IN, NC, NW, PARTS, HT>(in, out, img, lane, wr);
    else tchain_x6<NT_OUT, NKB, NT_IN, NC, D, PARTS, HT>(in, out, img, lane);
}
// the chain kernels' 4-tile products in the half-tile form: kHT (kernels.h, build flag SPWGNN_HT)

// Half-row operand of tgemm_x6: lane half h of column tile c holds features KH·h .. KH·h + KH-1
// of its row (chunk-major: chunk q of a 32-row block at + 256q), loaded whole up front.
template <int KH, int NC>
struct HalfRows {
    static constexpr int Q = KH / 4;
    float4 raw[NC][Q];
    __device__ __forceinline__ void load(const float* const (&blk)[NC], int lane) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const float* p = blk[c] + ((lane >> 5) * 32 + (lane & 31)) * 4;
#pragma unroll
            for (int q = 0; q < Q; ++q) raw[c][q] = *reinterpret_cast<const float4*>(p + 256 * q);
        }
    }
    // the blocks at element offsets off[c] of the array at base
    __device__ __forceinline__ void load_at(const float* base, const int64_t (&off)[NC], int lane) {
        const float* blk[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) blk[c] = base + off[c];
        load(blk, lane);
    }
    __device__ __forceinline__ void operator()(int c, int kb, float (&v)[8]) const {
        const float4 x = raw[c][2 * kb];
        const float4 y = 2 * kb + 1 < Q ? raw[c][2 * kb + 1] : make_float4(0.f, 0.f, 0.f, 0.f);
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
        v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
    }
};
// The same operand stored as bf16 at the element index of its fp32 layout (bf16 math):
// 8-byte loads, unpacked to fp32 (the bf16 math's operand rounding then reproduces the stored bits).
template <int KH, int NC>
struct HalfRowsB16 {
    static constexpr int Q = KH / 4;
    uint2 raw[NC][Q];
    // the blocks at element offsets off[c] of the bf16 array at base (element e at byte 2e)
    __device__ __forceinline__ void load_at(const float* base, const int64_t (&off)[NC], int lane) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const uint16_t* p = reinterpret_cast<const uint16_t*>(base) + off[c] + ((lane >> 5) * 32 + (lane & 31)) * 4;
#pragma unroll
            for (int q = 0; q < Q; ++q) raw[c][q] = *reinterpret_cast<const uint2*>(p + 256 * q);
        }
    }
    __device__ __forceinline__ void operator()(int c, int kb, float (&v)[8]) const {
        const float4 x = unpack4_bf16(raw[c][2 * kb]);
        const float4 y = 2 * kb + 1 < Q ? unpack4_bf16(raw[c][2 * kb + 1]) : make_float4(0.f, 0.f, 0.f, 0.f);
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
        v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
    }
};
// fp32 or bf16 (B16) half rows
template <int KH, int NC, bool B16>
using HalfRowsT = typename std::conditional<B16, HalfRowsB16<KH, NC>, HalfRows<KH, NC>>::type;
// bf16 half rows that also hand their stored pairs to a one-part product as they are (has_b16_words)
template <int KH, int NC>
struct HalfRowsB16W : HalfRowsB16<KH, NC> {
    __device__ __forceinline__ uint32_t word(int c, int kb, int m) const {
        const int q = 2 * kb + (m >> 1);
        return q < HalfRowsB16<KH, NC>::Q ? ((m & 1) ? this->raw[c][q].y : this->raw[c][q].x) : 0u;
    }
};
template <int KH, int NC, bool B16>
using HalfRowsWT = typename std::conditional<B16, HalfRowsB16W<KH, NC>, HalfRows<KH, NC>>::type;

}  // namespace spw
