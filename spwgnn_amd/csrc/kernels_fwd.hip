// Forward kernels of the propagation network (Networks.py:31-96) for gfx950.
//
//   k_prep           zero-padded / transposed / permuted copies of the 22 Keras tensors + x6 images
//   k_enc_node       om encoder (Networks.py:76,78) + P0 copy + first U/V projections
//   k_enc_edge       rm encoder (Networks.py:75,77) + step-invariant part of rmp layer 1
//   k_edge_fwd       per step: h1 = relu(A + U[s] + V[r]) → h2 = relu(h1·W2 + b2) → receiver
//                    segment sum (Networks.py:84-88, with rmp layer 3 moved behind the sum)
//   k_node_fwd       per step: rmp layer 3 on the summed messages, tanh, omp, state update,
//                    readout, next-step U/V (Networks.py:88-96)
#include <type_traits>
#include "kernels.h"
#include <cstdlib>

namespace spw {

// ------------------------------------------------------------------------------------------------
// Element (r, c) of pack d, straight from the flat Keras params (zero padding outside the source).
__device__ __forceinline__ float pack_elem(const PackDesc& d, const float* __restrict__ params, int r, int c) {
    if (r == d.bias_row) return c < d.src_cols ? params[d.bias_off + c] : 0.f;
    const int sa = d.transpose ? c : r;                                   // source row (before row0)
    const int sb = d.perm ? wo2_perm(d.transpose ? r : c) : (d.transpose ? r : c);   // source col
    return (sa >= 0 && sa < d.src_rows && sb >= 0 && sb < d.src_cols)
               ? params[d.src_off + (int64_t)(sa + d.src_row0) * d.src_ld + sb] : 0.f;
}

// One launch per call: rows blockIdx.y < PK_COUNT write the zero-padded / transposed / permuted
// packs; the rows after them (x non-null) write the x6 operand images (kernels.h X6Desc), one thread
// per (step, lane) splitting its 8 weights, taken from the same pack elements (pack_elem) so the
// images need not wait for the packs.
__global__ void k_prep(PrepArgs a, PrepX6Args x) {
    const int id = blockIdx.y;
    if (a.pro_row && id == (int)gridDim.y - 1) {   // a replayed step's prologue (PrologueArgs)
        const PrologueArgs& p = a.pro;
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < p.n16; i += (int64_t)gridDim.x * blockDim.x)
            p.dst[i] = ld_sys_u4(p.src + i);   // host staging: system-coherent reads
        if (p.key && blockIdx.x == 0 && threadIdx.x == 0) step_advance_dev(p.key, p.step, p.mode, p.seed, p.rank);
        return;
    }
    if (id < PK_COUNT) {
        const PackDesc& d = a.desc[id];
        const int total = d.rows * d.cols;
        // four elements per thread in flight (the largest pack, rmp.0's 350 × 150, is ≈ 13 elements per
        // thread: one parameter load's latency each when issued one after the other)
        const int stride = gridDim.x * blockDim.x;
        for (int base = blockIdx.x * blockDim.x + threadIdx.x; base < total; base += 4 * stride) {
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int idx = base + u * stride;
                int r, c;
                if (d.k4) {  // idx = ((r>>2)·cols + c)·4 + (r&3)
                    const int q = idx >> 2, kb = q / d.cols;
                    c = q - kb * d.cols;
                    r = 4 * kb + (idx & 3);
                } else {
                    r = idx / d.cols;
                    c = idx - r * d.cols;
                }
                v[u] = idx < total ? pack_elem(d, a.params, r, c) : 0.f;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (base + u * stride < total) a.pk[d.dst_off + base + u * stride] = v[u];
        }
        return;
    }
    const X6Desc& d = x.d[id - PK_COUNT];
    const PackDesc& pd = a.desc[d.pack];
    const int n = d.nkb * d.nt_out * 64;
    for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += gridDim.x * blockDim.x) {
        const int lane = idx & 63, u = idx >> 6, kb = u / d.nt_out, T = u - kb * d.nt_out;
        // half-tile slot (kernels.h X6Desc ht): lane (i, g) of the 16x16x32 operand of k-block pair kb >> 1
        const bool half = d.ht && T == 3;
        const bool live = !half || (kb & 1) || kb == d.nkb - 1;
        const int kbe = half ? (kb & ~1) + ((lane >> 4) & 1) : kb;
        const int col = half ? 96 + (lane & 15) : 32 * T + (lane & 31), h = half ? lane >> 5 : lane >> 5;
        float w[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int k = d.kh ? d.kh * h + 8 * kbe + e : 16 * kbe + 8 * (e >> 2) + 4 * h + (e & 3);
            const bool in = live && kbe < d.nkb && (!d.kh || 8 * kbe + e < d.kh);
            w[e] = in ? pack_elem(pd, a.params, k, col) : 0.f;
        }
        uint32_t hw[4], mw[4], lw[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) split2(w[2 * m], w[2 * m + 1], hw[m], mw[m], lw[m]);
        uint4* o = x.img + d.dst + (int64_t)u * 3 * 64 + lane;
        o[0] = make_uint4(hw[0], hw[1], hw[2], hw[3]);
        o[64] = make_uint4(mw[0], mw[1], mw[2], mw[3]);
        o[128] = make_uint4(lw[0], lw[1], lw[2], lw[3]);
    }
}

// ------------------------------------------------------------------------------------------------
// om encoder: c_o = dropout(relu(om(y, w))), P0, U0 = P0·W1b, V0 = P0·W1c (transposed orientation,
// 32 nodes per wave).
__global__ __launch_bounds__(256, 2) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_enc_node(EncNodeArgs a) {
    const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
    const int nb = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int n = nb * 32 + j;
    if (nb * 32 >= a.n_nodes) return;
    const bool valid = n < a.n_nodes;
    const int nc = valid ? n : a.n_nodes - 1;
    const float4 p = reinterpret_cast<const float4*>(a.pos)[nc];
    const float o0 = p.y, o1 = p.z;  // Networks.py:65-71: (y, width)

    f32x16 Z[4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int f = rho(r, 0) + 4 * h + 32 * t;
            Z[t][r] = relu(dense2(o0, o1, a.w_om0[f], a.w_om0[128 + f], a.b_om0[f]));
        }
    const int64_t bN = (int64_t)nb * kCmBlkN, bE = (int64_t)nb * kCmBlk;   // chunk-major node blocks
    if (a.zo1) store_cm<4>(a.zo1 + bN, Z, lane, valid);

    f32x16 C[4];
    zero_tiles(C);
    tchain_acc<4, 4, 4, kLdN>(Z, C, a.w_om1, lane);
    bias_act_rho<4, true>(C, a.b_om1, h);  // relu(om(.)) — Networks.py:76
    if (a.dropout_on) {                    // Networks.py:78
        const uint32_t key = drop_row_key(run_seed(a), 2u, (uint32_t)a.node_tower[nc], (uint32_t)a.node_local[nc], 0xffffu);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = rho(r, 0) + 4 * h + 32 * t;
                C[t][r] = drop_keep(key, (uint32_t)f, a.thresh) ? C[t][r] * a.scale : 0.f;
            }
    }
    store_cm<4>(a.co + bN, C, lane, valid);

    // P0: the 'propagation' input (Networks.py:29,79), ld 100 → workspace ld 128
    f32x16 P[4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int f0 = 32 * t + 8 * q + 4 * h;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (a.prop && f0 < kFN && valid) v = *reinterpret_cast<const float4*>(a.prop + (int64_t)n * kFN + f0);
            P[t][4 * q] = v.x;
            P[t][4 * q + 1] = v.y;
            P[t][4 * q + 2] = v.z;
            P[t][4 * q + 3] = v.w;
        }
    store_cm<4>(a.P0 + bN, P, lane, valid);

    f32x16 U[5];
    zero_tiles(U);
    tchain_acc<5, 4, 4, kLdE>(P, U, a.w1b, lane);
    store_cm<5>(a.U0 + bE, U, lane, valid);
    zero_tiles(U);
    tchain_acc<5, 4, 4, kLdE>(P, U, a.w1c, lane);
    store_cm<5>(a.V0 + bE, U, lane, valid);
}

// The om encoder in split-bf16 math: the k_enc_node chain on tchain_x6 (one 32-node column tile per
// wave, two waves per SIMD).
// NW > 0: weight images shared by the workgroup's waves (tgemm_x6_wg); a wave past the last node
// block runs on the last block and stores nothing.
template <int NP, int NW = 0>
__global__ __launch_bounds__(256, 2) void k_enc_node_x6(EncNodeArgs a) {
    const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
    const int nb = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int n = nb * 32 + j;
    const bool has = nb * 32 < a.n_nodes;
    if (NW == 0 && !has) return;
    __shared__ uint4 wring[NW > 0 ? kWgRing * kWgSlot : 1];
    const WgRing<NW> wr{wring, __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6))};
    const int nbk = has ? nb : (a.n_nodes + 31) / 32 - 1;
    const bool valid = has && n < a.n_nodes;
    const int nc = valid ? n : a.n_nodes - 1;
    const float4 p = reinterpret_cast<const float4*>(a.pos)[nc];
    const float o0 = p.y, o1 = p.z;  // Networks.py:65-71: (y, width)
    f32x16 Z[1][4], C[1][4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int f = rho(r, 0) + 4 * h + 32 * t;
            Z[0][t][r] = relu(dense2(o0, o1, a.w_om0[f], a.w_om0[128 + f], a.b_om0[f]));
        }
    const int64_t bN = (int64_t)nbk * kCmBlkN, bE = (int64_t)nbk * kCmBlk;   // chunk-major node blocks
    if (a.zo1 && has) store_cm<4>(a.zo1 + bN, Z[0], lane, valid);
    zero_tiles(C[0]);
    tchain_x6s<4, 7, 4, 1, kX6Ring, NP, NW, kHT>(Z, C, kHT ? a.xh_om1 : a.x_om1, lane, wr);
    bias_act_rho<4, true>(C[0], a.b_om1, h);  // relu(om(.)) — Networks.py:76
    if (a.dropout_on) {                       // Networks.py:78
        const uint32_t key = drop_row_key(run_seed(a), 2u, (uint32_t)a.node_tower[nc], (uint32_t)a.node_local[nc], 0xffffu);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = rho(r, 0) + 4 * h + 32 * t;
                C[0][t][r] = drop_keep(key, (uint32_t)f, a.thresh) ? C[0][t][r] * a.scale : 0.f;
            }
    }
    if (has) store_cm<4>(a.co + bN, C[0], lane, valid);
    // P0: the 'propagation' input (Networks.py:29,79), ld 100 → workspace ld 128 (Z's registers)
    f32x16 (&P)[1][4] = Z;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int f0 = 32 * t + 8 * q + 4 * h;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (a.prop && f0 < kFN && valid) v = *reinterpret_cast<const float4*>(a.prop + (int64_t)n * kFN + f0);
            P[0][t][4 * q] = v.x;
            P[0][t][4 * q + 1] = v.y;
            P[0][t][4 * q + 2] = v.z;
            P[0][t][4 * q + 3] = v.w;
        }
    if (has) store_cm<4>(a.P0 + bN, P[0], lane, valid);
    f32x16 U[1][5];
    zero_tiles(U[0]);
    tchain_x6s<5, 7, 4, 1, kX6Ring, NP, NW>(P, U, a.x_w1b, lane, wr);
    if (has) store_cm_uv<5>(a.U0, bE, U[0], lane, valid, NP == 1 ? a.uv16 : kUvF32);
    zero_tiles(U[0]);
    tchain_x6s<5, 7, 4, 1, kX6Ring, NP, NW>(P, U, a.x_w1c, lane, wr);
    if (has) store_cm_uv<5>(a.V0, bE, U[0], lane, valid, NP == 1 ? a.uv16 : kUvF32);
}

// ------------------------------------------------------------------------------------------------
// rm encoder (transposed orientation, one 32-edge block per wave): d = pos[r]-pos[s] (2 feats)
// → 150 → 150 → 150 → 150 (+relu, dropout) = c_r; A = c_r·W1a + b1 (step-invariant first-layer
// term of rmp: W1·[c_r|P_s|P_r] = (c_r·W1a + b1) + P_s·W1b + P_r·W1c).
// TRAIN: the activations/sign bits for the backward are stored (a compile-time switch: a branch
// inside the chains would split the MFMA blocks the stores are scheduled into)
template <bool TRAIN>
__global__ __launch_bounds__(256, 2) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_enc_edge(EncEdgeArgs a) {
    const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
    const int blk = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (blk >= a.n_eblocks) return;
    const int64_t e = (int64_t)blk * 32 + j;
    const int s = a.esrc[e], d = a.edst[e];
    const bool valid = s >= 0;
    float dx = 0.f, dy = 0.f;
    if (valid) {
        const float4 ps = reinterpret_cast<const float4*>(a.pos)[s];
        const float4 pd = reinterpret_cast<const float4*>(a.pos)[d];
        dx = pd.x - ps.x;  // Networks.py:58-62 (receiver − sender), (x, y)
        dy = pd.y - ps.y;
    }
    f32x16 X[5], Y[5];
#pragma unroll
    for (int t = 0; t < 5; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int f = rho(r, 0) + 4 * h + 32 * t;
            X[t][r] = relu(dense2(dx, dy, a.w_rm0[f], a.w_rm0[160 + f], a.b_rm0[f]));
        }
    constexpr bool zb = TRAIN;
    uint32_t* const mb = TRAIN ? a.zmask + (int64_t)blk * 4 * 3 * 64 : nullptr;
    // saved activations (padding-edge rows unmasked: finite, and met only by zero gradients)
    const int64_t cmo = (int64_t)blk * kCmBlk;
    if (zb) {
        if (a.ed && h == 0) a.ed[e] = make_float2(dx, dy);
        if (a.z1) store_cm<5>(a.z1 + cmo, X, lane, true);
        store_pos_bits<5>(mb, X, lane);
    }
    zero_tiles(Y);
    tchain_acc<5, 5, 12, kLdE>(X, Y, a.w_rm1, lane);
    bias_act_rho<5, true>(Y, a.b_rm1, h);
    if (zb) {
        store_cm<5>(a.z2 + cmo, Y, lane, true);
        store_pos_bits<5>(mb + 3 * 64, Y, lane);
    }
    zero_tiles(X);
    tchain_acc<5, 5, 12, kLdE>(Y, X, a.w_rm2, lane);
    bias_act_rho<5, true>(X, a.b_rm2, h);
    if (zb) {
        store_cm<5>(a.z3 + cmo, X, lane, true);
        store_pos_bits<5>(mb + 6 * 64, X, lane);
    }
    zero_tiles(Y);
    tchain_acc<5, 5, 12, kLdE>(X, Y, a.w_rm3, lane);
    bias_act_rho<5, true>(Y, a.b_rm3, h);  // rm's last Dense is linear; relu from Networks.py:75
    if (a.dropout_on && valid) {           // Networks.py:77
        const uint32_t tw = (uint32_t)a.node_tower[s];
        const uint32_t key = drop_row_key(run_seed(a), 1u, tw, (uint32_t)a.node_local[s], (uint32_t)a.node_local[d]);
#pragma unroll
        for (int t = 0; t < 5; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = rho(r, 0) + 4 * h + 32 * t;
                Y[t][r] = drop_keep(key, (uint32_t)f, a.thresh) ? Y[t][r] * a.scale : 0.f;
            }
    }
    if (zb) {
        store_cm<5>(a.cr + cmo, Y, lane, true);
        store_pos_bits<5>(mb + 9 * 64, Y, lane);
    }
    zero_tiles(X);
    tchain_acc<5, 5, 12, kLdE>(Y, X, a.w_w1a, lane);
    bias_act_rho<5, false>(X, a.b_w1a, h);
    store_cm<5>(a.A + (int64_t)blk * kCmBlk, X, lane, true);   // chunk-major; k_edge_fwd masks padding edges
}

// The rm encoder in split-bf16 math: NC 32-edge blocks per wave (column tiles c). Launched with
// NC = 1 at two waves per SIMD and the weight images shared by the workgroup's 4 waves through an
// LDS ring (NW = 4, tgemm_x6_wg); NC = 2 at one wave per SIMD (each 16-byte fragment feeding two
// MFMAs, in + out activations 320 registers) with per-wave rings is the measured alternative.
// B16 (bf16 math, training): z2, z3 and c_r — MFMA operands only (the weight gradients' X) — are
// stored as bf16 (exact), and so is A (rounded once before h1 = relu(A + U + V) adds it; §3g).
// waves per workgroup of the relation encoder and its backward (build options): all of a workgroup's
// waves share one pass of each weight image through the LDS ring. 8 instead of 4 was slower in both
// maths (round 6, same-box A/B, bitwise equal: bf16 config 3 encoder 4.2 → 4.8 ms, x6 headline 2.1 →
// 2.28 ms per step): the ring's per-slice barrier couples twice the waves, and halving the weight
// traffic bought nothing
#ifndef SPWGNN_ENC_NW_B16   // bf16 math, bf16 storage
#define SPWGNN_ENC_NW_B16 4
#endif
#ifndef SPWGNN_ENC_NW_X6    // the same in split-bf16 (x6) math
#define SPWGNN_ENC_NW_X6 4
#endif
template <bool TRAIN, int NC, int NP = 3, bool B16 = false, int NW = 0>
__global__ __launch_bounds__(NW > 4 ? 64 * NW : 256, NC == 1 && NW <= 4 ? 2 : 1) void k_enc_edge_x6(EncEdgeArgs a) {
    constexpr int kWaves = NW > 4 ? NW : 4;   // waves per workgroup (NW > 0: all share one weight ring)
    const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
    const int blk0 = (blockIdx.x * kWaves + (threadIdx.x >> 6)) * NC;
    if (NW == 0 && blk0 >= a.n_eblocks) return;   // NW > 0: no early exit (tgemm_x6_wg)
    __shared__ uint4 wring[NW > 0 ? kWgRing * kWgSlot : 1];
    const WgRing<NW> wr{wring, __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6))};
    f32x16 X[NC][5], Y[NC][5];
    int src[NC], dst[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int blk = blk0 + c;
        const int64_t e = (int64_t)min(blk, a.n_eblocks - 1) * 32 + j;
        src[c] = blk < a.n_eblocks ? a.esrc[e] : -1;
        dst[c] = blk < a.n_eblocks ? a.edst[e] : -1;
        float dx = 0.f, dy = 0.f;
        if (src[c] >= 0) {
            const float4 ps = reinterpret_cast<const float4*>(a.pos)[src[c]];
            const float4 pd = reinterpret_cast<const float4*>(a.pos)[dst[c]];
            dx = pd.x - ps.x;  // Networks.py:58-62 (receiver − sender), (x, y)
            dy = pd.y - ps.y;
        }
        if (TRAIN && a.ed && h == 0 && blk < a.n_eblocks) a.ed[e] = make_float2(dx, dy);
#pragma unroll
        for (int t = 0; t < 5; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = rho(r, 0) + 4 * h + 32 * t;
                X[c][t][r] = relu(dense2(dx, dy, a.w_rm0[f], a.w_rm0[160 + f], a.b_rm0[f]));
            }
    }
    auto save = [&](float* base, uint32_t* words, const f32x16 (&Z)[NC][5], bool b16 = false) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (blk0 + c >= a.n_eblocks) break;
            const int blk = blk0 + c;
            if (base) {
                if (B16 && b16) store_cm_b16<5>(reinterpret_cast<uint16_t*>(base) + (int64_t)blk * kCmBlk, Z[c], lane, true);
                else store_cm<5>(base + (int64_t)blk * kCmBlk, Z[c], lane, true);
            }
            if (words) store_pos_bits<5>(words + (int64_t)blk * 4 * 3 * 64, Z[c], lane);
        }
    };
    auto zero2 = [&](f32x16 (&Z)[NC][5]) {
#pragma unroll
        for (int c = 0; c < NC; ++c) zero_tiles(Z[c]);
    };
    if (TRAIN) save(a.z1, a.zmask, X);
    zero2(Y);
    tchain_x6s<5, 10, 5, NC, kX6Ring, NP, NW>(X, Y, a.x_rm1, lane, wr);
#pragma unroll
    for (int c = 0; c < NC; ++c) bias_act_rho<5, true>(Y[c], a.b_rm1, h);
    if (TRAIN) save(a.z2, a.zmask + 3 * 64, Y, true);
    zero2(X);
    tchain_x6s<5, 10, 5, NC, kX6Ring, NP, NW>(Y, X, a.x_rm2, lane, wr);
#pragma unroll
    for (int c = 0; c < NC; ++c) bias_act_rho<5, true>(X[c], a.b_rm2, h);
    if (TRAIN) save(a.z3, a.zmask + 6 * 64, X, true);
    zero2(Y);
    tchain_x6s<5, 10, 5, NC, kX6Ring, NP, NW>(X, Y, a.x_rm3, lane, wr);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        bias_act_rho<5, true>(Y[c], a.b_rm3, h);  // rm's last Dense is linear; relu from Networks.py:75
        if (a.dropout_on && src[c] >= 0) {         // Networks.py:77
            const uint32_t tw = (uint32_t)a.node_tower[src[c]];
            const uint32_t key = drop_row_key(run_seed(a), 1u, tw, (uint32_t)a.node_local[src[c]], (uint32_t)a.node_local[dst[c]]);
#pragma unroll
            for (int t = 0; t < 5; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int f = rho(r, 0) + 4 * h + 32 * t;
                    Y[c][t][r] = drop_keep(key, (uint32_t)f, a.thresh) ? Y[c][t][r] * a.scale : 0.f;
                }
        }
    }
    if (TRAIN) save(a.cr, a.zmask + 9 * 64, Y, true);
    zero2(X);
    tchain_x6s<5, 10, 5, NC, kX6Ring, NP, NW>(Y, X, a.x_w1a, lane, wr);
#pragma unroll
    for (int c = 0; c < NC; ++c) bias_act_rho<5, false>(X[c], a.b_w1a, h);
    if constexpr (TRAIN && NP == 1 && !B16) {   // bf16 math with fp32 storage (tiles of 17–32 nodes): A
#pragma unroll                                   // rounded as the bf16-stored copy is
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int t = 0; t < 5; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) X[c][t][r] = bf16_round(X[c][t][r]);
    }
    save(a.A, nullptr, X, true);   // chunk-major; k_edge_fwd masks padding edges (B16: bf16, §3g)
}

// ------------------------------------------------------------------------------------------------
// Receiver segment sum of one wave-tile on the matrix core (Networks.py:88 dot(receiver_relations,
// x)). C reg r of tile t of the h2 accumulators holds h2[edge rho(r,h)][feature 32t+i] — exactly a
// B operand whose k index runs over the edges, so  nodes += onehot(dst)·h2  needs no lane movement.
//  NW16 (≤ 16 nodes): 16x16x4 MFMAs, 10 tiles of 16 nodes × 16 features (40 registers). Lane l of
//    the B operand is edge rho(r, l>>5) (k = l>>4) carrying feature 32t + (l&31): lanes with
//    (l>>4) even carry feature tile 2t, odd ones tile 2t+1, so each (t, r) is two MFMAs whose
//    one-hot A operands are zero on the other parity.
//  else (≤ 32 nodes): one 32x32x2 MFMA per (t, r), 5 tiles of 32 nodes × 32 features.
// Padding edges have dst -1 and match no node; summation order is fixed (deterministic).
template <bool NW16> struct NodeSum;
template <> struct NodeSum<true> {
    f32x4 acc[10];
    int key, kq;
    __device__ __forceinline__ void init(int n0, int lane) {
        key = n0 + (lane & 15);
        kq = lane >> 4;
#pragma unroll
        for (int t = 0; t < 10; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __device__ __forceinline__ void add(const f32x16 (&h2)[5], int d) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int d0 = __builtin_amdgcn_readlane(d, rho(r, 0)), d1 = __builtin_amdgcn_readlane(d, rho(r, 1));
            const bool match = (kq < 2 ? d0 : d1) == key;
            const float ae = (match && !(kq & 1)) ? 1.f : 0.f, ao = (match && (kq & 1)) ? 1.f : 0.f;
#pragma unroll
            for (int t = 0; t < 5; ++t) {
                acc[2 * t] = mfma16(ae, h2[t][r], acc[2 * t]);
                acc[2 * t + 1] = mfma16(ao, h2[t][r], acc[2 * t + 1]);
            }
        }
    }
    // reg r of tile T: node 4·kq + r, feature 16T + (lane&15); H2s is chunk-major
    __device__ __forceinline__ void store(float* H2s, int n0, int nn, int lane) const {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int node = 4 * kq + r;
            if (node < nn) {
#pragma unroll
                for (int t = 0; t < 10; ++t) {
                    const int f = 16 * t + (lane & 15);
                    if (f < 2 * kKhE) H2s[cm_index<kKhE>(n0 + node, f)] = acc[t][r];
                }
            }
        }
    }
};
template <> struct NodeSum<false> {
    f32x16 acc[5];
    int key;
    __device__ __forceinline__ void init(int n0, int lane) {
        key = n0 + (lane & 31);
        zero_tiles(acc);
    }
    __device__ __forceinline__ void add(const f32x16 (&h2)[5], int d) {
        const int h = (threadIdx.x >> 5) & 1;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int d0 = __builtin_amdgcn_readlane(d, rho(r, 0)), d1 = __builtin_amdgcn_readlane(d, rho(r, 1));
            const float oh = ((h ? d1 : d0) == key) ? 1.f : 0.f;
#pragma unroll
            for (int t = 0; t < 5; ++t) acc[t] = mfma32(oh, h2[t][r], acc[t]);
        }
    }
    // reg r of tile t: node rho(r,h), feature 32t + (lane&31); H2s is chunk-major
    __device__ __forceinline__ void store(float* H2s, int n0, int nn, int lane) const {
        const int h = lane >> 5;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int node = rho(r, 0) + 4 * h;
            if (node < nn) {
#pragma unroll
                for (int t = 0; t < 5; ++t) {
                    const int f = 32 * t + (lane & 31);
                    if (f < 2 * kKhE) H2s[cm_index<kKhE>(n0 + node, f)] = acc[t][r];
                }
            }
        }
    }
};

// ------------------------------------------------------------------------------------------------
// One propagation step, edge side (natural orientation, one wave-tile of whole towers per wave;
// one 8-wave workgroup per CU walks the wave-tiles persistently).
// W2 lives in LDS as a [col][k] image (wl_fill): a lane's 4 consecutive k of one 32-column tile
// are one ds_read_b128, so a chunk (4 k-steps × 5 tiles) costs 5 LDS reads instead of 20 global
// loads, and only two tiles' fragments are live at a time.
// The receiver segment sum runs on the matrix core into registers (NodeSum).
template <bool NW16>
__global__ __launch_bounds__(512, 1) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_edge_fwd(EdgeFwdArgs a) {
    __shared__ __attribute__((aligned(16))) float wl[kWlFloats];
    wl_fill(wl, a.w2);
    const int lane = threadIdx.x & 63, h = lane >> 5, i = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const float* wrow = wl + i * kWlK + kKhE * h;
    const int4* wtiles = reinterpret_cast<const int4*>(a.wtile);
    const int wstep = gridDim.x * kEdgeWaves;
    // the per-block edge indices run one block ahead (across wave-tiles too): the U/V gathers of
    // a block depend on them
    auto load_sd = [&](int blk) { return make_int2(a.esrc[(int64_t)blk * 32 + i], a.edst[(int64_t)blk * 32 + i]); };
    int wt = blockIdx.x * kEdgeWaves + wave;
    int4 info = wtiles[min(wt, a.n_wtiles - 1)];
    int2 pre = load_sd(info.x);
    for (; wt < a.n_wtiles; wt += wstep) {
    const int fb = info.x, nb = info.y, n0 = info.z, nn = info.w;
    const int4 ninfo = wtiles[min(wt + wstep, a.n_wtiles - 1)];   // next wave-tile (clamped)
    NodeSum<NW16> nsum;
    nsum.init(n0, lane);

    for (int bb = 0; bb < nb; ++bb) {
        const int blk = fb + bb;
        const int64_t e = (int64_t)blk * 32 + i;
        const int2 cur = pre;
        pre = load_sd(bb + 1 < nb ? blk + 1 : ninfo.x);   // unconditional (clamped at the end)
        const int s = cur.x, d = cur.y;
        const bool valid = s >= 0;
        const int sc = valid ? s : n0, dc = valid ? d : n0;
        // h1 = relu(A + U[s] + V[r]) — rmp layer 1 (Networks.py:84-87), lane = edge, split
        // halves, streamed 4 features at a time straight into h2 = h1·W2 (rmp layer 2).
        const uint64_t vmask = __ballot(valid);
        const float vcap = valid ? __builtin_huge_valf() : 0.f;   // relu_valid: 0 on padding edges
        const float* Acm = a.A + (int64_t)blk * kCmBlk + h * 128 + i * 4;   // chunk q at + 256q
        // U[s], V[r]: chunk-major node rows (chunk q at +256q), gathered per lane
        const float4* U4 = reinterpret_cast<const float4*>(a.U + cm_index<kKhE>(sc, 4 * 0) + h * 128);
        const float4* V4 = reinterpret_cast<const float4*>(a.V + cm_index<kKhE>(dc, 4 * 0) + h * 128);
        // h1 > 0 bits (mask1: word per (block, feature), bit = edge): each chunk's 8 ballots go
        // into lanes 0..7 of one staging register (lanes 0-3: features 4q+c, lanes 4-7: 76+4q+c)
        // and are stored straight away.
        uint32_t* mrow = a.mask1 ? a.mask1 + (int64_t)blk * kLdE : nullptr;
        const int m1off = lane < 4 ? lane : kKhE + lane - 4;
        f32x16 acc[5];
        zero_tiles(acc);
        // A/U/V run two chunks ahead (A streams from HBM) in a 3-slot ring with static slot names
        // (loop unrolled by 3): no loop-carried register copies, so the waitcnt before a chunk
        // only covers that chunk's own loads
        float* h1cm = a.h1_out ? a.h1_out + (int64_t)blk * kCmBlk + h * 128 + i * 4 : nullptr;
        auto ldA = [&](int q) { return *reinterpret_cast<const float4*>(Acm + 256 * q); };
        struct AUV { float4 a, u, v; };
        AUV b0{ldA(0), U4[0], V4[0]}, b1{ldA(1), U4[64], V4[64]}, b2;
        auto chunk = [&](int q, const AUV& cur, AUV& ahead) {
            float xv[4];
            xv[0] = relu_valid(cur.a.x + cur.u.x + cur.v.x, vcap);
            xv[1] = relu_valid(cur.a.y + cur.u.y + cur.v.y, vcap);
            xv[2] = relu_valid(cur.a.z + cur.u.z + cur.v.z, vcap);
            xv[3] = relu_valid(cur.a.w + cur.u.w + cur.v.w, vcap);
            if (h1cm) *reinterpret_cast<float4*>(h1cm + 256 * q) = make_float4(xv[0], xv[1], xv[2], xv[3]);
            const int qn = min(q + 2, kKhE / 4 - 1);   // unconditional (clamped) prefetch
            ahead.a = ldA(qn);
            ahead.u = U4[64 * qn];
            ahead.v = V4[64 * qn];
            float4 wv = *reinterpret_cast<const float4*>(wrow + 4 * q);
#pragma unroll
            for (int t = 0; t < 5; ++t) {
                float4 wn;
                if (t < 4) wn = *reinterpret_cast<const float4*>(wrow + (t + 1) * 32 * kWlK + 4 * q);
                acc[t] = mfma32(xv[0], wv.x, acc[t]);
                acc[t] = mfma32(xv[1], wv.y, acc[t]);
                acc[t] = mfma32(xv[2], wv.z, acc[t]);
                acc[t] = mfma32(xv[3], wv.w, acc[t]);
                if (t < 4) wv = wn;
            }
            if (mrow) {
                uint32_t stg = 0u;
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const uint64_t bal = __ballot(xv[c] > 0.f);
                    stg = writelane_imm((uint32_t)bal, c, stg);
                    stg = writelane_imm((uint32_t)(bal >> 32), 4 + c, stg);
                }
                if (lane < 8) mrow[m1off + 4 * q] = stg;
            }
        };
        static_assert(kKhE / 4 == 19, "ring schedule below assumes 19 chunks");
#pragma unroll 1
        for (int q = 0; q < 18; q += 3) {
            chunk(q, b0, b2);
            chunk(q + 1, b1, b0);
            chunk(q + 2, b2, b1);
        }
        chunk(18, b0, b2);
        if (mrow && lane < 8) mrow[2 * kKhE + lane] = 0u;  // features 152..159 (padding)
#pragma unroll
        for (int t = 0; t < 5; ++t) {
            const float b = a.b2[32 * t + i];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                float v = relu(acc[t][r] + b);
                if (t == 4 && i == kDegCol - 128) v = 1.f;  // degree column (multiplies b3)
                const bool rv = (vmask >> (rho(r, 0) + 4 * h)) & 1;
                acc[t][r] = rv ? v : 0.f;
            }
        }
        if (a.mask2) {  // h2 > 0 bits, word per (block, tile, edge): bit = feature within tile
            uint32_t* m2row = a.mask2 + (int64_t)blk * kM2Blk;
            uint32_t mw[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int t = 0; t < 5; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const uint64_t bal = __ballot(acc[t][r] > 0.f);
                    const int w0 = m2_pos(rho(r, 0), t), w1 = m2_pos(rho(r, 1), t);
                    mw[w0 >> 6] = writelane_imm((uint32_t)bal, w0 & 63, mw[w0 >> 6]);
                    mw[w1 >> 6] = writelane_imm((uint32_t)(bal >> 32), w1 & 63, mw[w1 >> 6]);
                }
#pragma unroll
            for (int k = 0; k < 4; ++k) m2row[64 * k + lane] = mw[k];
        }
        nsum.add(acc, d);
    }
    // the wave-tile's node rows (each node is owned by exactly one wave-tile)
    nsum.store(a.H2s, n0, nn, lane);
    info = ninfo;
    }
}

// ------------------------------------------------------------------------------------------------
// One propagation step, node side (transposed orientation, 32 nodes per wave).
//   a  = tanh([H2s | deg]·[W3; b3])              (Networks.py:88, layer 3 after the sum)
//   o1 = relu([c_o | a | P]·Wo1 + bo1)            (Networks.py:89-90, omp layer 1)
//   x' = o1·Wo2' + bo2'   (x' = x with the logit moved to column 100)
//   P' = tanh(x'[0:100] + P); logit = x'[100]     (Networks.py:91, 94)
//   U' = P'·W1b, V' = P'·W1c for the next step
__global__ __launch_bounds__(256, 2) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_node_fwd(NodeFwdArgs a) {
    const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
    const int nb = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (nb * 32 >= a.n_nodes) return;
    const int n = nb * 32 + j;
    const bool valid = n < a.n_nodes;
    const int64_t bN = (int64_t)nb * kCmBlkN, bE = (int64_t)nb * kCmBlk;   // chunk-major node blocks

    f32x16 E[4];
    zero_tiles(E);
    {
        float xb[kKhE];
        load_half_cm<kKhE>(a.H2s + bE, lane, xb);
        tgemm_half_acc<4, kKhE, kLdN>(xb, E, a.w3a, lane);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int f = rho(r, 0) + 4 * h + 32 * t;
            E[t][r] = f < kFN ? tanhf(E[t][r]) : 0.f;
        }
    if (a.a_out) store_cm<4>(a.a_out + bN, E, lane, valid);

    f32x16 O[4];
    zero_tiles(O);
    {
        float xb[kKhN];
        load_half_cm<kKhN>(a.co + bN, lane, xb);
        tgemm_half_acc<4, kKhN, kLdN>(xb, O, a.wo1c, lane);
    }
    tchain_acc<4, 4, 4, kLdN>(E, O, a.wo1a, lane);
    {
        float xb[kKhN];
        load_half_cm<kKhN>(a.P + bN, lane, xb);
        tgemm_half_acc<4, kKhN, kLdN>(xb, O, a.wo1p, lane);
    }
    bias_act_rho<4, true>(O, a.bo1, h);
    if (a.o1_out) store_cm<4>(a.o1_out + bN, O, lane, valid);

    f32x16 X[4];
    zero_tiles(X);
    tchain_acc<4, 4, 4, kLdN>(O, X, a.wo2, lane);
    bias_act_rho<4, false>(X, a.bo2p, h);
    {
        f32x16 P[4];
        load_cm<4>(a.P + bN, P, lane);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = rho(r, 0) + 4 * h + 32 * t;
                E[t][r] = f < kFN ? tanhf(X[t][r] + P[t][r]) : 0.f;  // E := P'
            }
    }
    if (a.logits && h == 1 && valid) a.logits[n] = X[3][0];  // x' row 100 = rho(0,1) + 96
    store_cm<4>(a.Pn + bN, E, lane, valid);
    if (a.U) {
        f32x16 U[5];
        zero_tiles(U);
        tchain_acc<5, 4, 4, kLdE>(E, U, a.w1b, lane);
        store_cm<5>(a.U + bE, U, lane, valid);
        zero_tiles(U);
        tchain_acc<5, 4, 4, kLdE>(E, U, a.w1c, lane);
        store_cm<5>(a.V + bE, U, lane, valid);
    }
}

// ------------------------------------------------------------------------------------------------
// Node side of one step in split-bf16 math: the k_node_fwd chain on tgemm_x6, NC 32-node column
// tiles per wave (launched: NC = 1 at two waves per SIMD).
// NW > 0: the workgroup's 4 waves share each weight image through an LDS ring (tgemm_x6_wg; no
// early exit, a wave past the last node block runs on the clamped block and stores nothing).
// N16 (bf16 math, §3o): H2s read and o1 stored as bf16
template <int NC, int NP = 3, int NW = 0, bool N16 = false>
__global__ __launch_bounds__(256, NC == 1 ? 2 : 1) void k_node_fwd_x6(NodeFwdArgs a) {
    const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
    const int nb0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * NC;
    if (NW == 0 && nb0 * 32 >= a.n_nodes) return;
    __shared__ uint4 wring[NW > 0 ? kWgRing * kWgSlot : 1];
    const WgRing<NW> wr{wring, __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6))};
    const int nblocks = (a.n_nodes + 31) / 32;
    int nbc[NC];
    bool has[NC], valid[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        has[c] = nb0 + c < nblocks;
        nbc[c] = min(nb0 + c, nblocks - 1);
        valid[c] = has[c] && (nb0 + c) * 32 + j < a.n_nodes;
    }
    auto bN = [&](int c) { return (int64_t)nbc[c] * kCmBlkN; };
    auto bE = [&](int c) { return (int64_t)nbc[c] * kCmBlk; };
    auto zero2 = [&](f32x16 (&Z)[NC][4]) {
#pragma unroll
        for (int c = 0; c < NC; ++c) zero_tiles(Z[c]);
    };
    f32x16 E[NC][4], O[NC][4];
    zero2(E);
    {
        HalfRowsWT<kKhE, NC, N16> hr;
        int64_t off[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) off[c] = bE(c);
        hr.load_at(a.H2s, off, lane);
        tgemm_x6s<4, 10, NC, kX6Ring, NP, NW, kHT>(hr, E, kHT ? a.xh_w3a : a.x_w3a, lane, wr);
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = rho(r, 0) + 4 * h + 32 * t;
                E[c][t][r] = f < kFN ? acc_tanh(E[c][t][r]) : 0.f;
            }
        if (a.a_out && has[c]) store_cm<4>(a.a_out + bN(c), E[c], lane, valid[c]);
    }
    if (a.cw_in) {   // c_o·Wo1c of step 0 (bit-identical to repeating the product)
#pragma unroll
        for (int c = 0; c < NC; ++c) load_cm<4>(a.cw_in + bN(c), O[c], lane);
    } else {
        zero2(O);
        HalfRows<kKhN, NC> hr;
        const float* blk[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) blk[c] = a.co + bN(c);
        hr.load(blk, lane);
        tgemm_x6s<4, 7, NC, kX6Ring, NP, NW, kHT>(hr, O, kHT ? a.xh_wo1c : a.x_wo1c, lane, wr);
        if (a.cw_out)
#pragma unroll
            for (int c = 0; c < NC; ++c)
                if (has[c]) store_cm<4>(a.cw_out + bN(c), O[c], lane, true);
    }
    tchain_x6s<4, 7, 4, NC, kX6Ring, NP, NW, kHT>(E, O, kHT ? a.xh_wo1a : a.x_wo1a, lane, wr);
    {
        HalfRows<kKhN, NC> hr;
        const float* blk[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) blk[c] = a.P + bN(c);
        hr.load(blk, lane);
        tgemm_x6s<4, 7, NC, kX6Ring, NP, NW, kHT>(hr, O, kHT ? a.xh_wo1p : a.x_wo1p, lane, wr);
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        bias_act_rho<4, true>(O[c], a.bo1, h);
        if (a.o1_out && has[c]) {
            if constexpr (N16) store_cm_b16<4>(reinterpret_cast<uint16_t*>(a.o1_out) + bN(c), O[c], lane, valid[c]);
            else store_cm<4>(a.o1_out + bN(c), O[c], lane, valid[c]);
        }
    }
    // X reuses E's registers: x' = o1·Wo2' + b, then P' = tanh(x' + P) into E
    f32x16 (&X)[NC][4] = E;
    zero2(X);
    tchain_x6s<4, 7, 4, NC, kX6Ring, NP, NW, kHT>(O, X, kHT ? a.xh_wo2 : a.x_wo2, lane, wr);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        bias_act_rho<4, false>(X[c], a.bo2p, h);
        if (a.logits && h == 1 && valid[c]) a.logits[(nb0 + c) * 32 + j] = X[c][3][0];  // x' row 100 = rho(0,1) + 96
        f32x16 P[4];
        load_cm<4>(a.P + bN(c), P, lane);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = rho(r, 0) + 4 * h + 32 * t;
                X[c][t][r] = f < kFN ? acc_tanh(X[c][t][r] + P[t][r]) : 0.f;   // X := P'
            }
        if (has[c]) store_cm<4>(a.Pn + bN(c), X[c], lane, valid[c]);
    }
    if (a.U) {
        f32x16 U[NC][5];
#pragma unroll
        for (int c = 0; c < NC; ++c) zero_tiles(U[c]);
        tchain_x6s<5, 7, 4, NC, kX6Ring, NP, NW>(X, U, a.x_w1b, lane, wr);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (has[c]) store_cm_uv<5>(a.U, bE(c), U[c], lane, valid[c], NP == 1 ? a.uv16 : kUvF32);
            zero_tiles(U[c]);
        }
        tchain_x6s<5, 7, 4, NC, kX6Ring, NP, NW>(X, U, a.x_w1c, lane, wr);
#pragma unroll
        for (int c = 0; c < NC; ++c)
            if (has[c]) store_cm_uv<5>(a.V, bE(c), U[c], lane, valid[c], NP == 1 ? a.uv16 : kUvF32);
    }
}

// ------------------------------------------------------------------------------------------------
// One propagation step, edge side, in split-bf16 math (x6). Natural orientation as k_edge_fwd:
// lane (i, h) of a block holds edge i, features 76h + 8kb + e of k-block kb (two 4-feature chunks
// of the chunk-major A/U/V rows), so h1 = relu(A + U[s] + V[r]) is built, split and used as the A
// operand straight from the loads; W2 (x6 image, 150 KB) is the LDS B operand. The receiver sum
// runs as one-hot [node][edge] (exact in bf16) × h2 parts: 3 MFMAs per 16 edges per feature tile.
// 4 waves (one per SIMD: 512 registers) per CU, A/U/V prefetched kX6Pf k-blocks ahead.
template <int NP>
struct NodeSumX6 {
    f32x16 acc[5];
    int key;
    __device__ __forceinline__ void init(int n0, int lane) {
        key = n0 + (lane & 31);
        zero_tiles(acc);
    }
    // h2: C layout (reg r of lane (j, h) = edge rho(r, h), feature 32t + j); d: this lane's edge's receiver
    __device__ __forceinline__ void add(const f32x16 (&h2)[5], int d, int h) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            // A[node i][edge k], element e of half h ↔ edge 16s + 8(e>>2) + 4h + (e&3) = rho(8s+e, h)
            uint32_t oh[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                uint32_t w = 0u;
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int e = 2 * m + q;
                    const int d0 = __builtin_amdgcn_readlane(d, rho(8 * s + e, 0));
                    const int d1 = __builtin_amdgcn_readlane(d, rho(8 * s + e, 1));
                    w |= ((h ? d1 : d0) == key ? 0x3F80u : 0u) << (16 * q);
                }
                oh[m] = w;
            }
            bf16x8 a[1];
            a[0] = as_bf16x8(make_uint4(oh[0], oh[1], oh[2], oh[3]));
#pragma unroll
            for (int t = 0; t < 5; ++t) {
                uint32_t hw[4], mw[4], lw[4];
#pragma unroll
                for (int m = 0; m < 4; ++m) split2(h2[t][8 * s + 2 * m], h2[t][8 * s + 2 * m + 1], hw[m], mw[m], lw[m]);
                if constexpr (NP == 3) {
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], as_bf16x8(make_uint4(lw[0], lw[1], lw[2], lw[3])), acc[t], 0, 0, 0);
                    acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], as_bf16x8(make_uint4(mw[0], mw[1], mw[2], mw[3])), acc[t], 0, 0, 0);
                }
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], as_bf16x8(make_uint4(hw[0], hw[1], hw[2], hw[3])), acc[t], 0, 0, 0);
            }
        }
    }
    // reg r of tile t: node rho(r, h), feature 32t + (lane&31)
    template <bool B16 = false>
    __device__ __forceinline__ void store(float* H2s, int n0, int nn, int lane) const {
        static_assert(!B16, "bf16 H2s: ≤ 16-node tiles only (NodeSum16X6)");
        const int h = lane >> 5;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int node = rho(r, h);
            if (node < nn) {
#pragma unroll
                for (int t = 0; t < 5; ++t) {
                    const int f = 32 * t + (lane & 31);
                    if (f < 2 * kKhE) H2s[cm_index<kKhE>(n0 + node, f)] = acc[t][r];
                }
            }
        }
    }
};

// The same sum for wave-tiles of ≤ 16 nodes on 16x16x32 bf16 MFMAs: one v_permlane16_swap per
// register pair turns the 32-feature C tiles into two 16-feature B operands of 32 edges each
// (lane group g of a swapped register = edges of (s = g&1, h = g>>1)), so a block costs 30 MFMAs of
// 16 cycles into 40 accumulator registers.
template <int NP>
struct NodeSum16X6 {
    f32x4 acc[10];   // sub-tile u: features 16u + (lane & 15), nodes 4(lane >> 4) + r
    int key, n0;
    __device__ __forceinline__ void init(int n0_, int lane) {
        n0 = n0_;
        key = n0 + (lane & 15);
#pragma unroll
        for (int u = 0; u < 10; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    __device__ __forceinline__ void add(const f32x16 (&h2)[5], int d, int lane) {
        const int g = lane >> 4;
        // one-hot A: lane (node i, group g), element e ↔ edge 16(g&1) + 8(e>>2) + 4(g>>1) + (e&3)
#if SPWGNN_ONEHOT_BPERM
        // (the receiver's tile-local id fetched with one ds_bpermute per element: d − n0 == lane & 15
        // exactly when d == key, padding edges (d < 0) never)
        const int ld = d - n0, gb = 16 * (g & 1) + 4 * (g >> 1);
#endif
        uint32_t oh[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            uint32_t w = 0u;
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int e = 2 * m + q, base = 8 * (e >> 2) + (e & 3);
#if SPWGNN_ONEHOT_BPERM
                const int dn = __builtin_amdgcn_ds_bpermute(4 * (gb + base), ld);
                w |= (dn == (lane & 15) ? 0x3F80u : 0u) << (16 * q);
#else
                const int d0 = __builtin_amdgcn_readlane(d, base), d1 = __builtin_amdgcn_readlane(d, base + 16);
                const int d2 = __builtin_amdgcn_readlane(d, base + 4), d3 = __builtin_amdgcn_readlane(d, base + 20);
                const int dn = g == 0 ? d0 : g == 1 ? d1 : g == 2 ? d2 : d3;
                w |= (dn == key ? 0x3F80u : 0u) << (16 * q);
#endif
            }
            oh[m] = w;
        }
        const bf16x8 ao = as_bf16x8(make_uint4(oh[0], oh[1], oh[2], oh[3]));
#pragma unroll
        for (int t = 0; t < 5; ++t) {
            uint32_t P[2][3][4];
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int m = 0; m < 4; ++m)
                    split2(h2[t][8 * s + 2 * m], h2[t][8 * s + 2 * m + 1], P[s][0][m], P[s][1][m], P[s][2][m]);
#pragma unroll
            for (int p = 0; p < 3; ++p)
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const auto r = __builtin_amdgcn_permlane16_swap(P[0][p][m], P[1][p][m], false, false);
                    P[0][p][m] = r[0];   // sub-tile 2t
                    P[1][p][m] = r[1];   // sub-tile 2t + 1
                }
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int p = NP - 1; p >= 0; --p)
                    acc[2 * t + u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                        ao, as_bf16x8(make_uint4(P[u][p][0], P[u][p][1], P[u][p][2], P[u][p][3])), acc[2 * t + u], 0, 0, 0);
        }
    }
    // B16: bf16 at the element index (bf16 math: H2s only ever feeds bf16 MFMA operands, §3o)
    template <bool B16 = false>
    __device__ __forceinline__ void store(float* H2s, int n0, int nn, int lane) const {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int node = 4 * (lane >> 4) + r;
            if (node < nn) {
#pragma unroll
                for (int u = 0; u < 10; ++u) {
                    const int f = 16 * u + (lane & 15);
                    if (f < 2 * kKhE) {
                        if constexpr (B16) store_b16(H2s, cm_index<kKhE>(n0 + node, f), acc[u][r]);
                        else H2s[cm_index<kKhE>(n0 + node, f)] = acc[u][r];
                    }
                }
            }
        }
    }
};


// Wave-tiles of ≤ 16 nodes: 8 waves (2 per SIMD, 256 registers: the 16-node sum and a one-k-block
// ring); up to 32 nodes: 4 waves (1 per SIMD) with a 5-k-block ring.
#ifndef SPWGNN_EFWD_PF
#define SPWGNN_EFWD_PF 1
#endif
#ifndef SPWGNN_EFWD_PF_B16
#define SPWGNN_EFWD_PF_B16 2
#endif
// bf16 math: the A rows (the streamed HBM operand) may run deeper than the U/V gathers (cache hits)
#ifndef SPWGNN_EFWD_PFA_B16
#define SPWGNN_EFWD_PFA_B16 SPWGNN_EFWD_PF_B16
#endif
#ifndef SPWGNN_EFWD32_PF
#define SPWGNN_EFWD32_PF 1
#endif
// W8 (≤ 32-node tiles): 8 waves at two per SIMD (256 registers: the 32-node sum and a short ring)
// instead of 4 at one per SIMD with a 5-k-block ring
// N16: H2s stored as bf16 (bf16 math, §3o)
template <bool NW16, int DBG = 0, int NP = 3, bool AB16 = false, bool W8 = false, bool N16 = false>   // AB16: A stored as bf16 (§3g)
__global__ __launch_bounds__((NW16 || W8) ? 512 : 256, 1) __attribute__((amdgpu_waves_per_eu((NW16 || W8) ? 2 : 1, (NW16 || W8) ? 2 : 1)))
void k_edge_fwd_x6(EdgeFwdArgs a) {
    // bf16 math (NP = 1): a k-block is 5 MFMAs, too short to cover a load one k-block ahead
    constexpr int kWaves = (NW16 || W8) ? 8 : 4;
    constexpr int kX6Pf = NW16 ? (NP == 1 ? SPWGNN_EFWD_PF_B16 : SPWGNN_EFWD_PF) : (W8 ? SPWGNN_EFWD32_PF : 5);
    constexpr int kPfA = NW16 && NP == 1 ? SPWGNN_EFWD_PFA_B16 : kX6Pf;   // A rows' ring depth
    static_assert(10 % kX6Pf == 0 && 10 % kPfA == 0 && kPfA >= kX6Pf, "ring slots carry over between blocks");
    __shared__ uint4 wl[DBG == 2 ? 64 : 50 * 3 * 64];   // W2 x6 image: [kb·5 + T][part][lane]
    if constexpr (DBG != 2) {
        for (int idx = threadIdx.x; idx < 50 * 3 * 64; idx += blockDim.x) wl[idx] = a.x_w2[idx];
        __syncthreads();
    }
    const int lane = threadIdx.x & 63, h = lane >> 5, i = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int4* wtiles = reinterpret_cast<const int4*>(a.wtile);
    const int wstep = gridDim.x * kWaves;
    const WlBases wlb(wl + lane);
    auto load_sd = [&](int blk) { return make_int2(a.esrc[(int64_t)blk * 32 + i], a.edst[(int64_t)blk * 32 + i]); };
    // a block's h1 operand sources: A rows and the gathered U[s], V[r] rows (chunk q at +256q / +64q)
    // N16: U, V stored as bf16 (kUvB16, §3ze) — 8-byte pieces at the fp32 element index, unpacked at use
    using UVT = typename std::conditional<N16, uint2, float4>::type;
    struct Src { int64_t ai; const UVT *U, *V; };   // ai: element index of the A rows
    auto uv_at = [&](const float* base, int node) {
        const int64_t e = cm_index<kKhE>(node, 0) + h * 128;
        if constexpr (N16) return reinterpret_cast<const UVT*>(reinterpret_cast<const uint16_t*>(base) + e);
        else return reinterpret_cast<const UVT*>(base + e);
    };
    auto src_of = [&](int blk, int2 sd, int n0) {
        const int sc = DBG == 3 ? n0 : (sd.x >= 0 ? sd.x : n0), dc = DBG == 3 ? n0 : (sd.x >= 0 ? sd.y : n0);
        return Src{(int64_t)(DBG == 1 ? (blk & 7) : blk) * kCmBlk + h * 128 + i * 4, uv_at(a.U, sc), uv_at(a.V, dc)};
    };
    // k-block kb = chunks 2kb, 2kb+1 (chunk 19 does not exist: clamped, its W2 rows are zero)
    // (bf16 pieces stay packed in the ring and are unpacked where they are used)
    using AT = typename std::conditional<AB16, uint2, float4>::type;
    struct KA { AT a[2]; };
    struct KU { UVT u[2], v[2]; };
    auto ldA = [&](int64_t ai, int kb, KA& r) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int q = min(2 * kb + c, kKhE / 4 - 1);
            if constexpr (AB16)
                r.a[c] = ld_nt_u2(reinterpret_cast<const uint16_t*>(a.A) + ai + 256 * q);
            else
                r.a[c] = ld_nt_f4(a.A + ai + 256 * q);
        }
    };
    auto ldUV = [&](const Src& sr, int kb, KU& r) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int q = min(2 * kb + c, kKhE / 4 - 1);
            r.u[c] = sr.U[64 * q];
            r.v[c] = sr.V[64 * q];
        }
    };
    int wt = blockIdx.x * kWaves + wave;
    if (wt >= a.n_wtiles) return;
    int4 info = wtiles[wt];
    // the first block's sources and its first kX6Pf k-blocks; later blocks' arrive during the
    // previous block (the ring carries over)
    int2 cur_sd = load_sd(info.x);
    Src cur = src_of(info.x, cur_sd, info.z);
    KA ringA[kPfA];
    KU ringU[kX6Pf];
#pragma unroll
    for (int k = 0; k < kPfA; ++k) {
        ldA(cur.ai, k, ringA[k]);
        if (k < kX6Pf) ldUV(cur, k, ringU[k]);
    }
    for (; wt < a.n_wtiles; wt += wstep) {
    const int fb = info.x, nb = info.y, n0 = info.z, nn = info.w;
    const int4 ninfo = wtiles[min(wt + wstep, a.n_wtiles - 1)];
    typename std::conditional<NW16, NodeSum16X6<NP>, NodeSumX6<NP>>::type nsum;
    nsum.init(n0, lane);
    for (int bb = 0; bb < nb; ++bb) {
        const int blk = fb + bb;
        const int nblk = bb + 1 < nb ? blk + 1 : ninfo.x;   // the next block (clamped at the end)
        const int nn0 = bb + 1 < nb ? n0 : ninfo.z;
        const int2 nsd = load_sd(nblk);
        const int s = cur_sd.x, d = cur_sd.y;
        const bool valid = s >= 0;
        const uint64_t vmask = __ballot(valid);
        const float vcap = valid ? __builtin_huge_valf() : 0.f;   // relu_valid: 0 on padding edges
        uint32_t* mrow = a.mask1 ? a.mask1 + (int64_t)blk * kLdE : nullptr;
        const int m1off = lane < 4 ? lane : kKhE + lane - 4;
        Src nxt;
        const int64_t nai = (int64_t)(DBG == 1 ? (nblk & 7) : nblk) * kCmBlk + h * 128 + i * 4;   // = nxt.ai
        f32x16 acc[5];
        zero_tiles(acc);
#pragma unroll
        for (int kb = 0; kb < 10; ++kb) {
            KA& ca = ringA[kb % kPfA];
            KU& cu = ringU[kb % kX6Pf];
            float xv[8];
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const float4 av = unpack_uv(ca.a[c]), uv = unpack_uv(cu.u[c]), vv = unpack_uv(cu.v[c]);
                xv[4 * c + 0] = relu_valid(av.x + uv.x + vv.x, vcap);
                xv[4 * c + 1] = relu_valid(av.y + uv.y + vv.y, vcap);
                xv[4 * c + 2] = relu_valid(av.z + uv.z + vv.z, vcap);
                xv[4 * c + 3] = relu_valid(av.w + uv.w + vv.w, vcap);
            }
            uint32_t hw[4], mw[4], lw[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) split2(xv[2 * m], xv[2 * m + 1], hw[m], mw[m], lw[m]);
            if (kb + kPfA < 10) ldA(cur.ai, kb + kPfA, ca);
            else ldA(nai, kb + kPfA - 10, ca);
            if (kb + kX6Pf < 10) {
                ldUV(cur, kb + kX6Pf, cu);
            } else {
                if (kb + kX6Pf == 10) nxt = src_of(nblk, nsd, nn0);
                ldUV(nxt, kb + kX6Pf - 10, cu);
            }
            bf16x8 ap[3];
            ap[0] = as_bf16x8(make_uint4(hw[0], hw[1], hw[2], hw[3]));
            ap[1] = as_bf16x8(make_uint4(mw[0], mw[1], mw[2], mw[3]));
            ap[2] = as_bf16x8(make_uint4(lw[0], lw[1], lw[2], lw[3]));
            if (mrow) {   // h1 > 0 bits of the block's real chunks (ballots first, then the writelanes)
                uint64_t bal[2][4];
#pragma unroll
                for (int c = 0; c < 2; ++c)
#pragma unroll
                    for (int f = 0; f < 4; ++f) bal[c][f] = __ballot(xv[4 * c + f] > 0.f);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const int q = 2 * kb + c;
                    if (q < kKhE / 4) {
                        uint32_t v[8];
                        int ln[8];
#pragma unroll
                        for (int f = 0; f < 4; ++f) {
                            v[2 * f] = (uint32_t)bal[c][f];
                            ln[2 * f] = f;
                            v[2 * f + 1] = (uint32_t)(bal[c][f] >> 32);
                            ln[2 * f + 1] = 4 + f;
                        }
                        const uint32_t stg = writelane8_batched(0u, v, ln);
                        if (lane < 8) mrow[m1off + 4 * q] = stg;
                    }
                }
            }
            // output tiles in groups {0, 1}, {2, 3, 4}, products interleaved within a group
            auto group = [&](auto NTc, int T0) {
                constexpr int NT = decltype(NTc)::value;
                bf16x8 bp[NT][3];
#pragma unroll
                for (int v = 0; v < NT; ++v) {
                    const int u = (kb * 5 + T0 + v) * 3 * 64;
#pragma unroll
                    for (int q = 0; q < NP; ++q)   // DBG 2 (diagnosis): the image streamed from L2, LDS left free
                        bp[v][q] = as_bf16x8(DBG == 2 ? a.x_w2[u + 64 * q + lane] : wlb.at(u + 64 * q));
                }
                mfma32_x6_group<NP, NT>(ap, bp, acc + T0);
            };
            group(std::integral_constant<int, 2>{}, 0);
            group(std::integral_constant<int, 3>{}, 2);
        }
        if (mrow && lane < 8) mrow[2 * kKhE + lane] = 0u;  // features 152..159 (padding)
        const uint32_t vh = (uint32_t)vmask >> (4 * h);   // bit rho(r, 0): edge rho(r, h) is real
#pragma unroll
        for (int t = 0; t < 5; ++t) {
            const float b = a.b2[32 * t + i];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                float v = relu(acc[t][r] + b);
                if (t == 4 && i == kDegCol - 128) v = 1.f;  // degree column (multiplies b3)
                acc[t][r] = mask_bit(v, vh, rho(r, 0));
            }
        }
        if (a.mask2) {  // h2 > 0 bits, word per (block, tile, edge): bit = feature within tile
            uint32_t* m2row = a.mask2 + (int64_t)blk * kM2Blk;
            uint32_t mw2[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int t = 0; t < 5; ++t)
#pragma unroll
                for (int r0 = 0; r0 < 16; r0 += 8) {   // 8 ballots, then their 16 writelanes
                    uint64_t bal[8];
#pragma unroll
                    for (int r = 0; r < 8; ++r) bal[r] = __ballot(acc[t][r0 + r] > 0.f);
                    __builtin_amdgcn_sched_barrier(0);
                    // words m2_pos(rho(r, h), t) of ballots r = 4g..4g+3 all live in register g
                    // (m2_pos(rho(r, h), t) >> 6 == r >> 2): one 8-writelane batch per register
#pragma unroll
                    for (int g = 0; g < 2; ++g) {
                        uint32_t v[8];
                        int ln[8];
                        const int reg = (r0 >> 2) + g;
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const int r = 4 * g + e;
                            const int w0 = m2_pos(rho(r0 + r, 0), t), w1 = m2_pos(rho(r0 + r, 1), t);
                            v[2 * e] = (uint32_t)bal[r];
                            ln[2 * e] = w0 & 63;
                            v[2 * e + 1] = (uint32_t)(bal[r] >> 32);
                            ln[2 * e + 1] = w1 & 63;
                        }
                        mw2[reg] = writelane8_batched(mw2[reg], v, ln);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
#pragma unroll
            for (int k = 0; k < 4; ++k) m2row[64 * k + lane] = mw2[k];
        }
        nsum.add(acc, d, NW16 ? lane : h);
        cur_sd = nsd;
        cur = nxt;
    }
    nsum.template store<N16>(a.H2s, n0, nn, lane);
    info = ninfo;
    }
}

// Receiver blocks (spwgnn_plan_fill_recv, SPWGNN_BATCH_RECV_BLOCKS): block b holds the in-edges of
// node b alone (one block per node, in node order), so the receiver sum of a block is the COLUMN SUM
// of its h2 tile — 15 adds per register column and one v_permlane32_swap — instead of k_edge_fwd_x6's
// one-hot products (three bf16 parts of every h2 register and 30 MFMAs per block) and its node
// accumulators carried across a wave-tile's blocks. V[r] is one row per block (broadcast); U[s] are
// the tower's sender rows, which the 8 waves of a workgroup share from L1/L2: a workgroup walks a
// contiguous block range, wave w taking blocks w, w + 8, … of it (neighbouring receivers of one tower
// at a time). Products, k order and the h1/h2 bit masks are k_edge_fwd_x6's; the sum over a node's
// messages runs in a different (fixed) order: registers 0..15 of each half pairwise, then the halves.
// MASKS: training (h1/h2 bit masks stored); the inference instantiation carries none of that code
#ifndef SPWGNN_RB_PF
#define SPWGNN_RB_PF 2
#endif
template <int NP = 3, bool MASKS = true>
__global__ __launch_bounds__(512, 1) __attribute__((amdgpu_waves_per_eu(2, 2)))
void k_edge_fwd_rb_x6(EdgeFwdArgs a) {
    constexpr int kWaves = 8, kPf = SPWGNN_RB_PF;
    static_assert(10 % kPf == 0, "ring slots carry over between blocks");
    __shared__ uint4 wl[50 * 3 * 64];   // W2 x6 image: [kb·5 + T][part][lane]
    for (int idx = threadIdx.x; idx < 50 * 3 * 64; idx += blockDim.x) wl[idx] = a.x_w2[idx];
    __syncthreads();
    const int lane = threadIdx.x & 63, h = lane >> 5, i = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const WlBases wlb(wl + lane);
    const int nblk = a.n_nodes;   // one block per node
    const int per = ((nblk + gridDim.x - 1) / gridDim.x + kWaves - 1) / kWaves * kWaves;
    const int b0 = blockIdx.x * per, b1 = min(b0 + per, nblk);
    int blk = b0 + wave;
    if (blk >= b1) return;
    struct Src { int64_t ai; const float4 *U, *V; };
    auto src_of = [&](int b, int s) {
        const int sc = s >= 0 ? s : b;
        return Src{(int64_t)b * kCmBlk + h * 128 + i * 4,
                   reinterpret_cast<const float4*>(a.U + cm_index<kKhE>(sc, 0) + h * 128),
                   reinterpret_cast<const float4*>(a.V + cm_index<kKhE>(b, 0) + h * 128)};
    };
    struct KB { float4 a[2], u[2], v[2]; };
    auto ld = [&](const Src& sr, int kb, KB& r) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int q = min(2 * kb + c, kKhE / 4 - 1);
            r.a[c] = *reinterpret_cast<const float4*>(a.A + sr.ai + 256 * q);
            r.u[c] = sr.U[64 * q];
            r.v[c] = sr.V[64 * q];
        }
    };
    int cur_s = a.esrc[(int64_t)blk * 32 + i];
    Src cur = src_of(blk, cur_s);
    KB ring[kPf];
#pragma unroll
    for (int k = 0; k < kPf; ++k) ld(cur, k, ring[k]);
    for (; blk < b1; blk += kWaves) {
        const int nb = min(blk + kWaves, b1 - 1);   // the next block (clamped at the end)
        const int nxt_s = a.esrc[(int64_t)nb * 32 + i];
        const bool valid = cur_s >= 0;
        const uint64_t vmask = __ballot(valid);
        const float vcap = valid ? __builtin_huge_valf() : 0.f;   // relu_valid: 0 on padding edges
        uint32_t* mrow = MASKS && a.mask1 ? a.mask1 + (int64_t)blk * kLdE : nullptr;
        const int m1off = lane < 4 ? lane : kKhE + lane - 4;
        Src nxt;
        f32x16 acc[5];
        zero_tiles(acc);
#pragma unroll
        for (int kb = 0; kb < 10; ++kb) {
            KB& cr = ring[kb % kPf];
            float xv[8];
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                xv[4 * c + 0] = relu_valid(cr.a[c].x + cr.u[c].x + cr.v[c].x, vcap);
                xv[4 * c + 1] = relu_valid(cr.a[c].y + cr.u[c].y + cr.v[c].y, vcap);
                xv[4 * c + 2] = relu_valid(cr.a[c].z + cr.u[c].z + cr.v[c].z, vcap);
                xv[4 * c + 3] = relu_valid(cr.a[c].w + cr.u[c].w + cr.v[c].w, vcap);
            }
            uint32_t hw[4], mw[4], lw[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) split2(xv[2 * m], xv[2 * m + 1], hw[m], mw[m], lw[m]);
            if (kb + kPf < 10) {
                ld(cur, kb + kPf, cr);
            } else {
                if (kb + kPf == 10) nxt = src_of(nb, nxt_s);
                ld(nxt, kb + kPf - 10, cr);
            }
            bf16x8 ap[3];
            ap[0] = as_bf16x8(make_uint4(hw[0], hw[1], hw[2], hw[3]));
            ap[1] = as_bf16x8(make_uint4(mw[0], mw[1], mw[2], mw[3]));
            ap[2] = as_bf16x8(make_uint4(lw[0], lw[1], lw[2], lw[3]));
            if constexpr (!MASKS) __builtin_amdgcn_sched_barrier(0);   // keep the k-block order (as the mask code does)
            if (MASKS && mrow) {   // h1 > 0 bits of the block's real chunks (k_edge_fwd_x6's layout)
                uint64_t bal[2][4];
#pragma unroll
                for (int c = 0; c < 2; ++c)
#pragma unroll
                    for (int f = 0; f < 4; ++f) bal[c][f] = __ballot(xv[4 * c + f] > 0.f);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const int q = 2 * kb + c;
                    if (q < kKhE / 4) {
                        uint32_t v[8];
                        int ln[8];
#pragma unroll
                        for (int f = 0; f < 4; ++f) {
                            v[2 * f] = (uint32_t)bal[c][f];
                            ln[2 * f] = f;
                            v[2 * f + 1] = (uint32_t)(bal[c][f] >> 32);
                            ln[2 * f + 1] = 4 + f;
                        }
                        const uint32_t stg = writelane8_batched(0u, v, ln);
                        if (lane < 8) mrow[m1off + 4 * q] = stg;
                    }
                }
            }
            auto group = [&](auto NTc, int T0) {
                constexpr int NT = decltype(NTc)::value;
                bf16x8 bp[NT][3];
#pragma unroll
                for (int v = 0; v < NT; ++v) {
                    const int u = (kb * 5 + T0 + v) * 3 * 64;
#pragma unroll
                    for (int q = 0; q < NP; ++q) bp[v][q] = as_bf16x8(wlb.at(u + 64 * q));
                }
                mfma32_x6_group<NP, NT>(ap, bp, acc + T0);
            };
            group(std::integral_constant<int, 2>{}, 0);
            group(std::integral_constant<int, 3>{}, 2);
        }
        if (MASKS && mrow && lane < 8) mrow[2 * kKhE + lane] = 0u;  // features 152..159 (padding)
        const uint32_t vh = (uint32_t)vmask >> (4 * h);   // bit rho(r, 0): edge rho(r, h) is real
#pragma unroll
        for (int t = 0; t < 5; ++t) {
            const float b = a.b2[32 * t + i];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                float v = relu(acc[t][r] + b);
                if (t == 4 && i == kDegCol - 128) v = 1.f;  // degree column (multiplies b3)
                acc[t][r] = mask_bit(v, vh, rho(r, 0));
            }
        }
        if (MASKS && a.mask2) {  // h2 > 0 bits, word per (block, tile, edge): bit = feature within tile
            uint32_t* m2row = a.mask2 + (int64_t)blk * kM2Blk;
            uint32_t mw2[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int t = 0; t < 5; ++t)
#pragma unroll
                for (int r0 = 0; r0 < 16; r0 += 8) {
                    uint64_t bal[8];
#pragma unroll
                    for (int r = 0; r < 8; ++r) bal[r] = __ballot(acc[t][r0 + r] > 0.f);
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int g = 0; g < 2; ++g) {
                        uint32_t v[8];
                        int ln[8];
                        const int reg = (r0 >> 2) + g;
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const int r = 4 * g + e;
                            const int w0 = m2_pos(rho(r0 + r, 0), t), w1 = m2_pos(rho(r0 + r, 1), t);
                            v[2 * e] = (uint32_t)bal[r];
                            ln[2 * e] = w0 & 63;
                            v[2 * e + 1] = (uint32_t)(bal[r] >> 32);
                            ln[2 * e + 1] = w1 & 63;
                        }
                        mw2[reg] = writelane8_batched(mw2[reg], v, ln);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
#pragma unroll
            for (int k = 0; k < 4; ++k) m2row[64 * k + lane] = mw2[k];
        }
        // receiver sum of node blk = column sum of the block's h2 (padding rows are +0)
#pragma unroll
        for (int t = 0; t < 5; ++t) {
            float p8[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) p8[q] = acc[t][2 * q] + acc[t][2 * q + 1];
            const float s4a = (p8[0] + p8[1]) + (p8[2] + p8[3]), s4b = (p8[4] + p8[5]) + (p8[6] + p8[7]);
            const float sh = s4a + s4b;
            const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(sh), __float_as_uint(sh), false, false);
            const float tot = sh + __uint_as_float(sw[1]);   // lanes 0-31: + the other half's edges
            const int f = 32 * t + i;
            if (h == 0 && f < 2 * kKhE) a.H2s[cm_index<kKhE>(blk, f)] = tot;
        }
        cur_s = nxt_s;
        cur = nxt;
    }
}

int edge_grid(int n_wtiles, int waves) {
    static int cus = 0;  // compute units of the device (all devices of a node are alike)
    if (cus <= 0) {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
            v = 256;
        cus = v;
    }
    const int need = (n_wtiles + waves - 1) / waves;
    return need < 1 ? 1 : (need < cus ? need : cus);
}

#ifndef SPWGNN_PREP_GX   // workgroups per pack / image row (A/B at config 1: 8 / 16 / 32 → 0.1450 / 0.1417 / 0.1433 ms)
#define SPWGNN_PREP_GX 16
#endif
hipError_t launch_prep(const PrepArgs& a, const PrepX6Args* x, hipStream_t st) {
    const int rows = PK_COUNT + (x ? X6_PREP_COUNT : 0) + (a.pro_row ? 1 : 0);
    hipLaunchKernelGGL(k_prep, dim3(SPWGNN_PREP_GX, rows), dim3(256), 0, st, a, x ? *x : PrepX6Args{});
    return hipGetLastError();
}
hipError_t launch_enc_node(const EncNodeArgs& a, int math, hipStream_t st) {
    const int waves = (a.n_nodes + 31) / 32;
    if (a.uv16 && math != MATH_BF16) return hipErrorInvalidValue;   // rounded U0, V0: the bf16 kernels only
    if ((math == MATH_X6 || math == MATH_BF16) && team_blocks(waves)) return launch_enc_node_team(a, math, st);
    if (math == MATH_X6) {
        hipLaunchKernelGGL((k_enc_node_x6<3, 4>), dim3((waves + 3) / 4), dim3(256), 0, st, a);
        return hipGetLastError();
    }
    if (math == MATH_BF16) {
        hipLaunchKernelGGL((k_enc_node_x6<1, 4>), dim3((waves + 3) / 4), dim3(256), 0, st, a);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_enc_node, dim3((waves + 3) / 4), dim3(256), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_enc_edge(const EncEdgeArgs& a, int math, hipStream_t st) {
    const bool train = a.z1 || a.ed;   // z1 null with ed set: training, z1 rebuilt by the W1 gradient
    if ((math == MATH_X6 || math == MATH_BF16) && team_blocks(a.n_eblocks)) return launch_enc_edge_team(a, math, train, st);
    if (math == MATH_X6 || math == MATH_BF16) {
        // one 32-edge block per wave at two waves per SIMD, weight images shared by the workgroup's
        // 4 waves (x6: 2.48 → 2.11 ms against two blocks per wave at one wave per SIMD, per-wave rings)
        constexpr int NC = 1, NW = 4, NWB = SPWGNN_ENC_NW_B16;   // bf16: waves sharing one weight pass
        const dim3 g((a.n_eblocks + 4 * NC - 1) / (4 * NC)), gb((a.n_eblocks + NWB * NC - 1) / (NWB * NC));
        if (math == MATH_BF16) {
            if (train && a.b16) hipLaunchKernelGGL((k_enc_edge_x6<true, NC, 1, true, NWB>), gb, dim3(64 * NWB), 0, st, a);
            else if (train) hipLaunchKernelGGL((k_enc_edge_x6<true, NC, 1, false, NW>), g, dim3(256), 0, st, a);
            else hipLaunchKernelGGL((k_enc_edge_x6<false, NC, 1, false, NW>), g, dim3(256), 0, st, a);
        } else if (train) {
            constexpr int NWX = SPWGNN_ENC_NW_X6;
            const dim3 gx((a.n_eblocks + NWX * NC - 1) / (NWX * NC));
            hipLaunchKernelGGL((k_enc_edge_x6<true, NC, 3, false, NWX>), gx, dim3(64 * NWX), 0, st, a);
        } else {
            hipLaunchKernelGGL((k_enc_edge_x6<false, NC, 3, false, NW>), g, dim3(256), 0, st, a);
        }
        return hipGetLastError();
    }
    if (train)
        hipLaunchKernelGGL(k_enc_edge<true>, dim3((a.n_eblocks + 3) / 4), dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL(k_enc_edge<false>, dim3((a.n_eblocks + 3) / 4), dim3(256), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_edge_fwd(const EdgeFwdArgs& a, int math, hipStream_t st) {
    if (a.nw_max > kNwMaxLimit) return hipErrorInvalidValue;  // one-hot rows: ≤ 32 nodes per wave-tile
    if ((a.uv16 == kUvB16) != (a.n16 != 0)) return hipErrorInvalidValue;   // bf16 U, V: the N16 kernel reads them
    // small batches: a workgroup of five waves per wave-tile, one output tile per wave (kernels_team.hip)
    if ((math == MATH_X6 || math == MATH_BF16) && a.nw_max <= 16 && team_blocks(a.n_wtiles))
        return a.n16 ? hipErrorInvalidValue : launch_edge_fwd_team(a, math, st);   // team kernels: fp32 H2s
    if (a.n16 && (math != MATH_BF16 || a.nw_max > 16 || !a.a_b16)) return hipErrorInvalidValue;
    if (math == MATH_BF16 && a.n16) {
#ifdef SPWGNN_DIAG   // byte attribution (wrong results): 1 A rows from 8 cached blocks, 3 U/V rows of the tile's first node
        static const int ndbg = getenv("SPWGNN_EFWD_DBG") ? atoi(getenv("SPWGNN_EFWD_DBG")) : 0;
        if (ndbg == 1) {
            hipLaunchKernelGGL((k_edge_fwd_x6<true, 1, 1, true, false, true>), dim3(edge_grid(a.n_wtiles, 8)), dim3(512), 0, st, a);
            return hipGetLastError();
        }
        if (ndbg == 3) {
            hipLaunchKernelGGL((k_edge_fwd_x6<true, 3, 1, true, false, true>), dim3(edge_grid(a.n_wtiles, 8)), dim3(512), 0, st, a);
            return hipGetLastError();
        }
#endif
        hipLaunchKernelGGL((k_edge_fwd_x6<true, 0, 1, true, false, true>), dim3(edge_grid(a.n_wtiles, 8)), dim3(512), 0, st, a);
        return hipGetLastError();
    }
    if (math == MATH_BF16) {
#ifdef SPWGNN_DIAG   // 1: A rows from 8 cached blocks; 3: U, V rows of the tile's first node (wrong results)
        static const int bdbg = getenv("SPWGNN_EFWD_DBG") ? atoi(getenv("SPWGNN_EFWD_DBG")) : 0;
        if (a.nw_max <= 16 && a.a_b16 && bdbg == 1) {
            hipLaunchKernelGGL((k_edge_fwd_x6<true, 1, 1, true>), dim3(edge_grid(a.n_wtiles, 8)), dim3(512), 0, st, a);
            return hipGetLastError();
        }
        if (a.nw_max <= 16 && a.a_b16 && bdbg == 3) {
            hipLaunchKernelGGL((k_edge_fwd_x6<true, 3, 1, true>), dim3(edge_grid(a.n_wtiles, 8)), dim3(512), 0, st, a);
            return hipGetLastError();
        }
#endif
        if (a.nw_max <= 16 && a.a_b16)
            hipLaunchKernelGGL((k_edge_fwd_x6<true, 0, 1, true>), dim3(edge_grid(a.n_wtiles, 8)), dim3(512), 0, st, a);
        else if (a.a_b16)
            return hipErrorInvalidValue;
        else if (a.nw_max <= 16)
            hipLaunchKernelGGL((k_edge_fwd_x6<true, 0, 1>), dim3(edge_grid(a.n_wtiles, 8)), dim3(512), 0, st, a);
        else
            hipLaunchKernelGGL((k_edge_fwd_x6<false, 0, 1>), dim3(edge_grid(a.n_wtiles, 4)), dim3(256), 0, st, a);
        return hipGetLastError();
    }
    if (math == MATH_X6 && a.recv_blocks) {   // receiver blocks: column sums (spwgnn_plan_fill_recv)
        int cus = 0, dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        const int need = (a.n_nodes + 8 * 16 - 1) / (8 * 16);   // ≥ 16 blocks per wave
        const dim3 g(std::max(1, std::min(cus, need))), b(512);
        if (a.mask1 || a.mask2) hipLaunchKernelGGL((k_edge_fwd_rb_x6<3, true>), g, b, 0, st, a);
        else hipLaunchKernelGGL((k_edge_fwd_rb_x6<3, false>), g, b, 0, st, a);
        return hipGetLastError();
    }
    if (math == MATH_X6) {
#ifdef SPWGNN_DIAG   // 1: A rows from 8 cached blocks (diagnosis only: wrong results)
        static const int dbg = getenv("SPWGNN_EFWD_DBG") ? atoi(getenv("SPWGNN_EFWD_DBG")) : 0;
#else
        constexpr int dbg = 0;
#endif
        if (a.nw_max <= 16 && dbg == 1)   // diagnosis: A rows from 8 cached blocks
            hipLaunchKernelGGL((k_edge_fwd_x6<true, 1>), dim3(edge_grid(a.n_wtiles, 8)), dim3(512), 0, st, a);
#ifdef SPWGNN_DIAG
        else if (a.nw_max <= 16 && dbg == 2)   // diagnosis: W2 image from L2 instead of LDS
            hipLaunchKernelGGL((k_edge_fwd_x6<true, 2>), dim3(edge_grid(a.n_wtiles, 8)), dim3(512), 0, st, a);
#endif
        else if (a.nw_max <= 16)
            hipLaunchKernelGGL(k_edge_fwd_x6<true>, dim3(edge_grid(a.n_wtiles, 8)), dim3(512), 0, st, a);
        else   // ≤ 32-node tiles: two waves per SIMD (config 5: 37.5 -> 34.4 ms per forward, A/B on one box;
               // 36 spilled registers, an inference-only instantiation without the mask code spills 612)
            hipLaunchKernelGGL((k_edge_fwd_x6<false, 0, 3, false, true>), dim3(edge_grid(a.n_wtiles, 8)), dim3(512), 0, st, a);
        return hipGetLastError();
    }
    if (a.nw_max <= 16)
        hipLaunchKernelGGL(k_edge_fwd<true>, dim3(edge_grid(a.n_wtiles)), dim3(64 * kEdgeWaves), 0, st, a);
    else
        hipLaunchKernelGGL(k_edge_fwd<false>, dim3(edge_grid(a.n_wtiles)), dim3(64 * kEdgeWaves), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_node_fwd(const NodeFwdArgs& a, int math, hipStream_t st) {
    if ((a.uv16 == kUvB16) != (a.n16 != 0) || (a.uv16 && math != MATH_BF16)) return hipErrorInvalidValue;
    if ((math == MATH_X6 || math == MATH_BF16) && team_blocks((a.n_nodes + 31) / 32))
        return a.n16 ? hipErrorInvalidValue : launch_node_fwd_team(a, math, st);   // team kernels: fp32 arrays
    if (a.n16 && math != MATH_BF16) return hipErrorInvalidValue;
    const int waves = (a.n_nodes + 31) / 32;
    if (math == MATH_X6) {
        // one 32-node column tile per wave at two waves per SIMD (measured: 0.58 vs 0.62 ms for
        // two column tiles at one wave per SIMD, 393K nodes), weight images shared by the
        // workgroup's 4 waves through an LDS ring (0.532 → 0.437 ms)
        constexpr int NC = 1;
        const int w2 = (waves + NC - 1) / NC;
        hipLaunchKernelGGL((k_node_fwd_x6<NC, 3, 4>), dim3((w2 + 3) / 4), dim3(256), 0, st, a);
        return hipGetLastError();
    }
    if (math == MATH_BF16) {
        if (a.n16) hipLaunchKernelGGL((k_node_fwd_x6<1, 1, 4, true>), dim3((waves + 3) / 4), dim3(256), 0, st, a);
        else hipLaunchKernelGGL((k_node_fwd_x6<1, 1, 4>), dim3((waves + 3) / 4), dim3(256), 0, st, a);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_node_fwd, dim3((waves + 3) / 4), dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace spw
