// Backward kernels of the propagation network (replaces TF autodiff of Networks.py:31-96).
//
// Per step s (reverse order):
//   k_node_bwd   dP_{s+1} = dPpart + dU_{s+1}·W1bᵀ + dV_{s+1}·W1cᵀ;  dx' = [dP ⊙ (1-P²) | dlogit];
//                do1 = dx'·Wo2'ᵀ ⊙ [o1>0];  [dc_o | da | dP_omp] = do1·Wo1ᵀ;  g = da ⊙ (1-a²);
//                G3 = g·W3ᵀ (the per-edge dh2 is G3[receiver] — rmp layer 3 sits behind the sum)
//   k_edge_bwd   dh2pre = G3[r] ⊙ [h2>0];  dh1pre = dh2pre·W2ᵀ ⊙ [h1>0];  dA += dh1pre;
//                dU = Σ_sender dh1pre, dV = Σ_receiver dh1pre (deterministic LDS segment sums)
// Once:
//   k_enc_edge_bwd   dc_r = dA·W1aᵀ → rm backward chain (dz4..dz1, pre-activation grads)
//   k_enc_node_bwd   dc_o → om backward chain
#include "kernels.h"
#include <cstdlib>

namespace spw {

// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256, 2) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_node_bwd(NodeBwdArgs a) {
    const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
    const int nb = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (nb * 32 >= a.n_nodes) return;
    const int n = nb * 32 + j;
    const bool valid = n < a.n_nodes;
    const int64_t bN = (int64_t)nb * kCmBlkN, bE = (int64_t)nb * kCmBlk;   // chunk-major node blocks
    const int pj = (h * 32 + j) * 4;                                        // this lane's piece

    f32x16 D[4];
    if (a.first) {
        zero_tiles(D);
    } else {
        load_cm<4>(a.dPin + bN, D, lane);
        tgemm_stream_acc<4, kKhE, kLdN, 64>(a.dU + bE + pj, D, a.w1bt, lane);
        tgemm_stream_acc<4, kKhE, kLdN, 64>(a.dV + bE + pj, D, a.w1ct, lane);
    }
    if (a.tail) {  // dP0 = d/d 'propagation' (ld 100)
        if (valid) {
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int f0 = 32 * t + 8 * q + 4 * h;
                    if (f0 < kFN)
                        *reinterpret_cast<float4*>(a.dprop + (int64_t)n * kFN + f0) =
                            make_float4(D[t][4 * q], D[t][4 * q + 1], D[t][4 * q + 2], D[t][4 * q + 3]);
                }
        }
        return;
    }
    {
        f32x16 Pn[4];
        load_cm<4>(a.Pn + bN, Pn, lane);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = rho(r, 0) + 4 * h + 32 * t;
                const float p = Pn[t][r];
                D[t][r] = f < kFN ? D[t][r] * (1.f - p * p) : 0.f;  // tanh' (Networks.py:91)
            }
    }
    // the residual path: dP_s gets dpre directly (Add()([prop_layer(x), prop]))
    store_cm<4>(a.dPout + bN, D, lane, valid);
    if (a.first && h == 1) D[3][0] = valid ? a.dlogits[n] : 0.f;  // x' row 100 = logit
    store_cm<4>(a.dx + bN, D, lane, valid);

    f32x16 G[4];
    zero_tiles(G);
    tchain_acc<4, 4, 4, kLdN>(D, G, a.wo2t, lane);
    {
        f32x16 O1[4];
        load_cm<4>(a.o1 + bN, O1, lane);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) G[t][r] = O1[t][r] > 0.f ? G[t][r] : 0.f;
    }
    store_cm<4>(a.do1 + bN, G, lane, valid);

    // P part of omp's input → dP_s
    zero_tiles(D);
    tchain_acc<4, 4, 4, kLdN>(G, D, a.wo1pt, lane);
    {
        f32x16 T[4];
        load_cm<4>(a.dPout + bN, T, lane);
#pragma unroll
        for (int t = 0; t < 4; ++t) D[t] += T[t];
    }
    store_cm<4>(a.dPout + bN, D, lane, valid);
    // c_o part → dc_o (accumulated over steps in step order S-1..0)
    zero_tiles(D);
    tchain_acc<4, 4, 4, kLdN>(G, D, a.wo1ct, lane);
    if (a.dco_accumulate) {
        f32x16 T[4];
        load_cm<4>(a.dco + bN, T, lane);
#pragma unroll
        for (int t = 0; t < 4; ++t) D[t] = T[t] + D[t];
    }
    store_cm<4>(a.dco + bN, D, lane, valid);
    // effect part → g = da ⊙ (1 - a²) → G3 = g·W3ᵀ
    zero_tiles(D);
    tchain_acc<4, 4, 4, kLdN>(G, D, a.wo1at, lane);
    {
        f32x16 Aa[4];
        load_cm<4>(a.a + bN, Aa, lane);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float v = Aa[t][r];
                D[t][r] = D[t][r] * (1.f - v * v);
            }
    }
    store_cm<4>(a.g + bN, D, lane, valid);
    f32x16 H[5];
    zero_tiles(H);
    tchain_acc<5, 4, 4, kLdE>(D, H, a.w3t, lane);
    store_cm<5>(a.G3 + bE, H, lane, valid);
}

// Node side of one backward step in split-bf16 math: the k_node_bwd chain on tgemm_x6, NC 32-node
// column tiles per wave (launched: NC = 1 at two waves per SIMD).
// NW > 0: weight images shared by the workgroup's waves through an LDS ring (k_node_fwd_x6).
// N16 (bf16 math, §3g node side): dU, dV, o1 read and dx, g stored as bf16
template <int NC, int NP = 3, int NW = 0, bool N16 = false>
__global__ __launch_bounds__(256, NC == 1 ? 2 : 1) void k_node_bwd_x6(NodeBwdArgs a) {
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
    f32x16 D[NC][4], G[NC][4];
    if (a.first) {
        zero2(D);
    } else {
#pragma unroll
        for (int c = 0; c < NC; ++c) load_cm<4>(a.dPin + bN(c), D[c], lane);
        int64_t off[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) off[c] = bE(c);
        {
            HalfRowsT<kKhE, NC, N16> hr;
            hr.load_at(a.dU, off, lane);
            tgemm_x6s<4, 10, NC, kX6Ring, NP, NW, kHT>(hr, D, kHT ? a.xh_w1bt : a.x_w1bt, lane, wr);
        }
        {
            HalfRowsT<kKhE, NC, N16> hr;
            hr.load_at(a.dV, off, lane);
            tgemm_x6s<4, 10, NC, kX6Ring, NP, NW, kHT>(hr, D, kHT ? a.xh_w1ct : a.x_w1ct, lane, wr);
        }
    }
    if (a.tail) {  // dP0 = d/d 'propagation' (ld 100)
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (!valid[c]) continue;
            const int64_t n = (int64_t)(nb0 + c) * 32 + j;
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int f0 = 32 * t + 8 * q + 4 * h;
                    if (f0 < kFN)
                        *reinterpret_cast<float4*>(a.dprop + n * kFN + f0) =
                            make_float4(D[c][t][4 * q], D[c][t][4 * q + 1], D[c][t][4 * q + 2], D[c][t][4 * q + 3]);
                }
        }
        return;
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        f32x16 Pn[4];
        load_cm<4>(a.Pn + bN(c), Pn, lane);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = rho(r, 0) + 4 * h + 32 * t;
                const float p = Pn[t][r];
                D[c][t][r] = f < kFN ? D[c][t][r] * (1.f - p * p) : 0.f;  // tanh' (Networks.py:91)
            }
        // the residual path: dP_s gets dpre directly (Add()([prop_layer(x), prop]))
        if (has[c]) store_cm<4>(a.dPout + bN(c), D[c], lane, valid[c]);
        if (a.first && h == 1) D[c][3][0] = valid[c] ? a.dlogits[(nb0 + c) * 32 + j] : 0.f;  // x' row 100 = logit
        if (has[c]) {
            if constexpr (N16) store_cm_b16<4>(reinterpret_cast<uint16_t*>(a.dx) + bN(c), D[c], lane, valid[c]);
            else store_cm<4>(a.dx + bN(c), D[c], lane, valid[c]);
        }
    }
    zero2(G);
    tchain_x6s<4, 7, 4, NC, kX6Ring, NP, NW, kHT>(D, G, kHT ? a.xh_wo2t : a.x_wo2t, lane, wr);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        f32x16 O1[4];
        if constexpr (N16) load_cm_b16<4>(reinterpret_cast<const uint16_t*>(a.o1) + bN(c), O1, lane);
        else load_cm<4>(a.o1 + bN(c), O1, lane);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) G[c][t][r] = O1[t][r] > 0.f ? G[c][t][r] : 0.f;
        if (has[c]) store_cm<4>(a.do1 + bN(c), G[c], lane, valid[c]);
    }
    // P part of omp's input → dP_s
    zero2(D);
    tchain_x6s<4, 7, 4, NC, kX6Ring, NP, NW, kHT>(G, D, kHT ? a.xh_wo1pt : a.x_wo1pt, lane, wr);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        f32x16 T[4];
        load_cm<4>(a.dPout + bN(c), T, lane);
#pragma unroll
        for (int t = 0; t < 4; ++t) D[c][t] += T[t];
        if (has[c]) store_cm<4>(a.dPout + bN(c), D[c], lane, valid[c]);
    }
    // c_o part → dc_o (accumulated over steps in step order S-1..0); with dco_sum the product with
    // Wo1cᵀ is linear in do1 and runs once on Σ_s do1_s (k_enc_node_bwd)
    if (!a.dco_sum) {
        zero2(D);
        tchain_x6s<4, 7, 4, NC, kX6Ring, NP, NW, kHT>(G, D, kHT ? a.xh_wo1ct : a.x_wo1ct, lane, wr);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (a.dco_accumulate) {
                f32x16 T[4];
                load_cm<4>(a.dco + bN(c), T, lane);
#pragma unroll
                for (int t = 0; t < 4; ++t) D[c][t] = T[t] + D[c][t];
            }
            if (has[c]) store_cm<4>(a.dco + bN(c), D[c], lane, valid[c]);
        }
    }
    // effect part → g = da ⊙ (1 - a²) → G3 = g·W3ᵀ
    zero2(D);
    tchain_x6s<4, 7, 4, NC, kX6Ring, NP, NW, kHT>(G, D, kHT ? a.xh_wo1at : a.x_wo1at, lane, wr);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        f32x16 Aa[4];
        load_cm<4>(a.a + bN(c), Aa, lane);
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float v = Aa[t][r];
                D[c][t][r] = D[c][t][r] * (1.f - v * v);
            }
        if (has[c]) {
            if constexpr (N16) store_cm_b16<4>(reinterpret_cast<uint16_t*>(a.g) + bN(c), D[c], lane, valid[c]);
            else store_cm<4>(a.g + bN(c), D[c], lane, valid[c]);
        }
    }
    f32x16 H[NC][5];
#pragma unroll
    for (int c = 0; c < NC; ++c) zero_tiles(H[c]);
    tchain_x6s<5, 7, 4, NC, kX6Ring, NP, NW>(D, H, a.x_w3t, lane, wr);
#pragma unroll
    for (int c = 0; c < NC; ++c)
        if (has[c]) store_cm<5>(a.G3 + bE(c), H[c], lane, valid[c]);
}


// ------------------------------------------------------------------------------------------------
template <int WORD_BASE>
__device__ __forceinline__ void segsum_walk_b(const float* st, float* nacc, uint32_t csrw, int t, bool tv, int lane) {
    const int i = lane & 31, h = lane >> 5;
    // all LDS reads first (independent, pipelined), then the ordered per-node sums
    float vals[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        const uint32_t ow = (uint32_t)__builtin_amdgcn_readlane((int)csrw, WORD_BASE + (k >> 2));
        const int eo = (ow >> (8 * (k & 3))) & 31;
        vals[k] = st[h * 1056 + eo * 33 + i];
    }
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        const uint32_t nw = (uint32_t)__builtin_amdgcn_readlane((int)csrw, WORD_BASE + 8 + (k >> 2));
        const int nd = (nw >> (8 * (k & 3))) & 255;
        if (nd == 255) break;
        sum += vals[k];
        int ndn = 255;
        if (k < 31) {
            const uint32_t nw2 = (uint32_t)__builtin_amdgcn_readlane((int)csrw, WORD_BASE + 8 + ((k + 1) >> 2));
            ndn = (nw2 >> (8 * ((k + 1) & 3))) & 255;
        }
        if (ndn != nd) {
            if (tv) nacc[nd * kLdE + 32 * t + i] += sum;
            sum = 0.f;
        }
    }
}

// ONEHOT (wave-tiles of ≤ 16 nodes): both segment sums run on the matrix core as one product
//   nacc[t] += onehot·dh1pre[t],  A operand of lane (m, h) at k-step r (edge e = rho(r,h)):
//   m < 16: [dst(e) == n0+m] (receiver sum → dV),  m ≥ 16: [src(e) == n0+m−16] (sender sum → dU);
// otherwise (up to 32 nodes) the sums walk the block csr through a per-wave LDS stage.
// dA (Σ over steps of dh1pre) is written by the first backward step and accumulated by the later
// ones with no-return float atomics (one add per element per launch, launches stream-ordered:
// the summation order is fixed, so the result stays deterministic).
// B16 (bf16 math on wave-tiles of 17–32 nodes, which only this kernel serves): the products' operands
// dh2pre and W2ᵀ rounded to bf16 and the sender/receiver sums adding bf16(dh1pre) — the bf16
// arithmetic of the split-bf16 kernels on the fp32 matrix core; dA stays Σ fp32.
template <bool ONEHOT, bool ACCUM, bool B16 = false>
__global__ __launch_bounds__(ONEHOT ? 512 : 256, ONEHOT ? 1 : 2) __attribute__((amdgpu_waves_per_eu(2, 2)))
void k_edge_bwd(EdgeBwdArgs a) {
    const int lane = threadIdx.x & 63, h = lane >> 5, i = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // ONEHOT: persistent 8-wave workgroup with the W2ᵀ image in LDS (see k_edge_fwd);
    // otherwise one wave-tile per wave, LDS = segment-sum stage + node accumulators
    __shared__ __attribute__((aligned(16))) float wl[ONEHOT ? kWlFloats : 1];
    extern __shared__ __attribute__((aligned(16))) float smem[];
    if (ONEHOT) wl_fill(wl, a.w2t);
    const float* wrow = ONEHOT ? wl + i * kWlK + kKhE * h : a.w2t + (kKhE * h) * kLdE + i;
    const int wstep = ONEHOT ? gridDim.x * kEdgeWaves : a.n_wtiles;
    const int4* wtiles = reinterpret_cast<const int4*>(a.wtile);
    // per-block indices and h2>0 words run one block ahead (across wave-tiles too): the G3
    // gathers of a block depend on them
    struct Pre { int d, s; uint32_t w[5]; };
    auto load_pre = [&](int blk) {
        Pre p;
        const int64_t e = (int64_t)blk * 32 + i;
        p.d = a.edst[e];
        p.s = a.esrc[e];
        load_m2(a.mask2 + (int64_t)blk * kM2Blk, i, p.w);
        return p;
    };
    int wt = ONEHOT ? blockIdx.x * kEdgeWaves + wave : blockIdx.x * a.wpg + wave;
    int4 info = wtiles[min(wt, a.n_wtiles - 1)];
    Pre pre = load_pre(info.x);
    for (; wt < a.n_wtiles; wt += wstep) {
    const int fb = info.x, nb = info.y, n0 = info.z, nn = info.w;
    const int4 ninfo = wtiles[min(wt + wstep, a.n_wtiles - 1)];   // next wave-tile (clamped)
    float* st = smem + wave * (2112 + 2 * a.nw_max * kLdE);
    float* naccR = st + 2112;
    float* naccS = naccR + a.nw_max * kLdE;
    f32x16 nacc[5];
    const int key = n0 + (i & 15);
    if (ONEHOT) {
        zero_tiles(nacc);
    } else {
        for (int idx = lane; idx < nn * kLdE; idx += 64) {
            naccR[idx] = 0.f;
            naccS[idx] = 0.f;
        }
    }
    for (int bb = 0; bb < nb; ++bb) {
        const int blk = fb + bb;
        const int64_t e = (int64_t)blk * 32 + i;
        const Pre cur = pre;
        pre = load_pre(bb + 1 < nb ? blk + 1 : ninfo.x);   // unconditional (clamped at the end)
        const int d = cur.d;
        const bool valid = d >= 0;
        const int dc = valid ? d : n0;
        // dh1 mask words (used after the GEMM: the load has the whole GEMM to land)
        const uint32_t* m1 = a.mask1 + (int64_t)blk * kLdE + i;
        uint32_t m1w[5];
#pragma unroll
        for (int t = 0; t < 5; ++t) m1w[t] = m1[32 * t];
        // dh2pre (A operand, lane = edge, split halves): G3[receiver] ⊙ [h2 > 0]
        uint32_t w[5];
#pragma unroll
        for (int t = 0; t < 5; ++t) w[t] = valid ? cur.w[t] : 0u;
        // this lane's 76 feature bits (features 76h + 0..75) as a 64-bit low part and 12-bit tail
        const uint64_t mlo = h == 0 ? ((uint64_t)w[1] << 32 | w[0])
                                    : ((uint64_t)w[4] << 52 | (uint64_t)w[3] << 20 | (w[2] >> 12));
        const uint32_t mhi = h == 0 ? (w[2] & 0xfffu) : (w[4] >> 12);
        // G3[receiver]: chunk-major node row, chunk q at +64q float4
        const float4* G4 = reinterpret_cast<const float4*>(a.G3 + cm_index<kKhE>(dc, 0) + h * 128);
        f32x16 acc[5];
        zero_tiles(acc);
        // G3 rows (L2-resident node rows) run one chunk ahead in a 2-slot ring (loop unrolled by
        // 2, no register copies); W2ᵀ fragments come from the LDS image (ONEHOT) or global
        float4 g0 = G4[0], g1;
        float* dh2cm = a.dh2_out ? a.dh2_out + (int64_t)blk * kCmBlk + h * 128 + i * 4 : nullptr;   // optional dh2pre rows
        auto chunk = [&](int q, const float4& g, float4& ahead) {
            const uint32_t bits = (uint32_t)(q < 16 ? mlo >> (4 * q) : (uint64_t)(mhi >> (4 * q - 64)));
            float xv[4];
            xv[0] = (bits & 1u) ? g.x : 0.f;
            xv[1] = (bits & 2u) ? g.y : 0.f;
            xv[2] = (bits & 4u) ? g.z : 0.f;
            xv[3] = (bits & 8u) ? g.w : 0.f;
            if (a.dh2_out) *reinterpret_cast<float4*>(dh2cm + 256 * q) = make_float4(xv[0], xv[1], xv[2], xv[3]);
            if (B16) {
#pragma unroll
                for (int k = 0; k < 4; ++k) xv[k] = bf16_round(xv[k]);
            }
            ahead = G4[64 * min(q + 1, kKhE / 4 - 1)];  // unconditional (clamped) prefetch
            const float* wq = wrow + (ONEHOT ? 4 * q : 4 * q * kLdE);
            float4 wv = ONEHOT ? *reinterpret_cast<const float4*>(wq)
                               : make_float4(wq[0], wq[kLdE], wq[2 * kLdE], wq[3 * kLdE]);
#pragma unroll
            for (int t = 0; t < 5; ++t) {
                float4 wn;
                if (t < 4) {
                    const float* wt1 = wq + (t + 1) * (ONEHOT ? 32 * kWlK : 32);
                    wn = ONEHOT ? *reinterpret_cast<const float4*>(wt1)
                                : make_float4(wt1[0], wt1[kLdE], wt1[2 * kLdE], wt1[3 * kLdE]);
                }
                if (B16) wv = make_float4(bf16_round(wv.x), bf16_round(wv.y), bf16_round(wv.z), bf16_round(wv.w));
                acc[t] = mfma32(xv[0], wv.x, acc[t]);
                acc[t] = mfma32(xv[1], wv.y, acc[t]);
                acc[t] = mfma32(xv[2], wv.z, acc[t]);
                acc[t] = mfma32(xv[3], wv.w, acc[t]);
                if (t < 4) wv = wn;
            }
            __builtin_amdgcn_sched_barrier(0);  // no hoisting across chunks (register pressure)
        };
#pragma unroll 1
        for (int q = 0; q < 18; q += 2) {
            chunk(q, g0, g1);
            chunk(q + 1, g1, g0);
        }
        chunk(18, g0, g1);
        // dh1pre = dh1 ⊙ [h1 > 0]  (C layout: lane = feature 32t+i, rows = edges rho(r,h))
        float* dArow = a.dA + (int64_t)blk * 32 * kLdE + i;
#pragma unroll
        for (int t = 0; t < 5; ++t) {
            const uint32_t mw = m1w[t];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = rho(r, 0) + 4 * h;
                acc[t][r] = ((mw >> row) & 1u) ? acc[t][r] : 0.f;
            }
        }
        // dA: plain stores on the first backward step, no-return atomics after (ACCUM); in the
        // one-hot path they are issued beside the segment-sum MFMAs (same basic block)
        auto put_dA = [&](int t, int r) {
            float* p = dArow + (rho(r, 0) + 4 * h) * kLdE + 32 * t;
            if (ACCUM) unsafeAtomicAdd(p, acc[t][r]);
            else *p = acc[t][r];
        };
        if (ONEHOT) {  // segment sums on the matrix core (padding edges: src = dst = -1, no match)
            const int s = cur.s;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int d0 = __builtin_amdgcn_readlane(d, rho(r, 0)), d1 = __builtin_amdgcn_readlane(d, rho(r, 1));
                const int s0 = __builtin_amdgcn_readlane(s, rho(r, 0)), s1 = __builtin_amdgcn_readlane(s, rho(r, 1));
                const int node = i < 16 ? (h ? d1 : d0) : (h ? s1 : s0);
                const float oh = node == key ? 1.f : 0.f;
#pragma unroll
                for (int t = 0; t < 5; ++t) {
                    nacc[t] = mfma32(oh, acc[t][r], nacc[t]);
                    put_dA(t, r);
                }
            }
        } else {
#pragma unroll
            for (int t = 0; t < 5; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) put_dA(t, r);  // segment sums: receiver → dV, sender → dU
            const uint32_t csrw = reinterpret_cast<const uint32_t*>(a.csr)[(int64_t)blk * 32 + i];
#pragma unroll
            for (int rd = 0; rd < 3; ++rd) {
#pragma unroll
                for (int slot = 0; slot < 2; ++slot) {
                    const int t = 2 * rd + slot;
                    if (t >= 5) continue;
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        st[slot * 1056 + (rho(r, 0) + 4 * h) * 33 + i] = B16 ? bf16_round(acc[t][r]) : acc[t][r];
                }
                wave_lds_sync();
                const int t = 2 * rd + h;
                segsum_walk_b<0>(st, naccR, csrw, t, t < 5, lane);
                segsum_walk_b<16>(st, naccS, csrw, t, t < 5, lane);
                wave_lds_sync();
            }
        }
    }
    if (ONEHOT) {  // nacc[t] reg r = row rho(r,h): rows 0..15 receiver nodes, 16..31 sender nodes
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = rho(r, 0) + 4 * h;
            const int node = row & 15;
            if (node < nn) {
                float* o = row < 16 ? a.dV : a.dU;   // chunk-major node rows
#pragma unroll
                for (int t = 0; t < 5; ++t)
                    if (32 * t + i < 2 * kKhE) o[cm_index<kKhE>(n0 + node, 32 * t + i)] = nacc[t][r];
            }
        }
    } else {
        for (int idx = lane; idx < nn * kLdE; idx += 64) {
            const int node = idx / kLdE, f = idx - node * kLdE;
            if (f < 2 * kKhE) {
                const int64_t o = cm_index<kKhE>(n0 + node, f);   // chunk-major node rows
                a.dU[o] = naccS[idx];
                a.dV[o] = naccR[idx];
            }
        }
    }
    info = ninfo;
    }
}

// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256, 2) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_enc_edge_bwd(EncEdgeBwdArgs a) {
    const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
    const int blk = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (blk >= a.n_eblocks) return;
    const int64_t e = (int64_t)blk * 32 + j;
    const uint32_t* mb = a.zmask + (int64_t)blk * 4 * 3 * 64;   // z1, z2, z3, cr > 0 bits
    float* const db = a.dz4 + (int64_t)blk * kCmBlk;          // chunk-major outputs
    const int64_t cmo = (int64_t)blk * kCmBlk;
    f32x16 D[5], E[5];
    zero_tiles(D);
    tgemm_stream_acc<5, kKhE, kLdE>(a.dA + e * kLdE + kKhE * h, D, a.w1at, lane);  // dc_r = dA·W1aᵀ
    apply_pos_bits<5>(mb + 9 * 64, D, lane, a.scale);   // relu + dropout of c_r
    // each gradient is stored piecewise beside the next layer's MFMAs
    zero_tiles(E);
    tchain_acc<5, 5, 12, kLdE>(D, E, a.rm3t, lane, [&](int p) { store_cm_piece<5>(db, D, lane, p); });
    apply_pos_bits<5>(mb + 6 * 64, E, lane, 1.f);
    zero_tiles(D);
    tchain_acc<5, 5, 12, kLdE>(E, D, a.rm2t, lane, [&](int p) { store_cm_piece<5>(a.dz3 + cmo, E, lane, p); });
    apply_pos_bits<5>(mb + 3 * 64, D, lane, 1.f);
    zero_tiles(E);
    tchain_acc<5, 5, 12, kLdE>(D, E, a.rm1t, lane, [&](int p) { store_cm_piece<5>(a.dz2 + cmo, D, lane, p); });
    apply_pos_bits<5>(mb, E, lane, 1.f);
    store_cm<5>(a.dz1 + cmo, E, lane, true);
    (void)h;
}

// The same backward chain in split-bf16 math: NC 32-edge column tiles per wave (kernels_fwd.hip
// k_enc_edge_x6). dA rows (row-major) are loaded whole up front as half rows (lane half h: features
// 76h .. 76h+75, image kind kh = 76), into the registers the second layer's output uses later.
// B16 (bf16 math): dA is read and dz4..dz1 (the weight gradients' Y operands only) are stored as bf16
// (exact, §3g).
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
template <int NC, int NP = 3, bool B16 = false, int NW = 0>
__global__ __launch_bounds__(NW > 4 ? 64 * NW : 256, NC == 1 && NW <= 4 ? 2 : 1) void k_enc_edge_bwd_x6(EncEdgeBwdArgs a) {
    constexpr int kWaves = NW > 4 ? NW : 4;   // waves per workgroup (NW > 0: all share one weight ring)
    const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
    const int blk0 = (blockIdx.x * kWaves + (threadIdx.x >> 6)) * NC;
    if (NW == 0 && blk0 >= a.n_eblocks) return;   // NW > 0: no early exit (tgemm_x6_wg)
    __shared__ uint4 wring[NW > 0 ? kWgRing * kWgSlot : 1];
    const WgRing<NW> wr{wring, __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6))};
    f32x16 D[NC][5], E[NC][5];
    if constexpr (B16 && NP == 1) {
        // bf16 math over bf16-stored dA: the stored element pairs are the MFMA operand words as they are
        struct Rows {
            uint2 raw[NC][kKhE / 4];
            __device__ uint32_t word(int c, int kb, int m) const {
                const int q = 2 * kb + (m >> 1);
                return q < kKhE / 4 ? ((m & 1) ? raw[c][q].y : raw[c][q].x) : 0u;
            }
            __device__ void operator()(int c, int kb, float (&v)[8]) const {   // (unused: word() is taken)
                const float4 x = unpack4_bf16(raw[c][2 * kb]);
                const float4 y = 2 * kb + 1 < kKhE / 4 ? unpack4_bf16(raw[c][2 * kb + 1]) : make_float4(0.f, 0.f, 0.f, 0.f);
                v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
                v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
            }
        } rows;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int64_t e = (int64_t)min(blk0 + c, a.n_eblocks - 1) * 32 + j;
            const uint2* row = reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(a.dA) + e * kLdE + kKhE * h);
#pragma unroll
            for (int q = 0; q < kKhE / 4; ++q) rows.raw[c][q] = row[q];
            zero_tiles(D[c]);
        }
        tgemm_x6s<5, (kKhE + 7) / 8, NC, 6, NP, NW>(rows, D, a.x_w1at, lane, wr);   // dc_r = dA·W1aᵀ
    } else {
        float4 raw[NC][kKhE / 4];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int64_t e = (int64_t)min(blk0 + c, a.n_eblocks - 1) * 32 + j;
            if constexpr (B16) {
                const uint2* row = reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(a.dA) + e * kLdE + kKhE * h);
#pragma unroll
                for (int q = 0; q < kKhE / 4; ++q) raw[c][q] = unpack4_bf16(row[q]);
            } else {
                const float4* row = reinterpret_cast<const float4*>(a.dA + e * kLdE + kKhE * h);
#pragma unroll
                for (int q = 0; q < kKhE / 4; ++q) raw[c][q] = row[q];
            }
            zero_tiles(D[c]);
        }
        tgemm_x6s<5, (kKhE + 7) / 8, NC, 6, NP, NW>(
            [&](int c, int kb, float (&v)[8]) {
                const float4 x = raw[c][2 * kb];
                const float4 y = 2 * kb + 1 < kKhE / 4 ? raw[c][2 * kb + 1] : make_float4(0.f, 0.f, 0.f, 0.f);
                v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
                v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
            },
            D, a.x_w1at, lane, wr);   // dc_r = dA·W1aᵀ
    }
    auto save = [&](float* base, const f32x16 (&Z)[NC][5]) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (blk0 + c >= a.n_eblocks) break;
            if constexpr (B16) store_cm_b16<5>(reinterpret_cast<uint16_t*>(base) + (int64_t)(blk0 + c) * kCmBlk, Z[c], lane, true);
            else store_cm<5>(base + (int64_t)(blk0 + c) * kCmBlk, Z[c], lane, true);
        }
    };
    auto bits = [&](int layer, f32x16 (&Z)[NC][5], float scale) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int blk = min(blk0 + c, a.n_eblocks - 1);
            apply_pos_bits<5>(a.zmask + (int64_t)blk * 4 * 3 * 64 + layer * 3 * 64, Z[c], lane, scale);
        }
    };
    auto zero2 = [&](f32x16 (&Z)[NC][5]) {
#pragma unroll
        for (int c = 0; c < NC; ++c) zero_tiles(Z[c]);
    };
    bits(3, D, a.scale);   // relu + dropout of c_r
    save(a.dz4, D);
    zero2(E);
    tchain_x6s<5, 10, 5, NC, 6, NP, NW>(D, E, a.x_rm3t, lane, wr);
    bits(2, E, 1.f);
    save(a.dz3, E);
    zero2(D);
    tchain_x6s<5, 10, 5, NC, 6, NP, NW>(E, D, a.x_rm2t, lane, wr);
    bits(1, D, 1.f);
    save(a.dz2, D);
    zero2(E);
    tchain_x6s<5, 10, 5, NC, 6, NP, NW>(D, E, a.x_rm1t, lane, wr);
    bits(0, E, 1.f);
    save(a.dz1, E);
    (void)h;
}

__global__ __launch_bounds__(256, 2) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_enc_node_bwd(EncNodeBwdArgs a) {
    const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
    const int nb = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (nb * 32 >= a.n_nodes) return;
    const int n = nb * 32 + j;
    const bool valid = n < a.n_nodes;
    const int64_t bN = (int64_t)nb * kCmBlkN;   // chunk-major node block
    f32x16 D[4], Z[4], E[4];
    if (a.wo1ct) {   // dc_o = (Σ_s do1_s)·Wo1cᵀ (fp32 MFMA), steps summed in backward order S-1..0
        load_cm<4>(a.do1 + (int64_t)(a.S - 1) * a.do1_step + bN, E, lane);
        for (int s = a.S - 2; s >= 0; --s) {
            load_cm<4>(a.do1 + (int64_t)s * a.do1_step + bN, Z, lane);
#pragma unroll
            for (int t = 0; t < 4; ++t) E[t] += Z[t];
        }
        store_cm<4>(a.dco + bN, E, lane, valid);   // Σ_s do1_s: Y of the Wo1c weight gradient
        zero_tiles(D);
        tchain_acc<4, 4, 4, kLdN>(E, D, a.wo1ct, lane);
    } else {
        load_cm<4>(a.dco + bN, D, lane);
    }
    load_cm<4>(a.co + bN, Z, lane);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) D[t][r] = Z[t][r] > 0.f ? D[t][r] * a.scale : 0.f;
    store_cm<4>(a.dzo2 + bN, D, lane, valid);
    zero_tiles(E);
    tchain_acc<4, 4, 4, kLdN>(D, E, a.om1t, lane);
    if (a.zo1) {
        load_cm<4>(a.zo1 + bN, Z, lane);
    } else {   // the forward's own first-layer arithmetic (k_enc_node), not a stored row
        const float4 p = reinterpret_cast<const float4*>(a.pos)[valid ? n : a.n_nodes - 1];
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = rho(r, 0) + 4 * h + 32 * t;
                Z[t][r] = relu(dense2(p.y, p.z, a.w_om0[f], a.w_om0[128 + f], a.b_om0[f]));
            }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) E[t][r] = Z[t][r] > 0.f ? E[t][r] : 0.f;
    store_cm<4>(a.dzo1 + bN, E, lane, valid);
}

// ------------------------------------------------------------------------------------------------
hipError_t launch_node_bwd(const NodeBwdArgs& a, int math, hipStream_t st) {
    if ((math == MATH_X6 || math == MATH_BF16) && a.dco_sum && team_blocks((a.n_nodes + 31) / 32))
        return a.n16 ? hipErrorInvalidValue : launch_node_bwd_team(a, math, st);   // team kernels: fp32 arrays
    if (a.n16 && math != MATH_BF16) return hipErrorInvalidValue;
    if (math == MATH_BF16) {
        const int w = (a.n_nodes + 31) / 32;
        if (a.n16) hipLaunchKernelGGL((k_node_bwd_x6<1, 1, 4, true>), dim3((w + 3) / 4), dim3(256), 0, st, a);
        else hipLaunchKernelGGL((k_node_bwd_x6<1, 1, 4>), dim3((w + 3) / 4), dim3(256), 0, st, a);
        return hipGetLastError();
    }
    if (math == MATH_X6) {
        // one 32-node column tile per wave at two waves per SIMD, weight images shared by the
        // workgroup's 4 waves (0.474 ms vs 0.557 for two tiles per wave at one wave per SIMD with
        // per-wave rings, 0.630 for that with the shared ring: 393K nodes)
        constexpr int NC = 1, NW = 4;
        const int w2 = ((a.n_nodes + 31) / 32 + NC - 1) / NC;
        hipLaunchKernelGGL((k_node_bwd_x6<NC, 3, NW>), dim3((w2 + 3) / 4), dim3(256), 0, st, a);
        return hipGetLastError();
    }
    const int waves = (a.n_nodes + 31) / 32;
    hipLaunchKernelGGL(k_node_bwd, dim3((waves + 3) / 4), dim3(256), 0, st, a);
    return hipGetLastError();
}
// One propagation step, edge side, backward, in split-bf16 math (x6; wave-tiles of ≤ 16 nodes).
// As k_edge_fwd_x6: lane (i, h) holds edge i, features 76h + 8kb + e of k-block kb; the A operand
// is dh2pre = G3[receiver] ⊙ [h2 > 0] built from the G3 loads, W2ᵀ (x6 image) is the LDS B operand.
// dh1pre = dh1 ⊙ [h1 > 0] goes through one one-hot product (rows 0-15 receivers → dV, 16-31 senders
// → dU; 3 bf16 MFMAs per 16 edges per feature tile); dA is rebuilt after the step loop (k_dA_x6).
// Diagnosis builds keep a per-step dA form (stores on step S−1, read-add-writes after, in the
// rebuild's order: bitwise the same dA) for A/B: it made this kernel 2.6x slower (§3f). G3 rows run
// kX6Pf k-blocks ahead, carried across blocks.
#ifndef SPWGNN_EBWD_PF
#define SPWGNN_EBWD_PF 2
#endif
#ifndef SPWGNN_EBWD_PF_B16
#define SPWGNN_EBWD_PF_B16 5
#endif
#ifndef SPWGNN_DA_PF_B16
#define SPWGNN_DA_PF_B16 5
#endif
#ifndef SPWGNN_DA_INTERLEAVE
#define SPWGNN_DA_INTERLEAVE 1
#endif
// The 8 waves of a workgroup take neighbouring blocks (interleave); LOCKSTEP adds a workgroup barrier
// after each round of 8 blocks so they stay at the same (block round, step): blocks of one tile then
// gather the same receiver rows at the same time (L1/L2 hits) instead of drifting apart
#ifndef SPWGNN_DA_LOCKSTEP
#define SPWGNN_DA_LOCKSTEP 1
#endif
// the k-block of the wide edge backward's loop that builds the one-hot node operand (≥ 10: after the loop;
// A/B on one box, bitwise equal: kb 5 vs after the loop config 3 41.3 → 40.9 ms, config 4 34.2 → 34.0)
#ifndef SPWGNN_OH_KB
#define SPWGNN_OH_KB 5
#endif
// diagnosis builds only (wrong results, timing): 1 = every G3 row is node 0's (cache hits),
// 2 = also no mask-word loads (constants)
#ifndef SPWGNN_DA_DBG
#define SPWGNN_DA_DBG 0
#endif
// N16 (bf16 math, §3g node side): dU, dV stored as bf16
template <bool ACCUM, bool NODA = false, int NP = 3, int DBG = 0, bool N16 = false>   // DBG 3 (diagnosis): G3 rows of the tile's first node
__global__ __launch_bounds__(512, 1) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_edge_bwd_x6(EdgeBwdArgs a) {
    constexpr int PF = NP == 1 ? SPWGNN_EBWD_PF_B16 : SPWGNN_EBWD_PF, kWaves = 8;   // bf16: see k_dA_x6
    __shared__ uint4 wl[50 * 3 * 64];   // W2ᵀ x6 image: [kb·5 + T][part][lane]
    for (int idx = threadIdx.x; idx < 50 * 3 * 64; idx += blockDim.x) wl[idx] = a.x_w2t[idx];
    __syncthreads();
    const int lane = threadIdx.x & 63, h = lane >> 5, i = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int4* wtiles = reinterpret_cast<const int4*>(a.wtile);
    const int wstep = gridDim.x * kWaves;
    const WlBases wlb(wl + lane);
    struct Pre { int d, s; uint32_t w[5]; };
    auto load_pre = [&](int blk) {
        Pre p;
        const int64_t e = (int64_t)blk * 32 + i;
        p.d = a.edst[e];
        p.s = a.esrc[e];
        load_m2(a.mask2 + (int64_t)blk * kM2Blk, i, p.w);
        return p;
    };
    auto g_of = [&](int d, int n0) {
        return reinterpret_cast<const float4*>(a.G3 + cm_index<kKhE>(DBG == 3 ? n0 : (d >= 0 ? d : n0), 0) + h * 128);
    };
    struct KB { float4 g[2]; };
    auto ld = [&](const float4* G4, int kb, KB& r) {
#pragma unroll
        for (int c = 0; c < 2; ++c) r.g[c] = G4[64 * min(2 * kb + c, kKhE / 4 - 1)];
    };
    int wt = blockIdx.x * kWaves + wave;
    if (wt >= a.n_wtiles) return;
    int4 info = wtiles[wt];
    Pre cur = load_pre(info.x);
    const float4* G4 = g_of(cur.d, info.z);
    KB ring[PF];
#pragma unroll
    for (int k = 0; k < PF; ++k) ld(G4, k, ring[k]);
    for (; wt < a.n_wtiles; wt += wstep) {
    const int fb = info.x, nb = info.y, n0 = info.z, nn = info.w;
    const int4 ninfo = wtiles[min(wt + wstep, a.n_wtiles - 1)];
    const int key = i < 16 ? n0 + i : n0 + i - 16;   // one-hot rows: receivers, then senders
    const int kbits = i < 16 ? 0 : 16;                 // ... their half of a packed local-id word
    f32x16 nacc[5];
    zero_tiles(nacc);
    for (int bb = 0; bb < nb; ++bb) {
        const int blk = fb + bb;
        const int nblk = bb + 1 < nb ? blk + 1 : ninfo.x;
        const int nn0 = bb + 1 < nb ? n0 : ninfo.z;
        const Pre nxt = load_pre(nblk);
        const int d = cur.d;
        const bool valid = d >= 0;
        const uint32_t* m1 = a.mask1 + (int64_t)blk * kLdE + i;
        uint32_t m1w[5];   // loaded a few k-blocks before the dh1pre masking uses them
        uint32_t w[5];
#pragma unroll
        for (int t = 0; t < 5; ++t) w[t] = valid ? cur.w[t] : 0u;
        // this lane's 76 feature bits (features 76h + 0..75): a 64-bit low part and a 12-bit tail
        const uint64_t mlo = h == 0 ? ((uint64_t)w[1] << 32 | w[0])
                                    : ((uint64_t)w[4] << 52 | (uint64_t)w[3] << 20 | (w[2] >> 12));
        const uint32_t mhi = h == 0 ? (w[2] & 0xfffu) : (w[4] >> 12);
        const float4* NG4 = nullptr;
        // one-hot [node row][edge]: element e of half h ↔ edge rho(8s + e, h)
        const int s_ = cur.s;
        uint32_t oh2[2][4];
#if SPWGNN_ONEHOT_BPERM
        // the edges' tile-local ids packed (receiver | sender << 16; all ones where an id is not one of
        // the tile's 16 nodes, padding edges included), fetched per element with one ds_bpermute —
        // four readlanes and their selects before; the same 0/1 operand. Built inside the k-block loop
        // (SPWGNN_OH_KB) so the permute latency hides behind its MFMAs.
        auto build_oh = [&]() {
            const uint32_t ld_ = (uint32_t)(d - n0) < 16u ? (uint32_t)(d - n0) : 0xffffu;
            const uint32_t ls_ = (uint32_t)(s_ - n0) < 16u ? (uint32_t)(s_ - n0) : 0xffffu;
            const int pk = (int)(ld_ | (ls_ << 16));
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    uint32_t wv = 0u;
#pragma unroll
                    for (int q = 0; q < 2; ++q) {
                        const uint32_t v = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * rho(8 * s + 2 * m + q, h), pk);
                        wv |= (__builtin_amdgcn_ubfe(v, kbits, 16) == (uint32_t)(i & 15) ? 0x3F80u : 0u) << (16 * q);
                    }
                    oh2[s][m] = wv;
                }
        };
#endif
        f32x16 acc[5];
        zero_tiles(acc);
#pragma unroll
        for (int kb = 0; kb < 10; ++kb) {
            if (kb == 7) {
#pragma unroll
                for (int t = 0; t < 5; ++t) m1w[t] = m1[32 * t];
            }
#if SPWGNN_ONEHOT_BPERM && SPWGNN_OH_KB < 10
            if (kb == SPWGNN_OH_KB) build_oh();
#endif
            KB& cr = ring[kb % PF];
            float xv[8];
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const int q = 2 * kb + c;
                const uint32_t bits = q < 16 ? (uint32_t)(mlo >> (4 * q)) : (q < 19 ? mhi >> (4 * q - 64) : 0u);
                xv[4 * c + 0] = mask_bit(cr.g[c].x, bits, 0);
                xv[4 * c + 1] = mask_bit(cr.g[c].y, bits, 1);
                xv[4 * c + 2] = mask_bit(cr.g[c].z, bits, 2);
                xv[4 * c + 3] = mask_bit(cr.g[c].w, bits, 3);
            }
            uint32_t hw[4], mw[4], lw[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) split2(xv[2 * m], xv[2 * m + 1], hw[m], mw[m], lw[m]);
            if (kb + PF < 10) {
                ld(G4, kb + PF, cr);
            } else {
                if (kb + PF == 10) NG4 = g_of(nxt.d, nn0);
                ld(NG4, kb + PF - 10, cr);
            }
            bf16x8 ap[3];
            ap[0] = as_bf16x8(make_uint4(hw[0], hw[1], hw[2], hw[3]));
            ap[1] = as_bf16x8(make_uint4(mw[0], mw[1], mw[2], mw[3]));
            ap[2] = as_bf16x8(make_uint4(lw[0], lw[1], lw[2], lw[3]));
#pragma unroll
            for (int T = 0; T < 5; ++T) {   // (interleaved tile groups as in k_dA_x6 spill here: 0.615 -> 0.637 ms)
                const int u = (kb * 5 + T) * 3 * 64;
                bf16x8 bp[3];
                bp[0] = as_bf16x8(wlb.at(u));
                bp[1] = as_bf16x8(wlb.at(u + 64));
                bp[2] = as_bf16x8(wlb.at(u + 128));
                acc[T] = mfma32_x6<NP>(ap, bp, acc[T]);
            }
            __builtin_amdgcn_sched_barrier(0);   // no motion across k-blocks (register pressure)
        }
        // dh1pre = dh1 ⊙ [h1 > 0]  (C layout: lane = feature 32t+i, rows = edges rho(r,h))
#pragma unroll
        for (int t = 0; t < 5; ++t) {
            const uint32_t mh = m1w[t] >> (4 * h);   // bit rho(r, 0) = edge rho(r, h)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[t][r] = mask_bit(acc[t][r], mh, rho(r, 0));
        }
        float* dArow = a.dA + (int64_t)blk * 32 * kLdE + i;
#if SPWGNN_ONEHOT_BPERM && SPWGNN_OH_KB >= 10
        build_oh();
#endif
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            uint32_t oh[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) {
#if SPWGNN_ONEHOT_BPERM
                oh[m] = oh2[s][m];
#else
                uint32_t wv = 0u;
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int e = 2 * m + q;
                    const int d0 = __builtin_amdgcn_readlane(d, rho(8 * s + e, 0));
                    const int d1 = __builtin_amdgcn_readlane(d, rho(8 * s + e, 1));
                    const int s0 = __builtin_amdgcn_readlane(s_, rho(8 * s + e, 0));
                    const int s1 = __builtin_amdgcn_readlane(s_, rho(8 * s + e, 1));
                    const int node = i < 16 ? (h ? d1 : d0) : (h ? s1 : s0);
                    wv |= (node == key ? 0x3F80u : 0u) << (16 * q);
                }
                oh[m] = wv;
#endif
            }
            const bf16x8 ao = as_bf16x8(make_uint4(oh[0], oh[1], oh[2], oh[3]));
#pragma unroll
            for (int t = 0; t < 5; ++t) {
                uint32_t hw[4], mw[4], lw[4];
#pragma unroll
                for (int m = 0; m < 4; ++m) split2(acc[t][8 * s + 2 * m], acc[t][8 * s + 2 * m + 1], hw[m], mw[m], lw[m]);
                if constexpr (NP == 3) {
                    nacc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ao, as_bf16x8(make_uint4(lw[0], lw[1], lw[2], lw[3])), nacc[t], 0, 0, 0);
                    nacc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ao, as_bf16x8(make_uint4(mw[0], mw[1], mw[2], mw[3])), nacc[t], 0, 0, 0);
                }
                nacc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ao, as_bf16x8(make_uint4(hw[0], hw[1], hw[2], hw[3])), nacc[t], 0, 0, 0);
                // dA rows of this k-block's 8 registers, issued beside the MFMAs
#pragma unroll
                for (int r = 8 * s; r < 8 * s + 8; ++r) {
                    float* p = dArow + rho(r, h) * kLdE + 32 * t;
                    if constexpr (NODA) {
                    } else if (ACCUM) *p += acc[t][r];   // the wave owns the block: plain read-add-write
                    else *p = acc[t][r];
                }
            }
        }
        cur = nxt;
        G4 = NG4;
    }
    // nacc[t] reg r = row rho(r,h): rows 0..15 receiver nodes, 16..31 sender nodes
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row = rho(r, h);
        const int node = row & 15;
        if (node < nn) {
            float* o = row < 16 ? a.dV : a.dU;   // chunk-major node rows
#pragma unroll
            for (int t = 0; t < 5; ++t)
                if (32 * t + i < 2 * kKhE) {
                    if constexpr (N16) store_b16(o, cm_index<kKhE>(n0 + node, 32 * t + i), nacc[t][r]);
                    else o[cm_index<kKhE>(n0 + node, 32 * t + i)] = nacc[t][r];
                }
        }
    }
    info = ninfo;
    }
}

hipError_t launch_edge_bwd(const EdgeBwdArgs& a, int math, hipStream_t st) {
    if (math != MATH_F32 && a.nw_max <= 16 && a.no_dA && team_blocks(a.n_wtiles))   // small batches
        return a.n16 ? hipErrorInvalidValue : launch_edge_bwd_team(a, math, st);   // team kernels: fp32 dU/dV
    if (a.n16 && (math != MATH_BF16 || a.nw_max > 16 || !a.no_dA)) return hipErrorInvalidValue;
    if (math != MATH_F32 && a.nw_max <= 16) {
        const dim3 g(edge_grid(a.n_wtiles, 8)), b(512);   // two waves per SIMD
        // no_dA: dA = Σ_s dh1pre_s is rebuilt once after the step loop by k_dA_x6 (launch_dA)
        if (a.no_dA) {
#ifdef SPWGNN_DIAG
            static const int edbg = getenv("SPWGNN_EBWD_DBG") ? atoi(getenv("SPWGNN_EBWD_DBG")) : 0;
            if (math == MATH_BF16 && edbg == 3) {
                hipLaunchKernelGGL((k_edge_bwd_x6<false, true, 1, 3>), g, b, 0, st, a);
                return hipGetLastError();
            }
#endif
            if (math == MATH_BF16 && a.n16) hipLaunchKernelGGL((k_edge_bwd_x6<false, true, 1, 0, true>), g, b, 0, st, a);
            else if (math == MATH_BF16) hipLaunchKernelGGL((k_edge_bwd_x6<false, true, 1>), g, b, 0, st, a);
            else hipLaunchKernelGGL((k_edge_bwd_x6<false, true>), g, b, 0, st, a);
            return hipGetLastError();
        }
#ifdef SPWGNN_DIAG   // per-step dA read-add-writes (SPWGNN_DA_RMW A/B builds only: 2.6x slower, §3f)
        if (math != MATH_X6) return hipErrorInvalidValue;
        if (a.dA_accumulate) hipLaunchKernelGGL((k_edge_bwd_x6<true>), g, b, 0, st, a);
        else hipLaunchKernelGGL((k_edge_bwd_x6<false>), g, b, 0, st, a);
        return hipGetLastError();
#else
        return hipErrorInvalidValue;
#endif
    }
    if (a.nw_max <= 16) {
        if (a.dA_accumulate)
            hipLaunchKernelGGL((k_edge_bwd<true, true>), dim3(edge_grid(a.n_wtiles)), dim3(64 * kEdgeWaves), 0, st, a);
        else
            hipLaunchKernelGGL((k_edge_bwd<true, false>), dim3(edge_grid(a.n_wtiles)), dim3(64 * kEdgeWaves), 0, st, a);
    } else {
        const size_t lds = edge_bwd_lds_per_wave(a.nw_max) * a.wpg;
        const dim3 g((a.n_wtiles + a.wpg - 1) / a.wpg), b(64 * a.wpg);
        if (math == MATH_BF16) {
            if (a.dA_accumulate) hipLaunchKernelGGL((k_edge_bwd<false, true, true>), g, b, lds, st, a);
            else hipLaunchKernelGGL((k_edge_bwd<false, false, true>), g, b, lds, st, a);
        } else if (a.dA_accumulate) {
            hipLaunchKernelGGL((k_edge_bwd<false, true>), g, b, lds, st, a);
        } else {
            hipLaunchKernelGGL((k_edge_bwd<false, false>), g, b, lds, st, a);
        }
    }
    return hipGetLastError();
}

// dA = Σ_s dh1pre_s, rebuilt once after the backward step loop instead of accumulated by every
// step's edge kernel (float atomics into a row-major HBM array: the edge backward's bound, DESIGN.md
// §10). Per 32-edge block a wave recomputes each step's dh1pre_s = ((G3_s[receiver] ⊙ [h2_s > 0])·W2ᵀ)
// ⊙ [h1_s > 0] exactly as k_edge_bwd_x6 does (same operand order, same k order: bit-identical
// values), sums the steps in registers in the order the atomics did (S-1 first, then S-2 .. 0: the
// same fp32 sums, bit-identical dA) and stores dA once with plain stores.
// W2ᵀ (x6 image) is the LDS B operand; blocks are independent (no tile structure needed).
template <int NP = 3, bool B16 = false>
__global__ __launch_bounds__(512, 1) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_dA_x6(DaArgs a) {
    // bf16 math (NP = 1): a k-block is 5 MFMAs, so the G3 rows run further ahead to cover HBM latency
    constexpr int kWaves = 8, PF = NP == 1 ? SPWGNN_DA_PF_B16 : 2;
    static_assert(10 % PF == 0, "ring slots carry over between (block, step) pairs");
    __shared__ uint4 wl[50 * 3 * 64];   // W2ᵀ x6 image: [kb·5 + T][part][lane]
    for (int idx = threadIdx.x; idx < 50 * 3 * 64; idx += blockDim.x) wl[idx] = a.x_w2t[idx];
    __syncthreads();
    const int lane = threadIdx.x & 63, h = lane >> 5, i = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const WlBases wlb(wl + lane);
#if SPWGNN_DA_INTERLEAVE
    // a contiguous block range per WORKGROUP, its waves interleaved (wave w: blocks w, w + 8, …): the
    // 8 waves of a CU work on neighbouring blocks at once, so the receiver rows of a tower whose
    // blocks they share (N ≥ 9: several blocks per tower) are gathered from L1/L2 by all of them, where
    // a contiguous range per wave re-gathered every step's rows for each of the tower's blocks
    // (config 3: 21 GB of traffic per launch against ≈ 7.5 GB compulsory)
    constexpr int kStride = kWaves;
    const int perw = ((a.n_eblocks + gridDim.x - 1) / gridDim.x + kWaves - 1) / kWaves * kWaves;
    const int b0 = blockIdx.x * perw + wave, b1 = min(blockIdx.x * perw + perw, a.n_eblocks);
    // block rounds of this workgroup (wave 0 has the most) and of this wave
    const int wg_b0 = blockIdx.x * perw;
    const int rounds = SPWGNN_DA_LOCKSTEP ? max(0, (b1 - wg_b0 + kWaves - 1) / kWaves) : 0;
    const int mine = SPWGNN_DA_LOCKSTEP ? max(0, (b1 - b0 + kWaves - 1) / kWaves) : 0;
#else
    // a contiguous range of blocks per wave: a tower's blocks (same receiver rows) stay on one CU
    constexpr int kStride = 1;
    const int nw = gridDim.x * kWaves, gw = blockIdx.x * kWaves + wave;
    const int per = (a.n_eblocks + nw - 1) / nw;
    const int b0 = gw * per, b1 = min(b0 + per, a.n_eblocks);
#endif
#if SPWGNN_DA_INTERLEAVE && SPWGNN_DA_LOCKSTEP
    // every wave passes `rounds` barriers: one per block it sums, the rest after its last block
    auto tail_barriers = [&](int done) {
        for (int k = done; k < rounds; ++k) __syncthreads();
    };
    if (b0 >= b1) {
        tail_barriers(0);
        return;
    }
#else
    if (b0 >= b1) return;
#endif
    // one (block, step) pair: its receiver row pointer (G3 of that step) and its mask words
    struct Pair { const float4* G4; uint32_t w[5], m1w[5]; };
    auto load_pair = [&](int blk, int s, int d) {
        Pair p;
        const bool valid = d >= 0;
        p.G4 = reinterpret_cast<const float4*>(a.G3 + s * a.g3_step + cm_index<kKhE>(valid && SPWGNN_DA_DBG == 0 ? d : 0, 0) + h * 128);
        const uint32_t* m1 = a.mask1 + s * a.m1_step + (int64_t)blk * kLdE + i;
        if (SPWGNN_DA_DBG >= 2) {
#pragma unroll
            for (int t = 0; t < 5; ++t) p.w[t] = p.m1w[t] = valid ? 0x5a5a5a5au ^ (uint32_t)(blk * 5 + t) : 0u;
            return p;
        }
        load_m2(a.mask2 + s * a.m2_step + (int64_t)blk * kM2Blk, i, p.w);
#pragma unroll
        for (int t = 0; t < 5; ++t) {
            p.w[t] = valid ? p.w[t] : 0u;
            p.m1w[t] = m1[32 * t];
        }
        return p;
    };
    struct KB { float4 g[2]; };
    auto ld = [&](const float4* G4, int kb, KB& r) {
#pragma unroll
        for (int c = 0; c < 2; ++c) r.g[c] = G4[64 * min(2 * kb + c, kKhE / 4 - 1)];
    };
    int blk = b0, s = a.S - 1;
    int d = a.edst[(int64_t)blk * 32 + i];
    Pair cur = load_pair(blk, s, d);
    KB ring[PF];
#pragma unroll
    for (int k = 0; k < PF; ++k) ld(cur.G4, k, ring[k]);
    f32x16 dacc[5];
    zero_tiles(dacc);
    for (;;) {
        // the next pair (steps S-1 .. 0 of a block, then the next block; clamped at the range end)
        const bool last_step = s == 0;
        const bool has_next = !last_step || blk + kStride < b1;
        const int nblk = last_step ? (blk + kStride < b1 ? blk + kStride : blk) : blk;
        const int ns = last_step ? a.S - 1 : s - 1;
        const int nd = last_step ? a.edst[(int64_t)nblk * 32 + i] : d;
        const Pair nxt = load_pair(nblk, max(ns, 0), nd);
        const uint64_t mlo = h == 0 ? ((uint64_t)cur.w[1] << 32 | cur.w[0])
                                    : ((uint64_t)cur.w[4] << 52 | (uint64_t)cur.w[3] << 20 | (cur.w[2] >> 12));
        const uint32_t mhi = h == 0 ? (cur.w[2] & 0xfffu) : (cur.w[4] >> 12);
        f32x16 acc[5];
        zero_tiles(acc);
#pragma unroll
        for (int kb = 0; kb < 10; ++kb) {
            KB& cr = ring[kb % PF];
            float xv[8];
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const int q = 2 * kb + c;
                const uint32_t bits = q < 16 ? (uint32_t)(mlo >> (4 * q)) : (q < 19 ? mhi >> (4 * q - 64) : 0u);
                xv[4 * c + 0] = mask_bit(cr.g[c].x, bits, 0);
                xv[4 * c + 1] = mask_bit(cr.g[c].y, bits, 1);
                xv[4 * c + 2] = mask_bit(cr.g[c].z, bits, 2);
                xv[4 * c + 3] = mask_bit(cr.g[c].w, bits, 3);
            }
            uint32_t hw[4], mw[4], lw[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) split2(xv[2 * m], xv[2 * m + 1], hw[m], mw[m], lw[m]);
            if (kb + PF < 10) ld(cur.G4, kb + PF, cr);
            else ld(nxt.G4, kb + PF - 10, cr);
            bf16x8 ap[3];
            ap[0] = as_bf16x8(make_uint4(hw[0], hw[1], hw[2], hw[3]));
            ap[1] = as_bf16x8(make_uint4(mw[0], mw[1], mw[2], mw[3]));
            ap[2] = as_bf16x8(make_uint4(lw[0], lw[1], lw[2], lw[3]));
            // output tiles in groups {0, 1}, {2, 3, 4}, products interleaved within a group
            auto group = [&](auto NTc, int T0) {
                constexpr int NT = decltype(NTc)::value;
                bf16x8 bp[NT][3];
#pragma unroll
                for (int v = 0; v < NT; ++v) {
                    const int u = (kb * 5 + T0 + v) * 3 * 64;
#pragma unroll
                    for (int p = 0; p < NP; ++p) bp[v][p] = as_bf16x8(wlb.at(u + 64 * p));
                }
                mfma32_x6_group<NP, NT>(ap, bp, acc + T0);
            };
            group(std::integral_constant<int, 2>{}, 0);
            group(std::integral_constant<int, 3>{}, 2);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int t = 0; t < 5; ++t) {
            const uint32_t mh = cur.m1w[t] >> (4 * h);   // bit rho(r, 0) = edge rho(r, h)
#pragma unroll
            for (int r = 0; r < 16; ++r) dacc[t][r] += mask_bit(acc[t][r], mh, rho(r, 0));
        }
        if (last_step) {   // the block's S steps are summed: one plain store of its dA rows
            if constexpr (B16) {   // bf16 math: dA feeds MFMA operands only (§3g)
                __bf16* dArow = reinterpret_cast<__bf16*>(a.dA) + (int64_t)blk * 32 * kLdE + i;
#pragma unroll
                for (int t = 0; t < 5; ++t)
#pragma unroll
                    for (int r = 0; r < 16; ++r) dArow[rho(r, h) * kLdE + 32 * t] = (__bf16)dacc[t][r];
            } else {
                float* dArow = a.dA + (int64_t)blk * 32 * kLdE + i;
#pragma unroll
                for (int t = 0; t < 5; ++t)
#pragma unroll
                    for (int r = 0; r < 16; ++r) dArow[rho(r, h) * kLdE + 32 * t] = dacc[t][r];
            }
            zero_tiles(dacc);
#if SPWGNN_DA_INTERLEAVE && SPWGNN_DA_LOCKSTEP
            __syncthreads();   // this block round is done on every wave
#endif
        }
        if (!has_next) break;
        blk = nblk;
        s = ns;
        d = nd;
        cur = nxt;
    }
#if SPWGNN_DA_INTERLEAVE && SPWGNN_DA_LOCKSTEP
    tail_barriers(mine);
#endif
}

hipError_t launch_dA(const DaArgs& a, int math, hipStream_t st) {
    if ((math == MATH_X6 || math == MATH_BF16) && team_blocks(a.n_eblocks)) return launch_dA_team(a, math, st);
    const dim3 g(edge_grid(a.n_eblocks, 8)), b(512);
    if (math == MATH_BF16 && a.b16) hipLaunchKernelGGL((k_dA_x6<1, true>), g, b, 0, st, a);
    else if (math == MATH_BF16) hipLaunchKernelGGL((k_dA_x6<1>), g, b, 0, st, a);
    else hipLaunchKernelGGL((k_dA_x6<3>), g, b, 0, st, a);
    return hipGetLastError();
}
hipError_t launch_enc_edge_bwd(const EncEdgeBwdArgs& a, int math, hipStream_t st) {
    // one 32-edge block per wave at two waves per SIMD, weight images shared by the workgroup's 4
    // waves (x6: 2.44 → 2.33 ms against two blocks per wave at one wave per SIMD with per-wave rings)
    constexpr int NC = 1, NW = 4, NWB = SPWGNN_ENC_NW_B16;   // bf16: waves sharing one weight pass
    if ((math == MATH_X6 || math == MATH_BF16) && team_blocks(a.n_eblocks)) return launch_enc_edge_bwd_team(a, math, st);
    const dim3 g((a.n_eblocks + 4 * NC - 1) / (4 * NC)), gb((a.n_eblocks + NWB * NC - 1) / (NWB * NC));
    if (math == MATH_BF16) {
        if (a.b16) hipLaunchKernelGGL((k_enc_edge_bwd_x6<NC, 1, true, NWB>), gb, dim3(64 * NWB), 0, st, a);
        else hipLaunchKernelGGL((k_enc_edge_bwd_x6<NC, 1, false, NW>), g, dim3(256), 0, st, a);
        return hipGetLastError();
    }
    if (math == MATH_X6) {
        constexpr int NWX = SPWGNN_ENC_NW_X6;
        const dim3 gx((a.n_eblocks + NWX * NC - 1) / (NWX * NC));
        hipLaunchKernelGGL((k_enc_edge_bwd_x6<NC, 3, false, NWX>), gx, dim3(64 * NWX), 0, st, a);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_enc_edge_bwd, dim3((a.n_eblocks + 3) / 4), dim3(256), 0, st, a);
    return hipGetLastError();
}
// The om encoder's backward in split-bf16 math: k_enc_node_bwd's two 100×100 products (Σ_s do1_s ·
// Wo1cᵀ and om.1ᵀ) on tchain_x6 instead of the f32 matrix core (one 32-node column tile per wave, two
// waves per SIMD, as k_enc_node_x6).
template <int NP, int NW = 0>
__global__ __launch_bounds__(256, 2) void k_enc_node_bwd_x6(EncNodeBwdArgs a) {
    const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
    const int nb = blockIdx.x * 4 + (threadIdx.x >> 6);
    const bool has = nb * 32 < a.n_nodes;   // NW > 0: no early exit (k_enc_node_x6)
    if (NW == 0 && !has) return;
    __shared__ uint4 wring[NW > 0 ? kWgRing * kWgSlot : 1];
    const WgRing<NW> wr{wring, __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6))};
    const int n = nb * 32 + j;
    const bool valid = has && n < a.n_nodes;
    const int64_t bN = (int64_t)(has ? nb : (a.n_nodes + 31) / 32 - 1) * kCmBlkN;   // chunk-major node block
    f32x16 D[1][4], E[1][4], Z[4];
    // Σ_s do1_s in backward step order S-1..0 (the Y of the Wo1c weight gradient)
    load_cm<4>(a.do1 + (int64_t)(a.S - 1) * a.do1_step + bN, E[0], lane);
    for (int s = a.S - 2; s >= 0; --s) {
        load_cm<4>(a.do1 + (int64_t)s * a.do1_step + bN, Z, lane);
#pragma unroll
        for (int t = 0; t < 4; ++t) E[0][t] += Z[t];
    }
    if (has) store_cm<4>(a.dco + bN, E[0], lane, valid);
    zero_tiles(D[0]);
    tchain_x6s<4, 7, 4, 1, kX6Ring, NP, NW, kHT>(E, D, kHT ? a.xh_wo1ct : a.x_wo1ct, lane, wr);   // dc_o = (Σ_s do1_s)·Wo1cᵀ
    load_cm<4>(a.co + bN, Z, lane);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) D[0][t][r] = Z[t][r] > 0.f ? D[0][t][r] * a.scale : 0.f;
    if (has) store_cm<4>(a.dzo2 + bN, D[0], lane, valid);
    zero_tiles(E[0]);
    tchain_x6s<4, 7, 4, 1, kX6Ring, NP, NW, kHT>(D, E, kHT ? a.xh_om1t : a.x_om1t, lane, wr);
    if (a.zo1) {
        load_cm<4>(a.zo1 + bN, Z, lane);
    } else {   // the forward's own first-layer arithmetic (k_enc_node_x6), not a stored row
        const float4 p = reinterpret_cast<const float4*>(a.pos)[valid ? n : a.n_nodes - 1];
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = rho(r, 0) + 4 * h + 32 * t;
                Z[t][r] = relu(dense2(p.y, p.z, a.w_om0[f], a.w_om0[128 + f], a.b_om0[f]));
            }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) E[0][t][r] = Z[t][r] > 0.f ? E[0][t][r] : 0.f;
    if (has) store_cm<4>(a.dzo1 + bN, E[0], lane, valid);
}

hipError_t launch_enc_node_bwd(const EncNodeBwdArgs& a, int math, hipStream_t st) {
    const int waves = (a.n_nodes + 31) / 32;
    if (math != MATH_F32 && a.wo1ct && a.x_wo1ct && a.x_om1t) {
        if (team_blocks(waves)) return launch_enc_node_bwd_team(a, math, st);   // small batches
        if (math == MATH_BF16) hipLaunchKernelGGL((k_enc_node_bwd_x6<1, 4>), dim3((waves + 3) / 4), dim3(256), 0, st, a);
        else hipLaunchKernelGGL((k_enc_node_bwd_x6<3, 4>), dim3((waves + 3) / 4), dim3(256), 0, st, a);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_enc_node_bwd, dim3((waves + 3) / 4), dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace spw
