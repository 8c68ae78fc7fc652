// Latency-oriented ("team") variants of the transposed-orientation chain kernels, for small batches.
//
// At the reference's own training shape (main.py:92-98: batch 32; BASELINE config 1) a chain kernel
// has one 32-edge block per tower and a wave walks its block through the whole layer chain: the
// relation encoder is 4 layers × 5 output tiles × 10 k-blocks × 6 MFMAs = 1,200 dependent-ish
// 32-cycle products on ONE wave (≈ 18 µs of matrix time alone, 37 µs measured) while 1,000 SIMDs
// idle. Here a workgroup of five waves takes one block and wave T owns output tile T of every layer:
// 60 MFMAs per layer per wave. Layer outputs are exchanged through LDS in their C layout — the C
// layout of a tile IS the B operand of the next layer's k-blocks 2t, 2t+1 (tchain_x6), so the
// exchange is a plain per-lane store and load, no transposition. Every output tile sees the same
// products in the same order as tgemm_x6 (k-blocks ascending, mfma32_x6's product order), so a
// team kernel's results are bit-identical to the one-wave-per-block kernel's.
// Weight fragments: wave T reads only its tile's steps (u = kb·NT_OUT + T) straight from the x6
// image (L2); the next layer's fragment kb is requested as soon as this layer's k-block kb has
// issued, so it arrives during the rest of the layer, the epilogue and the barrier.
#include "kernels.h"
#include <atomic>
#include <cstdlib>

namespace spw {

#ifdef SPWGNN_DIAG   // phase stamps (shader clock) of workgroup 0's waves 0 and 4: spwgnn_diag_team_stamps
__device__ unsigned long long g_team_stamps[2][32];   // 0-15 node body / step loop, 16-24 edge body
#define TEAM_STAMP(i)                                                                              \
    do {                                                                                           \
        const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();   /* 100 MHz */            \
        if (blockIdx.x == 0 && (threadIdx.x == 0 || threadIdx.x == 256)) g_team_stamps[threadIdx.x >> 8][i] = t_; \
    } while (0)
#else
#define TEAM_STAMP(i) do {} while (0)
#endif

constexpr int kTeamEdge = 5;   // waves per edge block (150-wide layers: 5 tiles of 32 features)

// LDS exchange of C-layout tiles, already split: [buf][tile][kh][part][lane] uint4 = the bf16 parts
// (split2, as tgemm_x6 splits them) of registers 8kh .. 8kh+7 of the tile — the B operand of the
// next layer's k-block 2t + kh. The producer splits its tile once; the consumers only read.
template <int NT, int NP>
struct TeamAct {
    uint4* s;
    __device__ __forceinline__ uint4* at(int buf, int t, int kh, int p, int lane) const {
        return s + (((buf * NT + t) * 2 + kh) * NP + p) * 64 + lane;
    }
    __device__ __forceinline__ void put(int buf, int t, const f32x16& x, int lane) const {
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) {
            uint32_t sp[3][4];
#pragma unroll
            for (int m = 0; m < 4; ++m) split2(x[8 * kh + 2 * m], x[8 * kh + 2 * m + 1], sp[0][m], sp[1][m], sp[2][m]);
#pragma unroll
            for (int p = 0; p < NP; ++p) *at(buf, t, kh, p, lane) = make_uint4(sp[p][0], sp[p][1], sp[p][2], sp[p][3]);
        }
    }
    // the split B operand of k-block kb (tchain_x6: registers 8(kb&1) .. +7 of tile kb>>1)
    __device__ __forceinline__ void get(int buf, int kb, uint32_t (&sp)[3][4], int lane) const {
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            const uint4 u = p < NP ? *at(buf, kb >> 1, kb & 1, p, lane) : make_uint4(0u, 0u, 0u, 0u);
            sp[p][0] = u.x; sp[p][1] = u.y; sp[p][2] = u.z; sp[p][3] = u.w;
        }
    }
};
// the exchange barrier: waits for this wave's LDS writes only (__syncthreads would also drain the
// in-flight weight-fragment refills and the global stores of the layer's epilogue)
__device__ __forceinline__ void team_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}
// B values in registers (8 per k-block) → the split operand
__device__ __forceinline__ void split8(const float (&v)[8], uint32_t (&sp)[3][4]) {
#pragma unroll
    for (int m = 0; m < 4; ++m) split2(v[2 * m], v[2 * m + 1], sp[0][m], sp[1][m], sp[2][m]);
}

// wave T's fragments of one x6 image (the parts the math uses)
template <int NKB, int NP>
struct TeamFrags {
    uint4 f[NKB][3];
    __device__ __forceinline__ void load_kb(const uint4* __restrict__ img, int nt_out, int T, int lane, int kb) {
#pragma unroll
        for (int p = 0; p < NP; ++p) f[kb][p] = img[((kb * nt_out + T) * 3 + p) * 64 + lane];
    }
    template <int K = NKB>
    __device__ __forceinline__ void load(const uint4* __restrict__ img, int nt_out, int T, int lane) {
#pragma unroll
        for (int kb = 0; kb < K; ++kb) load_kb(img, nt_out, T, lane, kb);
    }
};

// acc = Σ_kb W(kb, T)ᵀ·B(kb) (tgemm_x6's per-tile sum); getsp(kb, sp) supplies k-block kb's split
// B operand. K-block kb+1's operand is requested before kb's products issue; after k-block kb,
// next(kb) may refill f[kb] with the next layer's fragment.
// K (default: all NKB) k-blocks: a layer of fewer k-blocks may run on the first K fragments of a
// larger set (one fragment array serves a 10-k-block layer and the 7-k-block layers after it)
template <int K = -1, int NKB, int NP, class GetSp, class Next>
__device__ __forceinline__ f32x16 team_gemm(TeamFrags<NKB, NP>& F, GetSp&& getsp, Next&& next, f32x16 acc = zero16()) {
    constexpr int NK = K < 0 ? NKB : K;
    static_assert(NK <= NKB, "k-blocks beyond the fragment set");
    uint32_t sp[2][3][4];
    getsp(0, sp[0]);
#pragma unroll
    for (int kb = 0; kb < NK; ++kb) {
        bf16x8 a[3], b[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            a[p] = as_bf16x8(p < NP ? F.f[kb][p] : make_uint4(0u, 0u, 0u, 0u));
            b[p] = as_bf16x8(make_uint4(sp[kb & 1][p][0], sp[kb & 1][p][1], sp[kb & 1][p][2], sp[kb & 1][p][3]));
        }
        if (kb + 1 < NK) getsp(kb + 1, sp[(kb + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        acc = mfma32_x6<NP>(a, b, acc);
        next(kb);
        __builtin_amdgcn_sched_barrier(0);   // keep the refills behind their k-block's products
    }
    return acc;
}

// ---- one tile of the chunk-major / sign-bit helpers (store_cm, store_pos_bits, apply_pos_bits)
template <int KH>
__device__ __forceinline__ void store_cm_tile(float* __restrict__ blk, const f32x16& x, int t, int lane) {
    const int j = lane & 31, h = lane >> 5;
#pragma unroll
    for (int q = 0; q < 4; ++q)
        if (32 * t + 8 * q + 4 < 2 * KH)
            *reinterpret_cast<float4*>(blk + cm_offk<KH>(j, 32 * t + 8 * q + 4 * h)) =
                make_float4(x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]);
}
template <int KH>
__device__ __forceinline__ void store_cm_tile(float* __restrict__ blk, const f32x16& x, int t, int lane, bool valid) {
    if (valid) {
        store_cm_tile<KH>(blk, x, t, lane);
    } else {
        f32x16 z = zero16();
        store_cm_tile<KH>(blk, z, t, lane);
    }
}
template <int KH>
__device__ __forceinline__ f32x16 load_cm_tile(const float* __restrict__ blk, int t, int lane) {
    const int j = lane & 31, h = lane >> 5;
    f32x16 x;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (32 * t + 8 * q + 4 < 2 * KH) v = *reinterpret_cast<const float4*>(blk + cm_offk<KH>(j, 32 * t + 8 * q + 4 * h));
        x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
    }
    return x;
}
// a chunk-major block's half rows as the B operand (HalfRows: lane half h holds features KH·h ..)
template <int KH>
struct TeamHalf {
    static constexpr int Q = KH / 4;
    float4 raw[Q];
    __device__ __forceinline__ void load(const float* __restrict__ blk, int lane) {
        const float* p = blk + ((lane >> 5) * 32 + (lane & 31)) * 4;
#pragma unroll
        for (int q = 0; q < Q; ++q) raw[q] = *reinterpret_cast<const float4*>(p + 256 * q);
    }
    // the same block held in LDS (an explicit LDS pointer: ds_read, not flat loads)
    __device__ __forceinline__ void load_lds(const float* blk_lds, int lane) {
        typedef __attribute__((address_space(3))) const float lds_f;
        const lds_f* p = (const lds_f*)blk_lds + ((lane >> 5) * 32 + (lane & 31)) * 4;
#pragma unroll
        for (int q = 0; q < Q; ++q) raw[q] = make_float4(p[256 * q], p[256 * q + 1], p[256 * q + 2], p[256 * q + 3]);
    }
    __device__ __forceinline__ void operator()(int kb, uint32_t (&sp)[3][4]) const {
        const float4 x = raw[2 * kb];
        const float4 y = 2 * kb + 1 < Q ? raw[2 * kb + 1] : make_float4(0.f, 0.f, 0.f, 0.f);
        const float v[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
        split8(v, sp);
    }
};
// B operand from C-layout tiles held in registers (tchain_x6: k-block kb = registers 8(kb&1).. of tile kb>>1)
template <int NT>
struct TeamRegs {
    const f32x16 (&x)[NT];
    __device__ __forceinline__ void operator()(int kb, uint32_t (&sp)[3][4]) const {
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = x[kb >> 1][8 * (kb & 1) + e];
        split8(v, sp);
    }
};
// threadIdx.x & 63, opaque to the compiler: a body inlined into a loop (k_fwd_fused_team) would
// otherwise have its ≈ 50 per-lane fragment offsets hoisted out of the loop and live across it
__device__ __forceinline__ int opaque_lane() {
    int lane = threadIdx.x & 63;
    asm volatile("" : "+v"(lane));
    return lane;
}
// The node rows of a team node body. Lane j's column of every node tile is node n: in a 32-node
// block launch n = 32·nb + j (lanes past the batch compute on padding rows and store zeros there, as
// the wide kernels do); in a fused wave-tile launch n = n0 + j for j < nn, the other lanes repeat
// row n0 and store nothing (their columns never mix with the valid ones). oN/oE are the chunk-major
// block offsets of n's block; vl is the "lane" the cm helpers take: the lane's half, n's row in its
// block. nc is n clamped into the batch (input arrays of n_nodes rows).
struct TeamRows {
    int n, nc, vl, jl;   // jl: the row within the wave-tile (tile mode) / the block (block mode)
    bool valid, zero_pad;
    int64_t oN, oE;
    __device__ __forceinline__ static TeamRows block(int nb, int n_nodes, int lane) {
        TeamRows R;
        R.n = nb * 32 + (lane & 31);
        R.valid = R.n < n_nodes;
        R.nc = R.valid ? R.n : n_nodes - 1;
        R.zero_pad = true;
        R.jl = lane & 31;
        R.oN = (int64_t)nb * kCmBlkN;
        R.oE = (int64_t)nb * kCmBlk;
        R.vl = lane;
        return R;
    }
    __device__ __forceinline__ static TeamRows tile(int n0, int nn, int lane) {
        TeamRows R;
        const int j = lane & 31;
        R.valid = j < nn;
        R.n = R.nc = n0 + (R.valid ? j : 0);
        R.jl = R.valid ? j : 0;
        R.zero_pad = false;
        R.oN = (int64_t)(R.n >> 5) * kCmBlkN;
        R.oE = (int64_t)(R.n >> 5) * kCmBlk;
        R.vl = (lane & 32) | (R.n & 31);
        return R;
    }
    // the same rows, opaque to the compiler (see opaque_lane): taken once per step of a fused loop
    __device__ __forceinline__ TeamRows opaque() const {
        TeamRows R = *this;
        asm volatile("" : "+v"(R.n), "+v"(R.nc), "+v"(R.vl), "+v"(R.jl), "+v"(R.oN), "+v"(R.oE));
        return R;
    }
    // a node tile's store: valid lanes their row; padding lanes of a block launch zeros
    template <int KH>
    __device__ __forceinline__ void store(float* __restrict__ base, const f32x16& x, int t) const {
        const int64_t o = KH == kKhE ? oE : oN;
        if (valid) store_cm_tile<KH>(base + o, x, t, vl);
        else if (zero_pad) store_cm_tile<KH>(base + o, zero16(), t, vl);
    }
    // a store the block kernels make for every lane (padding rows get the padding lanes' values)
    template <int KH>
    __device__ __forceinline__ void store_all(float* __restrict__ base, const f32x16& x, int t) const {
        if (valid || zero_pad) store_cm_tile<KH>(base + (KH == kKhE ? oE : oN), x, t, vl);
    }
    template <int KH>
    __device__ __forceinline__ f32x16 load(const float* __restrict__ base, int t) const {
        return load_cm_tile<KH>(base + (KH == kKhE ? oE : oN), t, vl);
    }
    template <int KH>
    __device__ __forceinline__ void half(TeamHalf<KH>& hr, const float* __restrict__ base) const {
        hr.load(base + (KH == kKhE ? oE : oN), vl);
    }
};
template <int KH>
__device__ __forceinline__ void store_cm_tile_b16(uint16_t* __restrict__ blk, const f32x16& x, int t, int lane) {
    const int j = lane & 31, h = lane >> 5;
#pragma unroll
    for (int q = 0; q < 4; ++q)
        if (32 * t + 8 * q + 4 < 2 * KH)
            *reinterpret_cast<uint2*>(blk + cm_offk<KH>(j, 32 * t + 8 * q + 4 * h)) =
                pack4_bf16(make_float4(x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]));
}
// bits 16t .. 16t+15 of the lane's words (store_pos_bits of NT tiles): the tile's half of word t>>1;
// the last tile of an odd NT owns its whole word (upper half zero, as store_pos_bits leaves it)
template <int NT>
__device__ __forceinline__ void store_pos_bits_tile(uint32_t* __restrict__ words, const f32x16& x, int t, int lane) {
    uint32_t w = 0u;
#pragma unroll
    for (int r = 15; r >= 0; --r) w = __builtin_amdgcn_alignbit(w, __float_as_uint(x[r]) + 0x7fffffffu, 31);
    uint32_t* p = words + 64 * (t >> 1) + lane;
    if ((NT & 1) && t == NT - 1) *p = w;
    else reinterpret_cast<uint16_t*>(p)[t & 1] = (uint16_t)w;
}
__device__ __forceinline__ void apply_pos_bits_tile(const uint32_t* __restrict__ words, f32x16& x, int t, int lane, float scale) {
    const uint32_t w = words[64 * (t >> 1) + lane] >> (16 * (t & 1));
#pragma unroll
    for (int r = 0; r < 16; ++r) x[r] = mask_bit(x[r] * scale, w, r);
}
// a tile's bias values (padded vector, feature rho(r, h) + 32t), loaded ahead of the product
__device__ __forceinline__ void bias_tile(float (&bv)[16], const float* __restrict__ b, int t, int h) {
#pragma unroll
    for (int r = 0; r < 16; ++r) bv[r] = b[rho(r, 0) + 4 * h + 32 * t];
}
template <bool RELU>
__device__ __forceinline__ void bias_act_tile(f32x16& x, const float (&bv)[16]) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const float v = x[r] + bv[r];
        x[r] = RELU ? relu(v) : v;
    }
}

// ------------------------------------------------------------------------------------------------
// rm encoder (k_enc_edge_x6's chain, Networks.py:75,77): d → relu(rm.0) → 3 × (150×150 + relu) →
// dropout = c_r → A = c_r·W1a + b1, one 32-edge block per 5-wave workgroup.
template <bool TRAIN, int NP, bool B16>
__device__ __forceinline__ void enc_edge_team_body(const EncEdgeArgs& a, int blk, uint4* act_s) {
    const TeamAct<kTeamEdge, NP> act{act_s};
    const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
    const int T = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int64_t e = (int64_t)blk * 32 + j;
    TEAM_STAMP(0);
    TeamFrags<10, NP> F;
    F.load(a.x_rm1, 5, T, lane);   // layer 1's fragments stream in during layer 0
    const int src = a.esrc[e], dst = a.edst[e];
    float dx = 0.f, dy = 0.f;
    if (src >= 0) {
        const float4 ps = reinterpret_cast<const float4*>(a.pos)[src];
        const float4 pd = reinterpret_cast<const float4*>(a.pos)[dst];
        dx = pd.x - ps.x;  // Networks.py:58-62 (receiver − sender), (x, y)
        dy = pd.y - ps.y;
    }
    if (TRAIN && a.ed && T == 0 && h == 0) a.ed[e] = make_float2(dx, dy);
    const bool drop = a.dropout_on && src >= 0;   // the dropout key's node fields, loaded early
    const uint32_t d_tw = drop ? (uint32_t)a.node_tower[src] : 0u, d_ls = drop ? (uint32_t)a.node_local[src] : 0u,
                   d_ld = drop ? (uint32_t)a.node_local[dst] : 0u;
    f32x16 x;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int f = rho(r, 0) + 4 * h + 32 * T;
        x[r] = relu(dense2(dx, dy, a.w_rm0[f], a.w_rm0[160 + f], a.b_rm0[f]));
    }
    const int64_t cmo = (int64_t)blk * kCmBlk;
    uint32_t* const mb = TRAIN ? a.zmask + (int64_t)blk * 4 * 3 * 64 : nullptr;
    auto save = [&](float* base, int layer, const f32x16& z, bool b16) {
        if (base) {
            if (B16 && b16) store_cm_tile_b16<kKhE>(reinterpret_cast<uint16_t*>(base) + cmo, z, T, lane);
            else store_cm_tile<kKhE>(base + cmo, z, T, lane);
        }
        if (layer >= 0) store_pos_bits_tile<5>(mb + layer * 3 * 64, z, T, lane);
    };
    TEAM_STAMP(1);
    if (TRAIN) save(a.z1, 0, x, false);
    act.put(0, T, x, lane);
    team_sync();
    TEAM_STAMP(2);
    const uint4* const next_img[4] = {a.x_rm2, a.x_rm3, a.x_w1a, nullptr};
    const float* const bias[4] = {a.b_rm1, a.b_rm2, a.b_rm3, a.b_w1a};
#pragma unroll
    for (int l = 0; l < 4; ++l) {
        float bv[16];
        bias_tile(bv, bias[l], T, h);
        x = team_gemm(
            F, [&](int kb, uint32_t (&sp)[3][4]) { act.get(l & 1, kb, sp, lane); },
            [&](int kb) {
                if (l < 3) F.load_kb(next_img[l], 5, T, lane, kb);
            });
        TEAM_STAMP(3 + 2 * l);
        if (l < 3) {
            bias_act_tile<true>(x, bv);   // rm's last Dense is linear; relu from Networks.py:75
        } else {
            bias_act_tile<false>(x, bv);
        }
        if (l == 2 && drop) {   // Networks.py:77
            const uint32_t key = drop_row_key(run_seed(a), 1u, d_tw, d_ls, d_ld);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = rho(r, 0) + 4 * h + 32 * T;
                x[r] = drop_keep(key, (uint32_t)f, a.thresh) ? x[r] * a.scale : 0.f;
            }
        }
        if (l == 3) {
            if constexpr (TRAIN && NP == 1 && !B16) {   // bf16 math, fp32 storage (tiles of 17–32 nodes):
#pragma unroll                                           // A rounded as the bf16-stored copy is (§6b)
                for (int r = 0; r < 16; ++r) x[r] = bf16_round(x[r]);
            }
            save(a.A, -1, x, true);   // chunk-major; k_edge_fwd masks padding edges (B16: bf16, §3g)
        } else {
            if (TRAIN) save(l == 0 ? a.z2 : l == 1 ? a.z3 : a.cr, l + 1, x, true);
            act.put((l + 1) & 1, T, x, lane);
            team_sync();
            TEAM_STAMP(4 + 2 * l);
        }
    }
    TEAM_STAMP(10);
}
template <bool TRAIN, int NP, bool B16>
__global__ __launch_bounds__(64 * kTeamEdge) void k_enc_edge_team(EncEdgeArgs a) {
    __shared__ uint4 act_s[2 * kTeamEdge * 2 * NP * 64];   // ≤ 60 KiB
    enc_edge_team_body<TRAIN, NP, B16>(a, blockIdx.x, act_s);
}

// ------------------------------------------------------------------------------------------------
// rm encoder backward (k_enc_edge_bwd_x6's chain): dc_r = dA·W1aᵀ (B from the dA half rows, read by
// every wave), then dz4 .. dz1 through the rm layers' transposed images.
template <int NP, bool B16>
__device__ __forceinline__ void enc_edge_bwd_team_body(const EncEdgeBwdArgs& a, int blk, uint4* act_s) {
    const TeamAct<kTeamEdge, NP> act{act_s};
    const int lane = opaque_lane(), h = lane >> 5, j = lane & 31;
    const int T = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int64_t e = (int64_t)blk * 32 + j;
    TeamFrags<10, NP> F;
    F.load(a.x_w1at, 5, T, lane);
    float4 raw[kKhE / 4];
    if constexpr (B16) {
        const uint2* row = reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(a.dA) + e * kLdE + kKhE * h);
#pragma unroll
        for (int q = 0; q < kKhE / 4; ++q) raw[q] = unpack4_bf16(row[q]);
    } else {
        const float4* row = reinterpret_cast<const float4*>(a.dA + e * kLdE + kKhE * h);
#pragma unroll
        for (int q = 0; q < kKhE / 4; ++q) raw[q] = row[q];
    }
    const int64_t cmo = (int64_t)blk * kCmBlk;
    const uint32_t* const mb = a.zmask + (int64_t)blk * 4 * 3 * 64;
    const uint4* const next_img[4] = {a.x_rm3t, a.x_rm2t, a.x_rm1t, nullptr};
    float* const out[4] = {a.dz4, a.dz3, a.dz2, a.dz1};
    f32x16 x = team_gemm(
        F,
        [&](int kb, uint32_t (&sp)[3][4]) {
            const float4 p = raw[2 * kb];
            const float4 q = 2 * kb + 1 < kKhE / 4 ? raw[2 * kb + 1] : make_float4(0.f, 0.f, 0.f, 0.f);
            const float v[8] = {p.x, p.y, p.z, p.w, q.x, q.y, q.z, q.w};
            split8(v, sp);
        },
        [&](int kb) { F.load_kb(next_img[0], 5, T, lane, kb); });   // dc_r = dA·W1aᵀ
#pragma unroll
    for (int l = 0; l < 4; ++l) {
        apply_pos_bits_tile(mb + (3 - l) * 3 * 64, x, T, lane, l == 0 ? a.scale : 1.f);   // relu (+ dropout) of layer 3 − l
        if constexpr (B16) store_cm_tile_b16<kKhE>(reinterpret_cast<uint16_t*>(out[l]) + cmo, x, T, lane);
        else store_cm_tile<kKhE>(out[l] + cmo, x, T, lane);
        if (l == 3) break;
        act.put(l & 1, T, x, lane);
        team_sync();
        x = team_gemm(
            F, [&](int kb, uint32_t (&sp)[3][4]) { act.get(l & 1, kb, sp, lane); },
            [&](int kb) {
                if (l < 2) F.load_kb(next_img[l + 1], 5, T, lane, kb);
            });
    }
}
template <int NP, bool B16>
__global__ __launch_bounds__(64 * kTeamEdge) void k_enc_edge_bwd_team(EncEdgeBwdArgs a) {
    __shared__ uint4 act_s[2 * kTeamEdge * 2 * NP * 64];
    enc_edge_bwd_team_body<NP, B16>(a, blockIdx.x, act_s);
}

// ------------------------------------------------------------------------------------------------
// om encoder (k_enc_node_x6's chain, Networks.py:76,78): every wave rebuilds the four tiles of
// z1 = relu(om.0(y, w)) and of P0 (the 'propagation' input) in registers — cheap VALU and loads — so
// no layer output crosses waves: wave T < 4 owns tile T of c_o, waves 0..4 tile T of U0 and V0.
template <int NP>
__device__ __forceinline__ void enc_node_team_body(const EncNodeArgs& a, const TeamRows& R) {
    const int lane = threadIdx.x & 63, h = lane >> 5;
    const int T = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int n = R.n, nc = R.nc;
    const bool valid = R.valid;
    TeamFrags<7, NP> F;
    if (T < 4) F.load(a.x_om1, 4, T, lane);
    else F.load(a.x_w1b, 5, T, lane);
    if (T < 4) {
        const float4 p = reinterpret_cast<const float4*>(a.pos)[nc];
        f32x16 Z[4];
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = rho(r, 0) + 4 * h + 32 * t;
                Z[t][r] = relu(dense2(p.y, p.z, a.w_om0[f], a.w_om0[128 + f], a.b_om0[f]));   // Networks.py:65-71: (y, width)
            }
        if (a.zo1) {
            f32x16 zt = Z[0];   // tile T (selected: a runtime index would put the array in scratch)
#pragma unroll
            for (int t = 1; t < 4; ++t)
                if (T == t) zt = Z[t];
            R.store<kKhN>(a.zo1, zt, T);
        }
        float bv[16];
        bias_tile(bv, a.b_om1, T, h);
        const uint32_t key = a.dropout_on ? drop_row_key(run_seed(a), 2u, (uint32_t)a.node_tower[nc], (uint32_t)a.node_local[nc], 0xffffu) : 0u;
        f32x16 C = team_gemm(F, TeamRegs<4>{Z}, [&](int kb) { F.load_kb(a.x_w1b, 5, T, lane, kb); });
        bias_act_tile<true>(C, bv);   // relu(om(.)) — Networks.py:76
        if (a.dropout_on) {           // Networks.py:78
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int f = rho(r, 0) + 4 * h + 32 * T;
                C[r] = drop_keep(key, (uint32_t)f, a.thresh) ? C[r] * a.scale : 0.f;
            }
        }
        R.store<kKhN>(a.co, C, T);
    }
    // P0: the 'propagation' input (Networks.py:29,79), ld 100 → workspace ld 128
    f32x16 P[4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int f0 = 32 * t + 8 * q + 4 * h;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (a.prop && f0 < kFN && valid) v = *reinterpret_cast<const float4*>(a.prop + (int64_t)n * kFN + f0);
            P[t][4 * q] = v.x; P[t][4 * q + 1] = v.y; P[t][4 * q + 2] = v.z; P[t][4 * q + 3] = v.w;
        }
    if (T < 4) {
        f32x16 pt = P[0];
#pragma unroll
        for (int t = 1; t < 4; ++t)
            if (T == t) pt = P[t];
        R.store<kKhN>(a.P0, pt, T);
    }
    f32x16 U = team_gemm(F, TeamRegs<4>{P}, [&](int kb) { F.load_kb(a.x_w1c, 5, T, lane, kb); });
    round_uv_tile(U, a.uv16);   // bf16 math (training): rounded as the wide kernels store them (§3ze)
    R.store<kKhE>(a.U0, U, T);
    U = team_gemm(F, TeamRegs<4>{P}, [&](int) {});
    round_uv_tile(U, a.uv16);
    R.store<kKhE>(a.V0, U, T);
}
template <int NP>
__global__ __launch_bounds__(64 * kTeamEdge) void k_enc_node_team(EncNodeArgs a) {
    enc_node_team_body<NP>(a, TeamRows::block(blockIdx.x, a.n_nodes, threadIdx.x & 63));
}
// Both encoders of a small batch in ONE launch (they are independent): workgroups [0, n_eblocks) run
// the relation encoder's blocks, the rest the object encoder's node blocks — one dependent launch and
// one ramp-up fewer in the replayed step of the reference's batch 32 (the object encoder's ≈ 10 µs
// run beside the relation encoder's 16 instead of before it).
template <bool TRAIN, int NP, bool B16>
__global__ __launch_bounds__(64 * kTeamEdge) void k_enc_pair_team(EncEdgeArgs e, EncNodeArgs n) {
    __shared__ uint4 act_s[2 * kTeamEdge * 2 * NP * 64];
    if ((int)blockIdx.x < e.n_eblocks) enc_edge_team_body<TRAIN, NP, B16>(e, blockIdx.x, act_s);
    else enc_node_team_body<NP>(n, TeamRows::block((int)blockIdx.x - e.n_eblocks, n.n_nodes, threadIdx.x & 63));
}

// ------------------------------------------------------------------------------------------------
// node side of one step (k_node_fwd_x6's chain, Networks.py:88-96): waves 0..3 own the four node
// tiles of a, o1, x' and P' (three LDS exchanges), all five waves one tile each of U', V'.
template <int NP>
// h2l (the fused forward): the tile's H2s rows as one chunk-major 32-row block in LDS, rows = R.jl,
// written by the step's edge side — read instead of the global rows (the same values)
__device__ __forceinline__ void node_fwd_team_body(const NodeFwdArgs& a, const TeamRows& R, uint4* act_s,
                                                   const float* h2l = nullptr) {
    const TeamAct<4, NP> act{act_s};
    const int lane = opaque_lane(), h = lane >> 5;
    const int T = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const bool valid = R.valid;
    const bool nw = T < 4;   // node-tile wave
    // one fragment set: W3a's ten k-blocks, refilled k-block by k-block with the 7-k-block layers
    TeamFrags<10, NP> F;
    const uint4* const first7 = a.cw_in ? a.x_wo1a : a.x_wo1c;
    if (nw) F.load(a.x_w3a, 4, T, lane);
    TEAM_STAMP(0);
    f32x16 O;
    if (nw) {
        // a = tanh([H2s | deg]·[W3; b3])   (Networks.py:88, layer 3 after the sum)
        f32x16 E;
        {
            TeamHalf<kKhE> hr;
            if (h2l) hr.load_lds(h2l, (lane & 32) | R.jl);
            else R.half(hr, a.H2s);
            E = team_gemm(F, hr, [&](int kb) {
                if (kb < 7) F.load_kb(first7, 4, T, lane, kb);
            });
        }
        TEAM_STAMP(1);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int f = rho(r, 0) + 4 * h + 32 * T;
            E[r] = f < kFN ? acc_tanh(E[r]) : 0.f;
        }
        if (a.a_out) R.store<kKhN>(a.a_out, E, T);
        act.put(0, T, E, lane);
        // o1 = relu([c_o | a | P]·Wo1 + bo1): c_o·Wo1c (or step 0's stored accumulator) first
        if (a.cw_in) {
            O = R.load<kKhN>(a.cw_in, T);
        } else {
            TeamHalf<kKhN> hr;
            R.half(hr, a.co);
            O = team_gemm<7>(F, hr, [&](int kb) { F.load_kb(a.x_wo1a, 4, T, lane, kb); });
            if (a.cw_out) R.store_all<kKhN>(a.cw_out, O, T);
        }
        TEAM_STAMP(2);
    }
    team_sync();
    TEAM_STAMP(3);
    if (nw) {
        O = team_gemm<7>(F, [&](int kb, uint32_t (&sp)[3][4]) { act.get(0, kb, sp, lane); },
                      [&](int kb) { F.load_kb(a.x_wo1p, 4, T, lane, kb); }, O);
        {
            TeamHalf<kKhN> hr;
            R.half(hr, a.P);
            float bv[16];
            bias_tile(bv, a.bo1, T, h);
            O = team_gemm<7>(F, hr, [&](int kb) { F.load_kb(a.x_wo2, 4, T, lane, kb); }, O);
            bias_act_tile<true>(O, bv);
        }
        if (a.o1_out) R.store<kKhN>(a.o1_out, O, T);
        act.put(1, T, O, lane);
        TEAM_STAMP(4);
    }
    team_sync();
    TEAM_STAMP(5);
    if (nw) {
        // x' = o1·Wo2' + bo2'; P' = tanh(x'[0:100] + P); logit = x'[100]  (Networks.py:91, 94)
        float bv[16];
        bias_tile(bv, a.bo2p, T, h);
        const f32x16 P = R.load<kKhN>(a.P, T);
        f32x16 X = team_gemm<7>(F, [&](int kb, uint32_t (&sp)[3][4]) { act.get(1, kb, sp, lane); },
                             [&](int kb) {
                                 if (a.U) F.load_kb(a.x_w1b, 5, T, lane, kb);
                             });
        bias_act_tile<false>(X, bv);
        if (T == 3 && a.logits && h == 1 && valid) a.logits[R.n] = X[0];   // x' row 100 = rho(0, 1) + 96
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int f = rho(r, 0) + 4 * h + 32 * T;
            X[r] = f < kFN ? acc_tanh(X[r] + P[r]) : 0.f;   // X := P'
        }
        R.store<kKhN>(a.Pn, X, T);
        act.put(0, T, X, lane);
        TEAM_STAMP(6);
    } else if (a.U) {
        F.template load<7>(a.x_w1b, 5, T, lane);
    }
    team_sync();
    TEAM_STAMP(7);
    if (a.U) {   // U' = P'·W1b, V' = P'·W1c for the next step
        f32x16 U = team_gemm<7>(F, [&](int kb, uint32_t (&sp)[3][4]) { act.get(0, kb, sp, lane); },
                             [&](int kb) { F.load_kb(a.x_w1c, 5, T, lane, kb); });
        round_uv_tile(U, a.uv16);   // bf16 math (training): rounded as the wide kernels store them (§3ze)
        R.store<kKhE>(a.U, U, T);
        TEAM_STAMP(8);
        U = team_gemm<7>(F, [&](int kb, uint32_t (&sp)[3][4]) { act.get(0, kb, sp, lane); }, [&](int) {});
        round_uv_tile(U, a.uv16);
        R.store<kKhE>(a.V, U, T);
        TEAM_STAMP(9);
    }
}

template <int NP>
__global__ __launch_bounds__(64 * kTeamEdge) void k_node_fwd_team(NodeFwdArgs a) {
    __shared__ uint4 act_s[2 * 4 * 2 * NP * 64];
    node_fwd_team_body<NP>(a, TeamRows::block(blockIdx.x, a.n_nodes, threadIdx.x & 63), act_s);
}

// ------------------------------------------------------------------------------------------------
// node side of one backward step (k_node_bwd_x6's chain, x6/bf16 math with dco_sum): waves 0..3 own
// the node tiles of dP, dx, do1, dP_out and g (two LDS exchanges), then one tile each of G3 — the
// fifth tile by wave 0 (NW = 4: one wave per SIMD, the block launch) or by wave 4 (NW = 5: the fused
// backward's five-wave workgroup; wave 4 only takes the barriers until then).
template <int NP, int NW>
__device__ __forceinline__ void node_bwd_team_body(const NodeBwdArgs& a, const TeamRows& R, uint4* act_s) {
    const TeamAct<4, NP> act{act_s};
    const int lane = opaque_lane(), h = lane >> 5;
    const int T = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const bool valid = R.valid;
    const bool nw = NW == 4 || T < 4;   // node-tile wave
    // one fragment set: W1bᵀ/W1cᵀ's ten k-blocks, then the 7-k-block layers
    TeamFrags<10, NP> F;
    if (nw && !a.first) F.load(a.x_w1bt, 4, T, lane);
    else if (nw && !a.tail) F.template load<7>(a.x_wo2t, 4, T, lane);
    else if (!nw && !a.tail) F.template load<7>(a.x_w3t, 5, 4, lane);   // wave 4: G3 tile 4
    f32x16 D = zero16();
    if (nw && !a.first) {   // dP = dPin + dU·W1bᵀ + dV·W1cᵀ
        D = R.load<kKhN>(a.dPin, T);
        TeamHalf<kKhE> hr;
        R.half(hr, a.dU);
        D = team_gemm(F, hr, [&](int kb) { F.load_kb(a.x_w1ct, 4, T, lane, kb); }, D);
        R.half(hr, a.dV);
        D = team_gemm(F, hr, [&](int kb) {
            if (!a.tail && kb < 7) F.load_kb(a.x_wo2t, 4, T, lane, kb);
        }, D);
    }
    if (a.tail) {   // dP0 = d/d 'propagation' (ld 100)
        if (nw && valid) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int f0 = 32 * T + 8 * q + 4 * h;
                if (f0 < kFN) *reinterpret_cast<float4*>(a.dprop + (int64_t)R.n * kFN + f0) = make_float4(D[4 * q], D[4 * q + 1], D[4 * q + 2], D[4 * q + 3]);
            }
        }
        return;
    }
    f32x16 dP;
    if (nw) {
        const f32x16 Pn = R.load<kKhN>(a.Pn, T);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int f = rho(r, 0) + 4 * h + 32 * T;
            D[r] = f < kFN ? D[r] * (1.f - Pn[r] * Pn[r]) : 0.f;   // tanh' (Networks.py:91)
        }
        // the residual path: dP_s gets dpre directly (Add()([prop_layer(x), prop]))
        R.store<kKhN>(a.dPout, D, T);
        dP = D;
        if (a.first && T == 3 && h == 1) {   // x' row 100 = logit
            if (a.bce_logits) {   // spwgnn_bce_backward: dL/dz here (spwgnn_bce's bits), also stored
                const float dl = valid ? bce_dlogit(a.bce_logits[R.n], a.bce_targets[R.n], 1.0f / (float)a.bce_n) : 0.f;
                if (valid) a.bce_dlogits[R.n] = dl;
                D[0] = dl;
            } else {
                D[0] = valid ? a.dlogits[R.n] : 0.f;
            }
        }
        R.store<kKhN>(a.dx, D, T);
        act.put(0, T, D, lane);
    }
    team_sync();
    if (nw) {   // do1 = dx'·Wo2'ᵀ ⊙ [o1 > 0]
        const f32x16 O1 = R.load<kKhN>(a.o1, T);
        f32x16 G = team_gemm<7>(F, [&](int kb, uint32_t (&sp)[3][4]) { act.get(0, kb, sp, lane); },
                                [&](int kb) { F.load_kb(a.x_wo1pt, 4, T, lane, kb); });
#pragma unroll
        for (int r = 0; r < 16; ++r) G[r] = O1[r] > 0.f ? G[r] : 0.f;
        R.store<kKhN>(a.do1, G, T);
        act.put(1, T, G, lane);
    }
    team_sync();
    if (nw) {
        // P part of omp's input → dP_s
        D = team_gemm<7>(F, [&](int kb, uint32_t (&sp)[3][4]) { act.get(1, kb, sp, lane); },
                         [&](int kb) { F.load_kb(a.x_wo1at, 4, T, lane, kb); });
#pragma unroll
        for (int r = 0; r < 16; ++r) D[r] += dP[r];
        R.store<kKhN>(a.dPout, D, T);
        // effect part → g = da ⊙ (1 − a²)
        const f32x16 Aa = R.load<kKhN>(a.a, T);
        D = team_gemm<7>(F, [&](int kb, uint32_t (&sp)[3][4]) { act.get(1, kb, sp, lane); },
                         [&](int kb) { F.load_kb(a.x_w3t, 5, T, lane, kb); });
#pragma unroll
        for (int r = 0; r < 16; ++r) D[r] = D[r] * (1.f - Aa[r] * Aa[r]);
        R.store<kKhN>(a.g, D, T);
        act.put(0, T, D, lane);
    }
    team_sync();
    // G3 = g·W3ᵀ (the per-edge dh2 is G3[receiver]): tile T (wave 4: tile 4), and NW = 4's wave 0 tile 4
    f32x16 H = team_gemm<7>(F, [&](int kb, uint32_t (&sp)[3][4]) { act.get(0, kb, sp, lane); }, [&](int kb) {
        if (NW == 4 && T == 0) F.load_kb(a.x_w3t, 5, 4, lane, kb);
    });
    R.store<kKhE>(a.G3, H, T);
    if (NW == 4 && T == 0) {
        H = team_gemm<7>(F, [&](int kb, uint32_t (&sp)[3][4]) { act.get(0, kb, sp, lane); }, [&](int) {});
        R.store<kKhE>(a.G3, H, 4);
    }
}
template <int NP>
__global__ __launch_bounds__(256, 1) void k_node_bwd_team(NodeBwdArgs a) {
    __shared__ uint4 act_s[2 * 4 * 2 * NP * 64];
    node_bwd_team_body<NP, 4>(a, TeamRows::block(blockIdx.x, a.n_nodes, threadIdx.x & 63), act_s);
}

// ---- shared A operands of the team edge kernels: wave T builds k-blocks 2T, 2T+1 (chunks 4T .. 4T+3)
// of the block's 32 × 152 operand, splits them and puts the parts in LDS ([kb][part][lane] uint4);
// after a barrier every wave runs its output tile's ten k-blocks on it (team_lds_gemm). One memory
// latency per block instead of one per k-block, and each operand element loaded once, not 5×.
// dh2pre = G3[receiver] ⊙ [h2 > 0] (the edge backward and the dA rebuild), as k_edge_bwd_x6 builds it.
template <int NP>
__device__ __forceinline__ void team_dh2_kblocks(const float* __restrict__ G3, const uint32_t* __restrict__ m2row,
                                                 int d, int n0, int T, int lane, uint4* buf) {
    const int h = lane >> 5, i = lane & 31;
    const bool valid = d >= 0;
    uint32_t w[5];
    load_m2(m2row, i, w);
#pragma unroll
    for (int t = 0; t < 5; ++t) w[t] = valid ? w[t] : 0u;
    // this lane's 76 feature bits (features 76h + 0..75): a 64-bit low part and a 12-bit tail
    const uint64_t mlo = h == 0 ? ((uint64_t)w[1] << 32 | w[0])
                                : ((uint64_t)w[4] << 52 | (uint64_t)w[3] << 20 | (w[2] >> 12));
    const uint32_t mhi = h == 0 ? (w[2] & 0xfffu) : (w[4] >> 12);
    const float4* G4 = reinterpret_cast<const float4*>(G3 + cm_index<kKhE>(valid ? d : n0, 0) + h * 128);
    float4 g[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) g[c] = G4[64 * min(4 * T + c, kKhE / 4 - 1)];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int kb = 2 * T + k;
        float xv[8];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int q = 2 * kb + c;
            const uint32_t bits = q < 16 ? (uint32_t)(mlo >> (4 * q)) : (q < 19 ? mhi >> (4 * q - 64) : 0u);
            const float4 gv = g[2 * k + c];
            xv[4 * c + 0] = mask_bit(gv.x, bits, 0);
            xv[4 * c + 1] = mask_bit(gv.y, bits, 1);
            xv[4 * c + 2] = mask_bit(gv.z, bits, 2);
            xv[4 * c + 3] = mask_bit(gv.w, bits, 3);
        }
        uint32_t sp[3][4];
#pragma unroll
        for (int m = 0; m < 4; ++m) split2(xv[2 * m], xv[2 * m + 1], sp[0][m], sp[1][m], sp[2][m]);
#pragma unroll
        for (int p = 0; p < NP; ++p) buf[(kb * 3 + p) * 64 + lane] = make_uint4(sp[p][0], sp[p][1], sp[p][2], sp[p][3]);
    }
}
// acc = Σ_kb A(kb) · W(kb, T) over the ten k-blocks in LDS, in mfma32_x6's product order
template <int NP>
__device__ __forceinline__ f32x16 team_lds_gemm(const uint4* buf, const uint4 (&wf)[10][NP], int lane) {
    f32x16 acc = zero16();
    uint4 cur[3], nxt[3];
#pragma unroll
    for (int p = 0; p < NP; ++p) cur[p] = buf[p * 64 + lane];
#pragma unroll
    for (int kb = 0; kb < 10; ++kb) {
        if (kb + 1 < 10) {
#pragma unroll
            for (int p = 0; p < NP; ++p) nxt[p] = buf[((kb + 1) * 3 + p) * 64 + lane];
        }
        bf16x8 ap[3], bp[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            ap[p] = as_bf16x8(p < NP ? cur[p] : make_uint4(0u, 0u, 0u, 0u));
            bp[p] = as_bf16x8(p < NP ? wf[kb][p] : make_uint4(0u, 0u, 0u, 0u));
        }
        __builtin_amdgcn_sched_barrier(0);
        acc = mfma32_x6<NP>(ap, bp, acc);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int p = 0; p < NP; ++p) cur[p] = nxt[p];
    }
    return acc;
}

// ---- edge side of one propagation step (k_edge_fwd_x6 for ≤ 16-node wave-tiles), team form ----
// A workgroup of five waves takes one wave-tile; wave T owns output feature tile T of h2 (and its
// receiver sums). Per 32-edge block, wave T builds k-blocks 2T and 2T+1 of h1 = relu(A + U[s] + V[r])
// (its loads all issued at once: one memory latency per block, not ten — the small-batch step is
// latency-bound), splits them and puts the three bf16 parts in LDS (and their h1 > 0 words); after one
// barrier every wave runs its tile's ten k-blocks on the shared operand with W2 fragments read straight
// from the x6 image (L2; no 150 KB LDS fill). Products, their per-accumulator order, the epilogue and
// the one-hot receiver sum of tile T are k_edge_fwd_x6's (mfma32_x6 / NodeSum16X6), so H2s and both
// masks are bit-identical. Wave T writes the h2 > 0 word of tile T (wave 0 also the padding words).
// hs: two buffers of 10 k-blocks × 3 parts × 64 lanes (uint4), 60 KiB, blocks alternate.
template <int NP, bool AB16>
__device__ __forceinline__ void edge_fwd_team_body(const EdgeFwdArgs& a, int wt, uint4* hs, float* h2l = nullptr) {
    const int lane = opaque_lane(), h = lane >> 5, i = lane & 31;
    const int T = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int4 info = reinterpret_cast<const int4*>(a.wtile)[wt];
    const int fb = info.x, nb = info.y, n0 = info.z, nn = info.w;
    TEAM_STAMP(16);
    uint4 wf[10][NP];   // tile T's W2 fragments, all ten k-blocks
#pragma unroll
    for (int kb = 0; kb < 10; ++kb)
#pragma unroll
        for (int p = 0; p < NP; ++p) wf[kb][p] = a.x_w2[((kb * 5 + T) * 3 + p) * 64 + lane];
    const float b2 = a.b2[32 * T + i];
    f32x4 nacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};   // NodeSum16X6 sub-tiles 2T, 2T+1
    const int key = n0 + (lane & 15);
    const int m1off = lane < 4 ? lane : kKhE + lane - 4;
    for (int bb = 0; bb < nb; ++bb) {
        const int blk = fb + bb;
        uint4* const buf = hs + (bb & 1) * (10 * 3 * 64);
        const int s = a.esrc[(int64_t)blk * 32 + i], d = a.edst[(int64_t)blk * 32 + i];
        const bool valid = s >= 0;
        const uint64_t vmask = __ballot(valid);
        TEAM_STAMP(22);
        const float vcap = valid ? __builtin_huge_valf() : 0.f;   // relu_valid: 0 on padding edges
        {   // k-blocks 2T, 2T+1: chunks q = 4T .. 4T+3 (q < 19)
            const int sc = valid ? s : n0, dc = valid ? d : n0;
            const int64_t ai = (int64_t)blk * kCmBlk + h * 128 + i * 4;
            const float4* U4 = reinterpret_cast<const float4*>(a.U + cm_index<kKhE>(sc, 0) + h * 128);
            const float4* V4 = reinterpret_cast<const float4*>(a.V + cm_index<kKhE>(dc, 0) + h * 128);
            float4 ra[4], ru[4], rv[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int q = min(4 * T + c, kKhE / 4 - 1);
                if constexpr (AB16)
                    ra[c] = unpack4_bf16(*reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(a.A) + ai + 256 * q));
                else
                    ra[c] = *reinterpret_cast<const float4*>(a.A + ai + 256 * q);
                ru[c] = U4[64 * q];
                rv[c] = V4[64 * q];
            }
            uint32_t* mrow = a.mask1 ? a.mask1 + (int64_t)blk * kLdE : nullptr;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int kb = 2 * T + k;
                float xv[8];
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const float4 av = ra[2 * k + c], uv = ru[2 * k + c], vv = rv[2 * k + c];
                    xv[4 * c + 0] = relu_valid(av.x + uv.x + vv.x, vcap);
                    xv[4 * c + 1] = relu_valid(av.y + uv.y + vv.y, vcap);
                    xv[4 * c + 2] = relu_valid(av.z + uv.z + vv.z, vcap);
                    xv[4 * c + 3] = relu_valid(av.w + uv.w + vv.w, vcap);
                }
                if (k == 0) TEAM_STAMP(23);
                uint32_t sp[3][4];
#pragma unroll
                for (int m = 0; m < 4; ++m) split2(xv[2 * m], xv[2 * m + 1], sp[0][m], sp[1][m], sp[2][m]);
#pragma unroll
                for (int p = 0; p < NP; ++p) buf[(kb * 3 + p) * 64 + lane] = make_uint4(sp[p][0], sp[p][1], sp[p][2], sp[p][3]);
                if (k == 0) TEAM_STAMP(24);
                if (mrow) {   // h1 > 0 bits of the block's real chunks (as k_edge_fwd_x6)
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
            }
            if (mrow && T == 0 && lane < 8) mrow[2 * kKhE + lane] = 0u;   // features 152..159 (padding)
        }
        TEAM_STAMP(17);
        team_sync();   // the block's split h1 (the other buffer is free: every wave passed this barrier)
        TEAM_STAMP(18);
        f32x16 acc = team_lds_gemm<NP>(buf, wf, lane);
        TEAM_STAMP(19);
        const uint32_t vh = (uint32_t)vmask >> (4 * h);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            float v = relu(acc[r] + b2);
            if (T == 4 && i == kDegCol - 128) v = 1.f;   // degree column (multiplies b3)
            acc[r] = mask_bit(v, vh, rho(r, 0));
        }
        if (a.mask2) {   // h2 > 0 bits of tile T: word m2_pos(edge, T) = 8·edge + T, in register edge >> 3
            uint32_t mw2[4] = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int r0 = 0; r0 < 16; r0 += 8) {
                uint64_t bal[8];
#pragma unroll
                for (int r = 0; r < 8; ++r) bal[r] = __ballot(acc[r0 + r] > 0.f);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    const int e0 = rho(r0 + r, 0), e1 = rho(r0 + r, 1);
                    mw2[e0 >> 3] = writelane((uint32_t)bal[r], 8 * (e0 & 7) + T, mw2[e0 >> 3]);
                    mw2[e1 >> 3] = writelane((uint32_t)(bal[r] >> 32), 8 * (e1 & 7) + T, mw2[e1 >> 3]);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            uint32_t* m2row = a.mask2 + (int64_t)blk * kM2Blk;
            const int t7 = lane & 7;
            if (t7 == T || (T == 0 && t7 >= 5))
#pragma unroll
                for (int k = 0; k < 4; ++k) m2row[64 * k + lane] = t7 == T ? mw2[k] : 0u;
        }
        TEAM_STAMP(20);
        // receiver sum of tile T (NodeSum16X6::add for t = T)
        {
            const int g = lane >> 4;
#if SPWGNN_ONEHOT_BPERM
            const int ld = d - n0, gb = 16 * (g & 1) + 4 * (g >> 1);   // (as NodeSum16X6::add)
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
            uint32_t P[2][3][4];
#pragma unroll
            for (int sh = 0; sh < 2; ++sh)
#pragma unroll
                for (int m = 0; m < 4; ++m)
                    split2(acc[8 * sh + 2 * m], acc[8 * sh + 2 * m + 1], P[sh][0][m], P[sh][1][m], P[sh][2][m]);
#pragma unroll
            for (int p = 0; p < 3; ++p)
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const auto r = __builtin_amdgcn_permlane16_swap(P[0][p][m], P[1][p][m], false, false);
                    P[0][p][m] = r[0];
                    P[1][p][m] = r[1];
                }
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int p = NP - 1; p >= 0; --p)
                    nacc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                        ao, as_bf16x8(make_uint4(P[u][p][0], P[u][p][1], P[u][p][2], P[u][p][3])), nacc[u], 0, 0, 0);
        }
    }
    TEAM_STAMP(21);
    // H2s rows of tile T (NodeSum16X6::store for sub-tiles 2T, 2T+1)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int node = 4 * (lane >> 4) + r;
        if (node < nn) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int f = 32 * T + 16 * u + (lane & 15);
                if (f < 2 * kKhE) {
                    a.H2s[cm_index<kKhE>(n0 + node, f)] = nacc[u][r];
                    if (h2l) h2l[cm_offk<kKhE>(node, f)] = nacc[u][r];
                }
            }
        }
    }
}

constexpr int kTeamHsU4 = 2 * 10 * 3 * 64;   // edge bodies' split-operand buffers (uint4), 60 KiB
// LDS of a launch that runs edge bodies and five-tile exchanges (TeamAct<5>) one after the other
template <int NP>
constexpr int kTeamLdsU4 = kTeamHsU4 > 2 * kTeamEdge * 2 * NP * 64 ? kTeamHsU4 : 2 * kTeamEdge * 2 * NP * 64;
template <int NP, bool AB16>
__global__ __launch_bounds__(64 * kTeamEdge) void k_edge_fwd_team(EdgeFwdArgs a) {
    __shared__ uint4 hs[kTeamHsU4];
    if ((int)blockIdx.x < a.n_wtiles) edge_fwd_team_body<NP, AB16>(a, blockIdx.x, hs);
}

// ---- a small batch's forward step loop in one launch (FwdFusedArgs, kernels.h) ----
// One workgroup of five waves per wave-tile: per step the edge side (H2s of the tile's nodes, also
// handed to the node side in LDS) and the node side (P', U', V' of the same rows); with `encoders`
// (diagnosis builds) the relation encoder on the tile's blocks and the object encoder on its rows
// first. The phases are the team kernels' bodies unchanged —
// same products in the same order, so every output is bit-identical to the launch-per-phase chain
// (tests/test_gpu_team.py) — and are separated by workgroup barriers instead of kernel boundaries:
// a wave-tile holds whole towers, so every row a phase reads was written by this workgroup.
// a pointer the compiler must treat as new in every step: keeps the bodies' per-lane fragment
// addresses from being hoisted out of the step loop (they would stay live across it and spill)
// (laundered as a global-address-space pointer: a generic one would turn every access through it
// into flat memory instructions, which also count against the LDS wait counter)
template <class T>
__device__ __forceinline__ void opaque(T*& p) {
    __attribute__((address_space(1))) T* g = (__attribute__((address_space(1))) T*)p;
    asm volatile("" : "+s"(g));
    p = (T*)g;
}
template <bool TRAIN, int NP, bool AB16>
__global__ __launch_bounds__(64 * kTeamEdge) void k_fwd_fused_team(FwdFusedArgs a) {
    __shared__ uint4 act_s[kTeamLdsU4<NP>];
    __shared__ float h2l[kCmBlk];   // the step's H2s rows of the tile (≤ 16 nodes), edge side → node side
    const int wt = blockIdx.x;
    const int4 info = reinterpret_cast<const int4*>(a.ef.wtile)[wt];
    const TeamRows R = TeamRows::tile(info.z, info.w, threadIdx.x & 63);
    TEAM_STAMP(10);
    if (a.encoders) {   // else both encoders ran before, side by side (k_enc_pair_team)
        for (int b = 0; b < info.y; ++b) enc_edge_team_body<TRAIN, NP, AB16>(a.ee, info.x + b, act_s);
        enc_node_team_body<NP>(a.en, R);
        __syncthreads();   // A, U0, V0 of the tile
    }
    for (int s = 0; s < a.S; ++s) {
        const int64_t sE = (int64_t)(a.training ? s : 0) * a.rowsE;   // Ws::U_at / V_at / H2s_at
        EdgeFwdArgs ef = a.ef;
        opaque(ef.x_w2);
        opaque(ef.b2);
        opaque(ef.A);
        ef.U += sE;
        ef.V += sE;
        ef.H2s += sE;
        if (ef.mask1) ef.mask1 += s * a.m1_step;
        if (ef.mask2) ef.mask2 += s * a.m2_step;
        if (s == 0) TEAM_STAMP(11);
        edge_fwd_team_body<NP, AB16>(ef, wt, act_s, h2l);
        if (s == 0) TEAM_STAMP(12);
        __syncthreads();   // H2s of step s
        NodeFwdArgs nf = a.nf;
        opaque(nf.x_w3a);
        opaque(nf.x_wo1c);
        opaque(nf.x_wo1a);
        opaque(nf.x_wo1p);
        opaque(nf.x_wo2);
        opaque(nf.x_w1b);
        opaque(nf.x_w1c);
        opaque(nf.bo1);
        opaque(nf.bo2p);
        opaque(nf.co);
        nf.H2s = ef.H2s;
        nf.P += (int64_t)(a.training ? s : (s & 1)) * a.rowsN;                 // Ws::P_at(s)
        nf.Pn = const_cast<float*>(a.nf.P) + (int64_t)(a.training ? s + 1 : ((s + 1) & 1)) * a.rowsN;
        if (nf.a_out) nf.a_out += (int64_t)s * a.rowsN;
        if (nf.o1_out) nf.o1_out += (int64_t)s * a.rowsN;
        nf.cw_out = s == 0 ? a.nf.cw_out : nullptr;
        nf.cw_in = s > 0 ? a.nf.cw_out : nullptr;
        nf.logits = s == a.S - 1 ? a.logits : nullptr;
        const int64_t sE1 = (int64_t)(a.training ? s + 1 : 0) * a.rowsE;
        nf.U = s + 1 < a.S ? const_cast<float*>(a.ef.U) + sE1 : nullptr;   // the same workspace arrays
        nf.V = s + 1 < a.S ? const_cast<float*>(a.ef.V) + sE1 : nullptr;
        if (s == 0) TEAM_STAMP(13);
        node_fwd_team_body<NP>(nf, R.opaque(), act_s, h2l);
        if (s == 0) TEAM_STAMP(14);
        __syncthreads();   // P', U', V' of step s + 1
        if (s == 0) TEAM_STAMP(15);
    }
}

// ---- edge side of one backward step (k_edge_bwd_x6 without dA: x6/bf16 rebuild it), team form ----
// Five waves per wave-tile; wave T owns feature tile T of dh1 = dh2pre·W2ᵀ: every wave builds the
// whole dh2pre = G3[receiver] ⊙ [h2 > 0] operand k-block by k-block, multiplies it by its tile's W2ᵀ
// fragments (from the x6 image in L2), masks with [h1 > 0] and runs tile T's one-hot receiver/sender
// sums — k_edge_bwd_x6's products in its per-accumulator order, so dU and dV are bit-identical.
// dacc (fused backward, tiles of ≤ kTeamDaBlocks blocks): dA = Σ_s dh1pre_s accumulated in LDS per
// (block, tile T, register, lane) across the steps, s = S−1 first (dacc_first) — the rebuild's order
// and products, so the same bits as k_dA_team's
constexpr int kTeamDaBlocks = 4;
template <int NP>
__device__ __forceinline__ void edge_bwd_team_body(const EdgeBwdArgs& a, int wt, uint4* hs, float* dacc = nullptr,
                                                   bool dacc_first = false) {
    const int lane = opaque_lane(), h = lane >> 5, i = lane & 31;
    const int T = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int4 info = reinterpret_cast<const int4*>(a.wtile)[wt];
    const int fb = info.x, nb = info.y, n0 = info.z, nn = info.w;
    uint4 wf[10][NP];   // tile T's W2ᵀ fragments
#pragma unroll
    for (int kb = 0; kb < 10; ++kb)
#pragma unroll
        for (int p = 0; p < NP; ++p) wf[kb][p] = a.x_w2t[((kb * 5 + T) * 3 + p) * 64 + lane];
    const int key = i < 16 ? n0 + i : n0 + i - 16;   // one-hot rows: receivers, then senders
    f32x16 nacc = zero16();
    for (int bb = 0; bb < nb; ++bb) {
        const int blk = fb + bb;
        uint4* const buf = hs + (bb & 1) * (10 * 3 * 64);
        const int64_t e = (int64_t)blk * 32 + i;
        const int d = a.edst[e], s_ = a.esrc[e];
        const uint32_t m1w = a.mask1[(int64_t)blk * kLdE + i + 32 * T];
        team_dh2_kblocks<NP>(a.G3, a.mask2 + (int64_t)blk * kM2Blk, d, n0, T, lane, buf);
        team_sync();   // the block's split dh2pre (the other buffer is free)
        f32x16 acc = team_lds_gemm<NP>(buf, wf, lane);
        // dh1pre = dh1 ⊙ [h1 > 0]  (C layout: lane = feature 32T+i, rows = edges rho(r,h))
        const uint32_t mh = m1w >> (4 * h);
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = mask_bit(acc[r], mh, rho(r, 0));
        if (dacc && bb < kTeamDaBlocks) {
            float* q = dacc + (bb * 5 + T) * 16 * 64 + lane;
#pragma unroll
            for (int r = 0; r < 16; ++r) q[r * 64] = (dacc_first ? 0.f : q[r * 64]) + acc[r];
        }
#if SPWGNN_ONEHOT_BPERM
        // packed tile-local ids, one ds_bpermute per element (as k_edge_bwd_x6)
        const uint32_t ld_ = (uint32_t)(d - n0) < 16u ? (uint32_t)(d - n0) : 0xffffu;
        const uint32_t ls_ = (uint32_t)(s_ - n0) < 16u ? (uint32_t)(s_ - n0) : 0xffffu;
        const int pk = (int)(ld_ | (ls_ << 16));
        const int kbits = i < 16 ? 0 : 16;
#endif
#pragma unroll
        for (int sh = 0; sh < 2; ++sh) {
            uint32_t oh[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                uint32_t wv = 0u;
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int ee = 2 * m + q;
#if SPWGNN_ONEHOT_BPERM
                    const uint32_t v = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * rho(8 * sh + ee, h), pk);
                    wv |= (__builtin_amdgcn_ubfe(v, kbits, 16) == (uint32_t)(i & 15) ? 0x3F80u : 0u) << (16 * q);
#else
                    const int d0 = __builtin_amdgcn_readlane(d, rho(8 * sh + ee, 0));
                    const int d1 = __builtin_amdgcn_readlane(d, rho(8 * sh + ee, 1));
                    const int s0 = __builtin_amdgcn_readlane(s_, rho(8 * sh + ee, 0));
                    const int s1 = __builtin_amdgcn_readlane(s_, rho(8 * sh + ee, 1));
                    const int node = i < 16 ? (h ? d1 : d0) : (h ? s1 : s0);
                    wv |= (node == key ? 0x3F80u : 0u) << (16 * q);
#endif
                }
                oh[m] = wv;
            }
            const bf16x8 ao = as_bf16x8(make_uint4(oh[0], oh[1], oh[2], oh[3]));
            uint32_t hw[4], mw[4], lw[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) split2(acc[8 * sh + 2 * m], acc[8 * sh + 2 * m + 1], hw[m], mw[m], lw[m]);
            if constexpr (NP == 3) {
                nacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ao, as_bf16x8(make_uint4(lw[0], lw[1], lw[2], lw[3])), nacc, 0, 0, 0);
                nacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ao, as_bf16x8(make_uint4(mw[0], mw[1], mw[2], mw[3])), nacc, 0, 0, 0);
            }
            nacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ao, as_bf16x8(make_uint4(hw[0], hw[1], hw[2], hw[3])), nacc, 0, 0, 0);
        }
    }
    // nacc reg r = row rho(r,h): rows 0..15 receiver nodes (dV), 16..31 sender nodes (dU)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row = rho(r, h);
        const int node = row & 15;
        if (node < nn && 32 * T + i < 2 * kKhE) {
            float* o = row < 16 ? a.dV : a.dU;
            o[cm_index<kKhE>(n0 + node, 32 * T + i)] = nacc[r];
        }
    }
}
template <int NP>
__global__ __launch_bounds__(64 * kTeamEdge) void k_edge_bwd_team(EdgeBwdArgs a) {
    __shared__ uint4 hs[kTeamHsU4];
    if ((int)blockIdx.x < a.n_wtiles) edge_bwd_team_body<NP>(a, blockIdx.x, hs);
}

// ---- dA = Σ_s dh1pre_s (k_dA_x6), team form: five waves per 32-edge block, wave T owns feature
// tile T; the same products, per-accumulator order and step order (S−1 first) as k_dA_x6.
template <int NP, bool B16>
__device__ __forceinline__ void dA_team_body(const DaArgs& a, int blk, uint4* hs) {
    const int lane = opaque_lane(), h = lane >> 5, i = lane & 31;
    const int T = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    uint4 wf[10][NP];   // tile T's W2ᵀ fragments
#pragma unroll
    for (int kb = 0; kb < 10; ++kb)
#pragma unroll
        for (int p = 0; p < NP; ++p) wf[kb][p] = a.x_w2t[((kb * 5 + T) * 3 + p) * 64 + lane];
    const int d = a.edst[(int64_t)blk * 32 + i];
    f32x16 dacc = zero16();
    for (int s = a.S - 1; s >= 0; --s) {
        uint4* const buf = hs + (s & 1) * (10 * 3 * 64);
        const uint32_t m1w = a.mask1[s * a.m1_step + (int64_t)blk * kLdE + i + 32 * T];
        team_dh2_kblocks<NP>(a.G3 + s * a.g3_step, a.mask2 + s * a.m2_step + (int64_t)blk * kM2Blk, d, 0, T, lane, buf);
        team_sync();   // step s's split dh2pre (the other buffer is free)
        const f32x16 acc = team_lds_gemm<NP>(buf, wf, lane);
        const uint32_t mh = m1w >> (4 * h);
#pragma unroll
        for (int r = 0; r < 16; ++r) dacc[r] += mask_bit(acc[r], mh, rho(r, 0));
    }
    if constexpr (B16) {   // bf16 math: dA feeds MFMA operands only (§3g)
        __bf16* dArow = reinterpret_cast<__bf16*>(a.dA) + (int64_t)blk * 32 * kLdE + i;
#pragma unroll
        for (int r = 0; r < 16; ++r) dArow[rho(r, h) * kLdE + 32 * T] = (__bf16)dacc[r];
    } else {
        float* dArow = a.dA + (int64_t)blk * 32 * kLdE + i;
#pragma unroll
        for (int r = 0; r < 16; ++r) dArow[rho(r, h) * kLdE + 32 * T] = dacc[r];
    }
}
template <int NP, bool B16>
__global__ __launch_bounds__(64 * kTeamEdge) void k_dA_team(DaArgs a) {
    __shared__ uint4 hs[kTeamHsU4];
    if ((int)blockIdx.x < a.n_eblocks) dA_team_body<NP, B16>(a, blockIdx.x, hs);
}

// ---- object-encoder backward (k_enc_node_bwd_x6), team form: four waves per 32-node block, wave T
// owns feature tile T of dc_o = (Σ_s do1_s)·Wo1cᵀ and of the om.1ᵀ product; the layer input is
// exchanged through LDS in its split C layout. Same products and order: bit-identical.
// NW = 5 (the fused backward): wave 4 takes the barrier only
template <int NP, int NW>
__device__ __forceinline__ void enc_node_bwd_team_body(const EncNodeBwdArgs& a, const TeamRows& R, uint4* act_s) {
    const TeamAct<4, NP> act{act_s};
    const int lane = opaque_lane(), h = lane >> 5;
    const int T = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (NW == 5 && T == 4) {
        team_sync();
        return;
    }
    TeamFrags<7, NP> F;
    F.load(a.x_wo1ct, 4, T, lane);
    // Σ_s do1_s in backward step order S-1..0 (the Y of the Wo1c weight gradient), every tile
    f32x16 E[4], Z[4];
    load_cm<4>(a.do1 + (int64_t)(a.S - 1) * a.do1_step + R.oN, E, R.vl);
    for (int s = a.S - 2; s >= 0; --s) {
        load_cm<4>(a.do1 + (int64_t)s * a.do1_step + R.oN, Z, R.vl);
#pragma unroll
        for (int t = 0; t < 4; ++t) E[t] += Z[t];
    }
    {
        f32x16 et = E[0];   // tile T (selected: a runtime index would put the array in scratch)
#pragma unroll
        for (int t = 1; t < 4; ++t)
            if (T == t) et = E[t];
        R.store<kKhN>(a.dco, et, T);
    }
    f32x16 D = team_gemm(F, TeamRegs<4>{E}, [&](int kb) { F.load_kb(a.x_om1t, 4, T, lane, kb); });   // dc_o
    const f32x16 C = R.load<kKhN>(a.co, T);
#pragma unroll
    for (int r = 0; r < 16; ++r) D[r] = C[r] > 0.f ? D[r] * a.scale : 0.f;
    R.store<kKhN>(a.dzo2, D, T);
    act.put(0, T, D, lane);
    team_sync();
    f32x16 G = team_gemm(F, [&](int kb, uint32_t (&sp)[3][4]) { act.get(0, kb, sp, lane); }, [&](int) {});
    f32x16 Zt;
    if (a.zo1) {
        Zt = R.load<kKhN>(a.zo1, T);
    } else {   // the forward's own first-layer arithmetic (k_enc_node_x6), not a stored row
        const float4 p = reinterpret_cast<const float4*>(a.pos)[R.nc];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int f = rho(r, 0) + 4 * h + 32 * T;
            Zt[r] = relu(dense2(p.y, p.z, a.w_om0[f], a.w_om0[128 + f], a.b_om0[f]));
        }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) G[r] = Zt[r] > 0.f ? G[r] : 0.f;
    R.store<kKhN>(a.dzo1, G, T);
}
template <int NP>
__global__ __launch_bounds__(256) void k_enc_node_bwd_team(EncNodeBwdArgs a) {
    __shared__ uint4 act_s[4 * 2 * NP * 64];
    enc_node_bwd_team_body<NP, 4>(a, TeamRows::block(blockIdx.x, a.n_nodes, threadIdx.x & 63), act_s);
}

// ---- a small batch's backward (before the weight gradients) in one launch (BwdFusedArgs) ----
// One five-wave workgroup per wave-tile: per step S−1 .. 0 the node side (dx, do1, g, G3 and dP of
// the tile's rows) and the edge side (dU, dV; dh1pre summed into dA in LDS), then d/d 'propagation'
// and the dA rows (k_bwd_enc_pair_team runs the encoder backwards next; with `encoders`, diagnosis
// builds, they run here). Bodies and products are the team kernels' (bit-identical results); phases
// meet at workgroup barriers.
// The fused backward's static LDS (exchange buffers + the dA sums) needs gfx950's 160 KiB per CU; a
// build for a smaller-LDS target stops here with this message rather than in the linker.
constexpr size_t kLdsBytesGfx950 = 160 * 1024;
static_assert(sizeof(uint4) * kTeamLdsU4<3> + sizeof(float) * kTeamDaBlocks * 5 * 16 * 64 <= kLdsBytesGfx950,
              "k_bwd_fused_team: exchange buffers + dA sums exceed the 160 KiB LDS of gfx950");
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "libspwgnn_hip targets gfx950 (160 KiB LDS per CU): the fused small-batch backward needs it"
#endif
template <int NP, bool B16>
__global__ __launch_bounds__(64 * kTeamEdge) void k_bwd_fused_team(BwdFusedArgs a) {
    __shared__ uint4 act_s[kTeamLdsU4<NP>];
    __shared__ float dacc_s[kTeamDaBlocks * 5 * 16 * 64];   // 80 KiB: dA of ≤ 4 blocks across the steps
    const int wt = blockIdx.x;
    const int4 info = reinterpret_cast<const int4*>(a.eb.wtile)[wt];
    const bool da_loop = a.dA_in_loop && info.y <= kTeamDaBlocks;
    const TeamRows R = TeamRows::tile(info.z, info.w, threadIdx.x & 63);
    const float* const dP0 = a.nb.dPout;   // Ws::dP_at(0); dP_at(k) alternates
    for (int s = a.S - 1; s >= 0; --s) {
        const bool first = s == a.S - 1;
        const int64_t sN = (int64_t)s * a.rowsN, sE = (int64_t)s * a.rowsE;
        NodeBwdArgs nb = a.nb;
        opaque(nb.x_w1bt);
        opaque(nb.x_w1ct);
        opaque(nb.x_wo2t);
        opaque(nb.x_wo1pt);
        opaque(nb.x_wo1at);
        opaque(nb.x_w3t);
        nb.first = first;
        nb.dPin = first ? nullptr : dP0 + ((s + 1) & 1) * a.rowsN;
        nb.dU = first ? nullptr : a.nb.dU + sE;   // the host passes dU_at(1) / dV_at(1)
        nb.dV = first ? nullptr : a.nb.dV + sE;
        nb.Pn += sN;
        nb.o1 += sN;
        nb.a += sN;
        nb.dx += sN;
        nb.do1 += sN;
        nb.g += sN;
        nb.G3 += sE;
        nb.dPout = const_cast<float*>(dP0) + (s & 1) * a.rowsN;
        node_bwd_team_body<NP, 5>(nb, R.opaque(), act_s);
        __syncthreads();   // G3 of step s
        EdgeBwdArgs eb = a.eb;
        opaque(eb.x_w2t);
        eb.mask1 += s * a.m1_step;
        eb.mask2 += s * a.m2_step;
        eb.G3 = nb.G3;
        eb.dU += sE;
        eb.dV += sE;
        edge_bwd_team_body<NP>(eb, wt, act_s, da_loop ? dacc_s : nullptr, first);
        __syncthreads();   // dU, dV of step s
    }
    if (a.has_tail) node_bwd_team_body<NP, 5>(a.tail, R, act_s);   // dP0 (reads only)
    if (da_loop) {   // dA rows of the tile's blocks from the LDS sums (each wave its tile T, as k_dA_team)
        const int lane = threadIdx.x & 63, h = lane >> 5, i = lane & 31;
        const int T = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
        for (int bb = 0; bb < info.y; ++bb) {
            const float* q = dacc_s + (bb * 5 + T) * 16 * 64 + lane;
            const int64_t blk = info.x + bb;
            if constexpr (B16) {
                __bf16* dArow = reinterpret_cast<__bf16*>(a.da.dA) + blk * 32 * kLdE + i;
#pragma unroll
                for (int r = 0; r < 16; ++r) dArow[rho(r, h) * kLdE + 32 * T] = (__bf16)q[r * 64];
            } else {
                float* dArow = a.da.dA + blk * 32 * kLdE + i;
#pragma unroll
                for (int r = 0; r < 16; ++r) dArow[rho(r, h) * kLdE + 32 * T] = q[r * 64];
            }
        }
    } else if (a.dA_in_loop) {   // a tile of more blocks: the rebuild, here
        for (int b = 0; b < info.y; ++b) {
            dA_team_body<NP, B16>(a.da, info.x + b, act_s);
            __syncthreads();   // its last operand buffer may be the next block's first
        }
    }
    if (!a.encoders) return;   // else k_bwd_enc_pair_team runs the rest, edge and node side by side
    if (!a.dA_in_loop) {
        for (int b = 0; b < info.y; ++b) {
            dA_team_body<NP, B16>(a.da, info.x + b, act_s);
            __syncthreads();   // the block's dA rows; its last operand buffer may be the next block's first
        }
    }
    __syncthreads();   // every wave's dA rows of the tile
    for (int b = 0; b < info.y; ++b) {
        enc_edge_bwd_team_body<NP, B16>(a.eeb, info.x + b, act_s);
        __syncthreads();   // its last exchange buffer is the next body's first
    }
    enc_node_bwd_team_body<NP, 5>(a.enb, R, act_s);
}
// After the fused step loop: workgroups [0, n_eblocks) rebuild dA of their block and run the
// relation-encoder backward on it, the others the object-encoder backward of a 32-node block —
// independent, so side by side (as the forward's k_enc_pair_team) instead of one after the other.
template <int NP, bool B16>
__global__ __launch_bounds__(64 * kTeamEdge) void k_bwd_enc_pair_team(DaArgs da, EncEdgeBwdArgs eeb, EncNodeBwdArgs enb,
                                                                    int with_dA) {
    __shared__ uint4 act_s[kTeamLdsU4<NP>];
    const int blk = blockIdx.x;
    if (blk < da.n_eblocks) {
        if (with_dA) {   // else the fused backward left dA in place
            dA_team_body<NP, B16>(da, blk, act_s);
            __syncthreads();   // the block's dA rows, written feature tile by feature tile
        }
        enc_edge_bwd_team_body<NP, B16>(eeb, blk, act_s);
    } else {
        enc_node_bwd_team_body<NP, 5>(enb, TeamRows::block(blk - da.n_eblocks, enb.n_nodes, threadIdx.x & 63), act_s);
    }
}

// The team limit in force (spwgnn_team_max_blocks): the compile-time kTeamMaxBlocks unless a caller
// moved it, e.g. a parity test that puts a small batch on the wide (chain) kernels the large-batch
// bench step runs. Read when a call plans its launches; a captured graph keeps the launches it planned.
static std::atomic<int> g_team_max{kTeamMaxBlocks};
int team_max_blocks(int set) {
    return set >= 0 ? g_team_max.exchange(set) : g_team_max.load(std::memory_order_relaxed);
}

bool team_blocks(int n_blocks) {
#ifdef SPWGNN_DIAG   // A/B: SPWGNN_NO_TEAM=1 keeps the one-wave-per-block kernels at every size
    static const bool off = getenv("SPWGNN_NO_TEAM") && atoi(getenv("SPWGNN_NO_TEAM"));
    if (off) return false;
#endif
    return n_blocks > 0 && n_blocks <= g_team_max.load(std::memory_order_relaxed);
}

hipError_t launch_edge_fwd_team(const EdgeFwdArgs& a, int math, hipStream_t st) {
    if (a.nw_max > 16 || a.uv16 == kUvB16) return hipErrorInvalidValue;   // team kernels: fp32 U, V
    const dim3 g(a.n_wtiles), b(64 * kTeamEdge);
    if (math == MATH_BF16) {
        if (a.a_b16) hipLaunchKernelGGL((k_edge_fwd_team<1, true>), g, b, 0, st, a);
        else hipLaunchKernelGGL((k_edge_fwd_team<1, false>), g, b, 0, st, a);
    } else if (math == MATH_X6 && !a.a_b16) {
        hipLaunchKernelGGL((k_edge_fwd_team<3, false>), g, b, 0, st, a);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
hipError_t launch_edge_bwd_team(const EdgeBwdArgs& a, int math, hipStream_t st) {
    if (a.nw_max > 16 || !a.no_dA) return hipErrorInvalidValue;
    const dim3 g(a.n_wtiles), b(64 * kTeamEdge);
    if (math == MATH_BF16) hipLaunchKernelGGL((k_edge_bwd_team<1>), g, b, 0, st, a);
    else if (math == MATH_X6) hipLaunchKernelGGL((k_edge_bwd_team<3>), g, b, 0, st, a);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}
hipError_t launch_dA_team(const DaArgs& a, int math, hipStream_t st) {
    const dim3 g(a.n_eblocks), b(64 * kTeamEdge);
    if (math == MATH_BF16 && a.b16) hipLaunchKernelGGL((k_dA_team<1, true>), g, b, 0, st, a);
    else if (math == MATH_BF16) hipLaunchKernelGGL((k_dA_team<1, false>), g, b, 0, st, a);
    else if (math == MATH_X6) hipLaunchKernelGGL((k_dA_team<3, false>), g, b, 0, st, a);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}
hipError_t launch_enc_node_bwd_team(const EncNodeBwdArgs& a, int math, hipStream_t st) {
    const dim3 g((a.n_nodes + 31) / 32), b(256);
    if (math == MATH_BF16) hipLaunchKernelGGL((k_enc_node_bwd_team<1>), g, b, 0, st, a);
    else if (math == MATH_X6) hipLaunchKernelGGL((k_enc_node_bwd_team<3>), g, b, 0, st, a);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}
hipError_t launch_enc_edge_team(const EncEdgeArgs& a, int math, bool train, hipStream_t st) {
    const dim3 g(a.n_eblocks), b(64 * kTeamEdge);
    if (math == MATH_BF16) {
        if (train && a.b16) hipLaunchKernelGGL((k_enc_edge_team<true, 1, true>), g, b, 0, st, a);
        else if (train) hipLaunchKernelGGL((k_enc_edge_team<true, 1, false>), g, b, 0, st, a);
        else hipLaunchKernelGGL((k_enc_edge_team<false, 1, false>), g, b, 0, st, a);
    } else if (math == MATH_X6) {
        if (train) hipLaunchKernelGGL((k_enc_edge_team<true, 3, false>), g, b, 0, st, a);
        else hipLaunchKernelGGL((k_enc_edge_team<false, 3, false>), g, b, 0, st, a);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
hipError_t launch_enc_node_team(const EncNodeArgs& a, int math, hipStream_t st) {
    if (a.uv16 == kUvB16) return hipErrorInvalidValue;
    const dim3 g((a.n_nodes + 31) / 32), b(64 * kTeamEdge);
    if (math == MATH_BF16) hipLaunchKernelGGL((k_enc_node_team<1>), g, b, 0, st, a);
    else if (math == MATH_X6) hipLaunchKernelGGL((k_enc_node_team<3>), g, b, 0, st, a);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}
bool enc_pair_team(int n_eblocks, int n_nodes, int math) {
    return (math == MATH_X6 || math == MATH_BF16) && team_blocks(n_eblocks) && team_blocks((n_nodes + 31) / 32);
}
hipError_t launch_enc_pair_team(const EncEdgeArgs& e, const EncNodeArgs& n, int math, bool train, hipStream_t st) {
    if (!enc_pair_team(e.n_eblocks, n.n_nodes, math) || n.uv16 == kUvB16) return hipErrorInvalidValue;
    const dim3 g(e.n_eblocks + (n.n_nodes + 31) / 32), b(64 * kTeamEdge);
    if (math == MATH_BF16) {
        if (train && e.b16) hipLaunchKernelGGL((k_enc_pair_team<true, 1, true>), g, b, 0, st, e, n);
        else if (train) hipLaunchKernelGGL((k_enc_pair_team<true, 1, false>), g, b, 0, st, e, n);
        else hipLaunchKernelGGL((k_enc_pair_team<false, 1, false>), g, b, 0, st, e, n);
    } else if (train) {
        hipLaunchKernelGGL((k_enc_pair_team<true, 3, false>), g, b, 0, st, e, n);
    } else {
        hipLaunchKernelGGL((k_enc_pair_team<false, 3, false>), g, b, 0, st, e, n);
    }
    return hipGetLastError();
}
bool fwd_fused_team(int n_wtiles, int nw_max, int n_eblocks, int n_nodes, int math) {
    return nw_max <= 16 && team_blocks(n_wtiles) && enc_pair_team(n_eblocks, n_nodes, math);
}
hipError_t launch_fwd_fused_team(const FwdFusedArgs& a, int math, bool train, hipStream_t st) {
    if (!fwd_fused_team(a.ef.n_wtiles, a.ef.nw_max, a.ee.n_eblocks, a.en.n_nodes, math) || a.S < 1 || a.ef.n16 ||
        a.nf.n16 || a.ef.recv_blocks || a.ee.b16 != a.ef.a_b16 || !a.nf.cw_out || a.en.uv16 == kUvB16 ||
        a.nf.uv16 == kUvB16 || a.ef.uv16 == kUvB16)
        return hipErrorInvalidValue;
    const dim3 g(a.ef.n_wtiles), b(64 * kTeamEdge);
    if (math == MATH_BF16) {
        if (train && a.ee.b16) hipLaunchKernelGGL((k_fwd_fused_team<true, 1, true>), g, b, 0, st, a);
        else if (train) hipLaunchKernelGGL((k_fwd_fused_team<true, 1, false>), g, b, 0, st, a);
        else if (!a.ee.b16) hipLaunchKernelGGL((k_fwd_fused_team<false, 1, false>), g, b, 0, st, a);
        else return hipErrorInvalidValue;
    } else if (math == MATH_X6 && !a.ee.b16) {
        if (train) hipLaunchKernelGGL((k_fwd_fused_team<true, 3, false>), g, b, 0, st, a);
        else hipLaunchKernelGGL((k_fwd_fused_team<false, 3, false>), g, b, 0, st, a);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
hipError_t launch_bwd_fused_team(const BwdFusedArgs& a, int math, hipStream_t st) {
    if (!fwd_fused_team(a.eb.n_wtiles, a.eb.nw_max, a.da.n_eblocks, a.nb.n_nodes, math) || a.S < 1 || !a.eb.no_dA ||
        !a.nb.dco_sum || a.nb.n16 || a.eb.n16 || a.da.b16 != a.eeb.b16)
        return hipErrorInvalidValue;
    const dim3 g(a.eb.n_wtiles), b(64 * kTeamEdge);
    if (math == MATH_BF16 && a.da.b16) hipLaunchKernelGGL((k_bwd_fused_team<1, true>), g, b, 0, st, a);
    else if (math == MATH_BF16) hipLaunchKernelGGL((k_bwd_fused_team<1, false>), g, b, 0, st, a);
    else if (math == MATH_X6 && !a.da.b16) hipLaunchKernelGGL((k_bwd_fused_team<3, false>), g, b, 0, st, a);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}
hipError_t launch_bwd_enc_pair_team(const DaArgs& da, const EncEdgeBwdArgs& eeb, const EncNodeBwdArgs& enb, int math,
                                    int with_dA, hipStream_t st) {
    if (!team_blocks(da.n_eblocks) || !team_blocks((enb.n_nodes + 31) / 32) || da.b16 != eeb.b16 || !enb.wo1ct)
        return hipErrorInvalidValue;
    const dim3 g(da.n_eblocks + (enb.n_nodes + 31) / 32), b(64 * kTeamEdge);
    if (math == MATH_BF16 && da.b16) hipLaunchKernelGGL((k_bwd_enc_pair_team<1, true>), g, b, 0, st, da, eeb, enb, with_dA);
    else if (math == MATH_BF16) hipLaunchKernelGGL((k_bwd_enc_pair_team<1, false>), g, b, 0, st, da, eeb, enb, with_dA);
    else if (math == MATH_X6 && !da.b16) hipLaunchKernelGGL((k_bwd_enc_pair_team<3, false>), g, b, 0, st, da, eeb, enb, with_dA);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}
hipError_t launch_node_fwd_team(const NodeFwdArgs& a, int math, hipStream_t st) {
    if (a.uv16 == kUvB16) return hipErrorInvalidValue;
    const dim3 g((a.n_nodes + 31) / 32), b(64 * kTeamEdge);
    if (math == MATH_BF16) hipLaunchKernelGGL((k_node_fwd_team<1>), g, b, 0, st, a);
    else if (math == MATH_X6) hipLaunchKernelGGL((k_node_fwd_team<3>), g, b, 0, st, a);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}
hipError_t launch_node_bwd_team(const NodeBwdArgs& a, int math, hipStream_t st) {
    if (!a.dco_sum) return hipErrorInvalidValue;
    const dim3 g((a.n_nodes + 31) / 32), b(64 * kTeamEdge);
    if (math == MATH_BF16) hipLaunchKernelGGL((k_node_bwd_team<1>), g, dim3(256), 0, st, a);
    else if (math == MATH_X6) hipLaunchKernelGGL((k_node_bwd_team<3>), g, dim3(256), 0, st, a);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}
hipError_t launch_enc_edge_bwd_team(const EncEdgeBwdArgs& a, int math, hipStream_t st) {
    const dim3 g(a.n_eblocks), b(64 * kTeamEdge);
    if (math == MATH_BF16) {
        if (a.b16) hipLaunchKernelGGL((k_enc_edge_bwd_team<1, true>), g, b, 0, st, a);
        else hipLaunchKernelGGL((k_enc_edge_bwd_team<1, false>), g, b, 0, st, a);
    } else if (math == MATH_X6) {
        hipLaunchKernelGGL((k_enc_edge_bwd_team<3, false>), g, b, 0, st, a);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace spw

#ifdef SPWGNN_DIAG
extern "C" int32_t spwgnn_diag_team_stamps(unsigned long long* out64) {
    return hipMemcpyFromSymbol(out64, HIP_SYMBOL(spw::g_team_stamps), sizeof(spw::g_team_stamps)) == hipSuccess ? 0 : -1;
}
#endif
