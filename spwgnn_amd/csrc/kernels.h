// Kernel argument structs and declarations (libspwgnn_hip).
#pragma once

// one-hot node operands of the wide edge kernels built with ds_bpermute from packed tile-local ids
// (SPWGNN_ONEHOT_BPERM=0: the readlane form, for A/B)
#ifndef SPWGNN_ONEHOT_BPERM
#define SPWGNN_ONEHOT_BPERM 1
#endif
#include "gemm_blocks.h"

namespace spw {

struct PackDesc {
    int64_t dst_off;   // floats into the pack buffer
    int64_t src_off;   // floats into the flat params
    int32_t rows, cols;          // destination dims
    int32_t src_rows, src_cols;  // valid source extent (in destination orientation before transpose)
    int32_t src_ld, src_row0;
    int32_t transpose, perm;
    int32_t k4;        // 1: k4-blocked image W4[((r>>2)·cols + c)·4 + (r&3)] (16-byte A-operand fragments)
    int32_t bias_row;  // ≥ 0: destination row filled from a bias vector (PK_W3A row 150 = rmp.2 bias)
    int64_t bias_off;  // floats into the flat params of that bias vector
};
// A replayed step's prologue folded into the prep launch (spwgnn_run.prologue): its last row of
// workgroups copies the batch from pinned, device-mapped staging (as k_copy_in) and one thread
// advances the dropout key and step words (as k_step_advance) — two launches fewer per step.
struct PrologueArgs {
    const uint4* src;
    uint4* dst;
    int64_t n16;        // 16-byte units to copy (0: none)
    uint64_t* key;      // null: no advance
    int32_t* step;
    int32_t mode, rank;
    uint64_t seed;
};
struct PrepArgs {
    const float* params;
    float* pk;
    PackDesc desc[PK_COUNT];  // by value (kernel-argument memory): no host→device copy, capturable
    PrologueArgs pro;
    int32_t pro_row;          // 1: the launch's last row of workgroups runs `pro`
};

// Split-bf16 (x6) operand images of the weights, built in the same launch as the fp32 packs (k_prep)
// from the pack elements they hold (pack_elem: the values are computed from the flat params, not read back).
// Transposed-orientation A operands of tgemm_x6: [step u = kb·nt_out + T][part][lane] uint4 (8 bf16),
// element e of lane (i, h) = W[k(kb, e, h)][32T + i] with
//   kh == 0 (chain: B is a C layout)          k = 16kb + 8(e>>2) + 4h + (e&3)
//   kh > 0  (half rows: lane half h holds features kh·h ..)  k = kh·h + 8kb + e, zero if 8kb + e ≥ kh
// ht (half tile, 4-tile images of the chain kernels): slot T = 3 of k-block kb holds,
// when kb is odd or the last, the 16x16x32 A operand of k-block pair P = kb >> 1 for output columns
// 96..111: lane (i, g) = W[k(2P + (g&1), e, g>>1)][96 + i] (zero for a k-block ≥ nkb), otherwise zeros
enum X6Id : int {
    X6_RM1 = 0, X6_RM2, X6_RM3, X6_W1A,          // relation encoder (chains)
    X6_W1AT, X6_RM3T, X6_RM2T, X6_RM1T,           // its backward
    X6_W2, X6_W2T,                                // edge side (LDS B operands)
    X6_W3A, X6_WO1C, X6_WO1A, X6_WO1P, X6_WO2, X6_W1B, X6_W1C,   // node side
    X6_W1BT, X6_W1CT, X6_WO2T, X6_WO1PT, X6_WO1CT, X6_WO1AT, X6_W3T,   // its backward
    X6_OM1,                                       // object encoder
    X6_OM1T,                                      // its backward
    // half-tile forms of the 4-tile images (the chain kernels; the fused team kernels read the above)
    X6_W3A_H, X6_WO1C_H, X6_WO1A_H, X6_WO1P_H, X6_WO2_H,
    X6_W1BT_H, X6_W1CT_H, X6_WO2T_H, X6_WO1PT_H, X6_WO1CT_H, X6_WO1AT_H, X6_OM1_H, X6_OM1T_H,
    X6_COUNT
};
// (image, fp32 pack, output tiles, k-blocks, kh, ht) — the images every x6 run builds
struct X6Spec { int id, pack, nt_out, nkb, kh, ht = 0; };
constexpr X6Spec kX6Specs[X6_COUNT] = {
    {X6_RM1, PK_RM1, 5, 10, 0},    {X6_RM2, PK_RM2, 5, 10, 0},    {X6_RM3, PK_RM3, 5, 10, 0},
    {X6_W1A, PK_W1A, 5, 10, 0},    {X6_W1AT, PK_W1AT, 5, 10, kKhE}, {X6_RM3T, PK_RM3T, 5, 10, 0},
    {X6_RM2T, PK_RM2T, 5, 10, 0},  {X6_RM1T, PK_RM1T, 5, 10, 0},  {X6_W2, PK_W2, 5, 10, kKhE},
    {X6_W2T, PK_W2T, 5, 10, kKhE}, {X6_W3A, PK_W3A, 4, 10, kKhE}, {X6_WO1C, PK_WO1C, 4, 7, kKhN},
    {X6_WO1A, PK_WO1A, 4, 7, 0},   {X6_WO1P, PK_WO1P, 4, 7, kKhN}, {X6_WO2, PK_WO2, 4, 7, 0},
    {X6_W1B, PK_W1B, 5, 7, 0},     {X6_W1C, PK_W1C, 5, 7, 0},
    {X6_W1BT, PK_W1BT, 4, 10, kKhE}, {X6_W1CT, PK_W1CT, 4, 10, kKhE}, {X6_WO2T, PK_WO2T, 4, 7, 0},
    {X6_WO1PT, PK_WO1PT, 4, 7, 0}, {X6_WO1CT, PK_WO1CT, 4, 7, 0}, {X6_WO1AT, PK_WO1AT, 4, 7, 0},
    {X6_W3T, PK_W3T, 5, 7, 0},     {X6_OM1, PK_OM1, 4, 7, 0},
    {X6_OM1T, PK_OM1T, 4, 7, 0},
    {X6_W3A_H, PK_W3A, 4, 10, kKhE, 1}, {X6_WO1C_H, PK_WO1C, 4, 7, kKhN, 1}, {X6_WO1A_H, PK_WO1A, 4, 7, 0, 1},
    {X6_WO1P_H, PK_WO1P, 4, 7, kKhN, 1}, {X6_WO2_H, PK_WO2, 4, 7, 0, 1},
    {X6_W1BT_H, PK_W1BT, 4, 10, kKhE, 1}, {X6_W1CT_H, PK_W1CT, 4, 10, kKhE, 1}, {X6_WO2T_H, PK_WO2T, 4, 7, 0, 1},
    {X6_WO1PT_H, PK_WO1PT, 4, 7, 0, 1}, {X6_WO1CT_H, PK_WO1CT, 4, 7, 0, 1}, {X6_WO1AT_H, PK_WO1AT, 4, 7, 0, 1},
    {X6_OM1_H, PK_OM1, 4, 7, 0, 1},     {X6_OM1T_H, PK_OM1T, 4, 7, 0, 1},
};
// The half-tile form is a build option (-DSPWGNN_HT=1): measured −0.5 % at the
// headline, and it ends the bitwise equality of the chain and team kernels. Off, its images are empty.
#ifndef SPWGNN_HT
#define SPWGNN_HT 0
#endif
constexpr bool kHT = SPWGNN_HT != 0;
inline int x6_nkb(const X6Spec& s) { return s.ht && !kHT ? 0 : s.nkb; }
struct X6Desc {
    int32_t pack;       // source fp32 pack (PackId): element (k, col) of it
    int32_t nt_out, nkb;
    int32_t kh, ht;
    int64_t dst;        // uint4 offset into the image buffer
};
// the images k_prep builds: the half-tile forms only in kHT builds (kernel-argument space)
constexpr int X6_PREP_COUNT = kHT ? X6_COUNT : X6_W3A_H;
struct PrepX6Args {
    uint4* img;
    X6Desc d[X6_PREP_COUNT];
};
inline int64_t x6_chain_uint4(int nt_out, int nkb) { return (int64_t)nkb * nt_out * 3 * 64; }

struct EncNodeArgs {
    int n_nodes;
    const float* pos;
    const float* prop;
    const int32_t* node_tower;
    const int32_t* node_local;
    const float *w_om0, *b_om0, *w_om1, *b_om1, *w1b, *w1c;
    const uint4 *x_om1, *x_w1b, *x_w1c;   // x6 images (x6 math)
    const uint4* xh_om1;                  // its half-tile form (the chain kernel, §3w)
    float *zo1, *co, *P0, *U0, *V0;
    int uv16;                   // U0, V0 in bf16 math (training): kUvRound / kUvB16 (gemm_blocks.h store_cm_uv)
    int dropout_on;
    uint32_t thresh;
    float scale;
    uint64_t seed;
    const uint64_t* seed_dev;   // non-null: the dropout key is read from device memory (replayable steps)
};

struct EncEdgeArgs {
    int n_eblocks;
    const float* pos;
    const int32_t *esrc, *edst, *node_tower, *node_local;
    const float *w_rm0, *b_rm0, *w_rm1, *b_rm1, *w_rm2, *b_rm2, *w_rm3, *b_rm3, *w_w1a, *b_w1a;
    const uint4 *x_rm1, *x_rm2, *x_rm3, *x_w1a;   // x6 images (math == MATH_X6)
    float *z1, *z2, *z3, *cr, *A;   // chunk-major blocks (z1 null: the W1 gradient rebuilds it from ed)
    float2* ed;                     // training: per-edge (dx, dy), rows of the 32-edge blocks
    uint32_t* zmask;                // [blk][4 layers: z1,z2,z3,cr][3 words][64 lanes] — activation > 0 bits
    int b16;                        // bf16 math: z2, z3, c_r stored as bf16 (same element layout)
    int dropout_on;
    uint32_t thresh;
    float scale;
    uint64_t seed;
    const uint64_t* seed_dev;   // non-null: the dropout key is read from device memory (replayable steps)
};

// The run's dropout key: a kernel argument, or (graph-replayed training steps) a device word the
// step-advance kernel rewrites before each replay.
template <class Args>
__device__ __forceinline__ uint64_t run_seed(const Args& a) {
    return a.seed_dev ? *a.seed_dev : a.seed;
}

struct EdgeFwdArgs {
    int n_wtiles, nw_max, wpg;
    int n_nodes;       // receiver blocks: one block per node
    int recv_blocks;   // SPWGNN_BATCH_RECV_BLOCKS plan: k_edge_fwd_rb_x6 (x6 math)
    const int32_t *wtile, *esrc, *edst;
    const uint32_t* csr;
    const float *A, *U, *V, *w2, *b2;
    float* H2s;
    uint32_t *mask1, *mask2;
    float* h1_out;     // training: h1 rows, chunk-major blocks (kCmBlk), for the W2 gradient
    int a_b16;         // bf16 math (training): A stored as bf16
    int n16;           // bf16 math (training, wide kernels): H2s stored as bf16 (§3g, node side)
    int uv16;          // how U, V were stored (store_cm_uv): kUvB16 exactly when n16 (the N16 kernel reads bf16)
    const uint4* x_w2; // x6 image of W2 (half rows, kh 76) — the LDS B operand (math == MATH_X6)
};

struct NodeFwdArgs {
    int n_nodes;
    const float *H2s, *P, *co;
    float *a_out, *o1_out, *Pn, *logits, *U, *V;
    // x6/bf16: c_o·Wo1c is step-invariant — step 0 stores the accumulator after that product
    // (cw_out), later steps start from it (cw_in) instead of repeating the product
    const float* cw_in;
    float* cw_out;
    const float *w3a, *wo1c, *wo1a, *wo1p, *wo2, *w1b, *w1c, *bo1, *bo2p;
    const uint4 *x_w3a, *x_wo1c, *x_wo1a, *x_wo1p, *x_wo2, *x_w1b, *x_w1c;   // x6 images
    const uint4 *xh_w3a, *xh_wo1c, *xh_wo1a, *xh_wo1p, *xh_wo2;            // half-tile forms (chain kernel, §3w)
    int n16;        // bf16 math (training, wide kernels): H2s read and o1 stored as bf16 (§3g, node side)
    int uv16;       // U, V in bf16 math (training): kUvRound, or kUvB16 (exactly when n16)
};

struct NodeBwdArgs {
    int n_nodes;
    int first;      // 1 for the last propagation step (no incoming dP, dlogits present)
    int tail;       // 1: only compute dP0 = dPpart + dU·W1bᵀ + dV·W1cᵀ into dprop (ld 100)
    const float *dPin, *dU, *dV;   // from step s+1 (null when first)
    const float *Pn, *o1, *a;      // P_{s+1}, o1_s, a_s
    const float* dlogits;
    float *dx, *do1, *g, *G3, *dPout, *dco, *dprop;
    int dco_accumulate;
    int dco_sum;    // x6: no dco here; k_enc_node_bwd applies Wo1cᵀ once to Σ_s do1_s (linear)
    const float *w1bt, *w1ct, *wo2t, *wo1ct, *wo1at, *wo1pt, *w3t;
    const uint4 *x_w1bt, *x_w1ct, *x_wo2t, *x_wo1ct, *x_wo1at, *x_wo1pt, *x_w3t;   // x6 images
    const uint4 *xh_w1bt, *xh_w1ct, *xh_wo2t, *xh_wo1ct, *xh_wo1at, *xh_wo1pt;      // half-tile forms (§3w)
    int n16;        // bf16 math (training, wide kernels): dU, dV, o1 read and dx, g stored as bf16 (§3g)
    // spwgnn_bce_backward on the fused small-batch loop: the first step computes dlogits from the
    // logits and targets itself (k_bce_partial's expression, also stored to bce_dlogits) instead of
    // reading dlogits
    const float *bce_logits, *bce_targets;
    float* bce_dlogits;
    int64_t bce_n;
};

struct EdgeBwdArgs {
    int n_wtiles, nw_max, wpg;
    int dA_accumulate;
    int no_dA;         // x6/bf16: no dA here — k_dA_x6 rebuilds Σ_s dh1pre_s after the step loop
    const int32_t *wtile, *esrc, *edst;
    const uint32_t* csr;
    const uint32_t *mask1, *mask2;
    const float *G3, *w2t;
    float *dA, *dU, *dV;
    float* dh2_out;    // dh2pre rows, chunk-major blocks (kCmBlk), for the W2 gradient
    const uint4* x_w2t; // x6 image of W2ᵀ (half rows, kh 76) — the LDS B operand (math == MATH_X6)
    int n16;           // bf16 math (training, wide kernels): dU, dV stored as bf16 (§3g, node side)
};

struct DaArgs {           // k_dA_x6: dA = Σ_s dh1pre_s, recomputed per 32-edge block
    int n_eblocks, S;
    int b16;                             // bf16 math: dA stored as bf16 (row-major [e][160])
    int64_t g3_step, m1_step, m2_step;   // per-step strides (floats / u32 words)
    const int32_t* edst;
    const uint32_t *mask1, *mask2;
    const float* G3;
    float* dA;                           // row-major [e][160]
    const uint4* x_w2t;
};

struct EncEdgeBwdArgs {
    int n_eblocks;
    int b16;                        // bf16 math: dA read and dz4..dz1 stored as bf16
    const float* dA;                // row-major [e][160] (accumulated by k_edge_bwd)
    const uint32_t* zmask;          // from k_enc_edge
    const float *w1at, *rm3t, *rm2t, *rm1t;
    const uint4 *x_w1at, *x_rm3t, *x_rm2t, *x_rm1t;   // x6 images (math == MATH_X6)
    float *dz4, *dz3, *dz2, *dz1;
    float scale;   // dropout 1/(1-p) (1 when off)
};

struct EncNodeBwdArgs {
    int n_nodes;
    float* dco;                       // dc_o in; with wo1ct: Σ_s do1_s out
    const float *co, *zo1, *om1t;
    const float* pos;                 // zo1 null: its relu mask is rebuilt from (y, w) and om.0
    const float *w_om0, *b_om0;
    const float* wo1ct;               // non-null: dc_o = (Σ_s do1_s)·Wo1cᵀ here, from the per-step do1
                                      //   rows; Σ_s do1_s is stored into dco (Wo1c gradient)
    const float* do1;                 //   rows (do1 + s·do1_step, s < S) instead of dco
    int64_t do1_step;
    int S;
    float *dzo2, *dzo1;
    float scale;
    const uint4 *x_wo1ct, *x_om1t;    // split-bf16 maths: x6 images of Wo1cᵀ and om.1ᵀ
    const uint4 *xh_wo1ct, *xh_om1t;  // their half-tile forms (the chain kernel, §3w)
};

// ---- weight gradients: dW = Σ_rows X[row]ᵀ·Y[row] (deterministic split-row slabs) ----
enum XMode : int {
    XM_ROW = 0,     // ptr[phys_row * ld + f]; f == ones_col → 1 (row-major rows, width ld)
    XM_EDGE_D,      // (pos[dst] - pos[src])[f] for f < 2, f == 2 → 1; padding edge → 0
    XM_NODE_O,      // pos[n][1 + f] for f < 2, f == 2 → 1
    XM_CM,          // chunk-major edge blocks (kCmBlk per 32 rows, f < 152); f == ones_col → 1
    XM_H1,          // relu(A[e] + U_s[src] + V_s[dst]) recomputed (row = s·RE + e), f == ones_col → 1
};
enum YMode : int {
    YM_ROW = 0,
    YM_CM,          // chunk-major edge blocks
    YM_DH2,         // G3_s[dst] ⊙ [h2_s > 0] recomputed from the node rows and mask2 (row = s·RE + e)
};
struct WgradArgs {
    int64_t rows;          // logical rows L = s*count + n
    int64_t rows_per_chunk;
    int xmode, ymode;
    int kx_pad, ny_pad;    // multiples of 32, <= 160
    // X: physical row = (stride ? (L / count) * stride : 0) + L % count
    const float* x_ptr;
    int x_ld, x_width, x_ones;
    int64_t x_count, x_stride;
    // Y
    const float* y_ptr;
    int y_ld, y_width;
    int64_t y_count, y_stride;
    // edge/node context
    const float* pos;
    const int32_t *esrc, *edst;
    const float *A, *U, *V, *G3;   // chunk-major; U, V, G3 per step at s·RN·kRowE
    const uint32_t* mask2;         // per step at s·(RE/32)·kM2Blk
    int64_t RE, RN;
    int S;                         // steps (XM_H1 / YM_DH2 walk rows as (edge block, step) stages)
    int a_b16;                     // bf16 math: A stored as bf16 (k_w2grad_ws)
    int uv16;                      // bf16 math: U, V stored as bf16 (k_w2grad_tile only)
    const int32_t* wtile;          // the batch plan's wave-tiles (k_w2grad_tile walks whole tiles)
    int n_wtiles, nw_max;
    int w2_tile;                   // 1: the W2 gradient with LDS-staged node rows (bf16 math)
    float* slab;           // [chunks][kx_pad][ny_pad]
};
struct WgWsArgs {          // k_wgrad_ws: stages (s, nb) of a [S][nbs] grid of 32-row blocks
    const float* x;        // chunk-major
    const float* y;        // chunk-major, or row-major with stride 160 (yrow)
    const float2* xd;      // XD 1: per-edge (dx, dy); X = [relu(rm.0(dx, dy)) | 1] (= z1) is rebuilt
    const float4* xp;      // XD 2: node positions; X = [relu(om.0(y, w)) | 1] (= zo1) is rebuilt
    const float *w0, *b0;  // XD: the first-layer pack [2][KXP] and its bias [KXP]
    float* slab;           // [wgs][kx_pad][ny_pad]
    int64_t nbs, S, x_sb, y_sb, count, stages_per_wg;
    int x_ones, pad0;
};
// bf16 storage of the weight gradients' edge operands (bf16 math, §3g): bit 0 X, bit 1 Y
enum : int { kB16X = 1, kB16Y = 2, kB16A = 4, kB16UV = 8 };   // kB16A / kB16UV: the W2 gradient's A / U, V rows
struct ReduceArgs {
    const float* slab;
    int chunks, kx_pad, ny_pad;
    float* out;            // flat grads base
    int64_t kernel_off;    // tensor offset (kernel), -1 none
    int kernel_rows, kernel_cols, kernel_row0;  // write rows [0, kernel_rows) of slab → tensor rows kernel_row0+
    int64_t bias_off;      // tensor offset (bias), -1 none
    int bias_row;          // slab row holding the bias (ones column)
    int perm;              // 1: omp.1 column permutation (slab col f' → tensor col wo2_perm(f'))
};

// k_wgrad_ws shapes (KXP × NYP, Y row-major, rebuilt X, bf16-stored operands) as one batched launch
enum WsVariant : int {
    WSV_160_160 = 0, WSV_160_160_ROW, WSV_128_160, WSV_160_128, WSV_128_128, WSV_XD_EDGE, WSV_XD_NODE,
    WSV_XD_EDGE_B16Y, WSV_160_160_ROW_B16, WSV_160_160_B16,   // bf16 math only
    WSV_128_160_B16Y, WSV_160_128_B16, WSV_128_128_B16,        // bf16 math, bf16-stored node arrays
    WSV_NONE = -1
};
struct WsJob {
    WgWsArgs a;
    int variant, wg0;      // WsVariant; first workgroup of the job in the batched grid
    int gn, gi;            // operand-sharing group (ws_group): its size (≤ 1: none) and this job's index
};
constexpr int kMaxWsJobs = 16;
struct WsBatch {           // the k_wgrad_ws gradients of one backward (k_wgrad_ws_batch)
    WsJob j[kMaxWsJobs];
    int n, wgs;
    // a small batch's x6 W2 gradient (k_w2grad_ws) as the launch's last w2_wgs workgroups (0: none)
    WgradArgs w2;
    int64_t w2_bpw;
    int w2_wgs;
};

constexpr int kMaxReduce = 16;
constexpr int kMaxZero = 48;
struct BceArgs {
    const float *logits, *targets;
    int64_t n;
    float* dlogits;
    float* partial;   // [blocks][2]
    float* out3;
    int blocks;
    const double* w3;   // non-null: tot3[k] += (double)out3[k] * w3[k] by the thread that writes out3
    double* tot3;
};
// Keras binary_crossentropy (Networks.py:102): clip(ŷ, 1e-7, 1-1e-7) ≡ clamp(z, ±ln((1-ε)/ε)).
constexpr float kLogitClip = 16.11809565f;
// dL/dz of one node (k_bce_partial's expression; the fused backward's inline form uses it too)
__device__ __forceinline__ float bce_dlogit(float z0, float t, float inv_n) {
    const float p = 1.f / (1.f + expf(-z0));
    return fabsf(z0) < kLogitClip ? (p - t) * inv_n : 0.f;
}
struct ReduceBatch {       // the weight gradients of one backward, reduced in one launch (blockIdx.y)
    ReduceArgs r[kMaxReduce];
    int n;
    // 1: the launch's last row (its first workgroup) is k_bce_partial<true> on `bce` (one workgroup's
    // loss / accuracy sums: spwgnn_bce_backward's loss, off the backward's critical path)
    int bce_row;
    BceArgs bce;
    // float ranges of the flat gradient buffer no reduction writes (the 64-float alignment gaps between
    // tensors, tensors without rows in this batch): zeroed by the extra row blockIdx.y == n of the
    // same launch (was a separate hipMemsetAsync of the whole buffer before the backward)
    int nzero;
    int64_t zoff[kMaxZero];
    int32_t zlen[kMaxZero];
};
struct AdamArgs {
    float *p, *m, *v;
    const float* g;
    int64_t n;
    float lr_t, b1, b2, eps, l2, gscale;
    const int32_t* step_dev;   // non-null: lr_t = lr_table[min(*step_dev, table_len - 1)]
    const float* lr_table;
    int32_t table_len;
};

// Host launchers (defined next to their kernels; each returns hipGetLastError()).
// packs and (x: non-null) the x6 images in one launch
hipError_t launch_prep(const PrepArgs& a, const PrepX6Args* x, hipStream_t st);
hipError_t launch_enc_node(const EncNodeArgs& a, int math, hipStream_t st);
hipError_t launch_enc_edge(const EncEdgeArgs& a, int math, hipStream_t st);
hipError_t launch_edge_fwd(const EdgeFwdArgs& a, int math, hipStream_t st);
hipError_t launch_node_fwd(const NodeFwdArgs& a, int math, hipStream_t st);
hipError_t launch_node_bwd(const NodeBwdArgs& a, int math, hipStream_t st);
hipError_t launch_edge_bwd(const EdgeBwdArgs& a, int math, hipStream_t st);
hipError_t launch_enc_edge_bwd(const EncEdgeBwdArgs& a, int math, hipStream_t st);
hipError_t launch_dA(const DaArgs& a, int math, hipStream_t st);
hipError_t launch_enc_node_bwd(const EncNodeBwdArgs& a, int math, hipStream_t st);
enum MathMode : int { MATH_F32 = 0, MATH_X6 = 1, MATH_BF16 = 2 };   // = SPWGNN_MATH_* (spwgnn.h)
hipError_t launch_wgrad(const WgradArgs& a, int chunks, int math, hipStream_t st);
hipError_t launch_wgrad_ws(const WgWsArgs& a, int wgs, int kx_pad, int ny_pad, int yrow, int mask, int math,
                           hipStream_t st, int b16 = 0);
// the variant k_wgrad_ws runs for these arguments (WSV_NONE: no such kernel)
int wgrad_ws_variant(const WgWsArgs& a, int kx_pad, int ny_pad, int yrow, int mask, int math, int b16);
struct Pos3Batch;
// p3: a small batch's k_wgrad_pos3 gradients as trailing workgroups of the same launch
hipError_t launch_wgrad_ws_batch(const WsBatch& b, int math, hipStream_t st, const Pos3Batch* p3 = nullptr);
hipError_t launch_wgrad_bf16(const WgradArgs& a, int chunks, hipStream_t st, int b16 = 0);
hipError_t launch_w2grad_ws(const WgradArgs& a, int wgs, int64_t blk_per_wg, int math, hipStream_t st);
hipError_t launch_wgrad_reduce_all(const ReduceBatch& rb, hipStream_t st);
// k_wgrad_pos3: the 3-column first-layer gradients (rm.0, om.0) in the split-bf16 maths
struct Pos3Args {
    const float* y;          // chunk-major Y (fp32, or bf16 with the fp32 element layout: b16)
    const float4* pos;       // om.0: X = (y, w) of the node positions
    const float2* ed;        // rm.0: the encoder's per-edge (dx, dy) (padding edge: esrc < 0 → X = 0)
    const int32_t* esrc;
    float* slab;             // [chunks][32][NYP]
    int64_t nblk, blk_per_wg, count;
};
struct Pos3Batch {          // the backward's two k_wgrad_pos3 gradients, one launch
    Pos3Args e, n;         // rm.0 (edge rows), om.0 (node rows)
    int ce, cn;            // their workgroups (0: not queued)
    int b16e;              // rm.0's Y (dz1) stored as bf16
};
hipError_t launch_wgrad_pos3(const Pos3Batch& p, hipStream_t st);
hipError_t launch_bce(const BceArgs& a, hipStream_t st);
hipError_t launch_adam(const AdamArgs& a, hipStream_t st);
hipError_t launch_step_advance(uint64_t* key, int32_t* step, int mode, uint64_t seed, int32_t rank, hipStream_t st);
hipError_t launch_sigmoid(const float* z, float* p, int64_t n, hipStream_t st);
hipError_t launch_accumulate_out3(const float* out3, const double* w, double* tot, hipStream_t st);
hipError_t launch_copy_in(const void* src, void* dst, int64_t n16, hipStream_t st);
hipError_t launch_tower_readout(const float* z, const int32_t* off, int n_towers, int mode, float* out, hipStream_t st);

// Team kernels (kernels_team.hip): one block per workgroup of waves that split each layer's output
// tiles — the latency-bound small batches (the reference's batch 32) up to kTeamMaxBlocks blocks
#ifndef SPWGNN_TEAM_MAX_BLOCKS   // diagnosis builds lift it to time the team / fused kernels at large batches
#define SPWGNN_TEAM_MAX_BLOCKS 512
#endif
constexpr int kTeamMaxBlocks = SPWGNN_TEAM_MAX_BLOCKS;
bool team_blocks(int n_blocks);   // 32-row blocks of the launch (edge or node blocks)
int team_max_blocks(int set);      // set >= 0: the new limit (returns the previous one); < 0: query
hipError_t launch_enc_node_team(const EncNodeArgs& a, int math, hipStream_t st);
hipError_t launch_edge_fwd_team(const EdgeFwdArgs& a, int math, hipStream_t st);
hipError_t launch_edge_bwd_team(const EdgeBwdArgs& a, int math, hipStream_t st);
hipError_t launch_dA_team(const DaArgs& a, int math, hipStream_t st);
hipError_t launch_enc_node_bwd_team(const EncNodeBwdArgs& a, int math, hipStream_t st);
hipError_t launch_node_fwd_team(const NodeFwdArgs& a, int math, hipStream_t st);
hipError_t launch_node_bwd_team(const NodeBwdArgs& a, int math, hipStream_t st);
hipError_t launch_enc_edge_team(const EncEdgeArgs& a, int math, bool train, hipStream_t st);
// both encoders of a small batch in one launch (when both would take their team form)
bool enc_pair_team(int n_eblocks, int n_nodes, int math);
hipError_t launch_enc_pair_team(const EncEdgeArgs& e, const EncNodeArgs& n, int math, bool train, hipStream_t st);
hipError_t launch_enc_edge_bwd_team(const EncEdgeBwdArgs& a, int math, hipStream_t st);
// A small batch's S-step forward loop in ONE launch (after k_enc_pair_team; `encoders` puts both
// encoders in front of it instead): one workgroup per wave-tile runs the S propagation steps (edge
// side, node side), separated by workgroup barriers — a wave-tile holds whole towers, so no row it
// reads is written by another workgroup. The step arrays are the step-0 pointers of ef/nf; step s adds the run's per-step
// strides (Ws::*_at: per step when training, U/V/H2s shared and P alternating when not).
struct FwdFusedArgs {
    EncEdgeArgs ee;
    EncNodeArgs en;
    EdgeFwdArgs ef;       // U, V, H2s, mask1, mask2 of step 0
    NodeFwdArgs nf;       // P, Pn, a_out, o1_out, U, V of step 0; cw_out (step 0) / cw_in (later)
    int S, training;
    int encoders;             // 1: both encoders first, in this launch; 0: they ran before (k_enc_pair_team)
    int64_t rowsN, rowsE;     // floats per step of a 104- / 152-feature node array (RN·kRowN, RN·kRowE)
    int64_t m1_step, m2_step; // u32 words per step of mask1 / mask2
    float* logits;
};
bool fwd_fused_team(int n_wtiles, int nw_max, int n_eblocks, int n_nodes, int math);
// ... and its backward up to the weight gradients (same batches): per wave-tile the S steps' node
// and edge sides, d/d 'propagation', the dA rebuild, both encoder backwards. nb holds step 0's
// pointers (Pn = P_at(1), dPout = dP_at(0), dU/dV = dU_at(1)/dV_at(1): the incoming gradients of
// step 0); eb holds step 0's (mask1/2, G3, dU, dV); tail (has_tail) the dprop pass.
struct BwdFusedArgs {
    NodeBwdArgs nb, tail;
    EdgeBwdArgs eb;
    DaArgs da;
    EncEdgeBwdArgs eeb;
    EncNodeBwdArgs enb;
    int S, has_tail;
    int encoders;   // 1: dA rebuild and both encoder backwards in this launch; 0: k_bwd_enc_pair_team after it
    int dA_in_loop; // 1: this launch leaves dA (Σ_s dh1pre_s summed in LDS through the step loop)
    int64_t rowsN, rowsE, m1_step, m2_step;
};
hipError_t launch_fwd_fused_team(const FwdFusedArgs& a, int math, bool train, hipStream_t st);
hipError_t launch_bwd_fused_team(const BwdFusedArgs& a, int math, hipStream_t st);
hipError_t launch_bwd_enc_pair_team(const DaArgs& da, const EncEdgeBwdArgs& eeb, const EncNodeBwdArgs& enb, int math,
                                    int with_dA, hipStream_t st);

// LDS bytes per wave of the edge kernels (stage [2][32][33] + node accumulators)
// persistent edge-kernel grid: one 8-wave workgroup per CU (at most one wave-tile per wave)
int edge_grid(int n_wtiles, int waves = kEdgeWaves);
inline size_t edge_fwd_lds_per_wave(int nw_max) { return (size_t)(2112 + nw_max * kLdE) * 4; }
inline size_t edge_bwd_lds_per_wave(int nw_max) { return (size_t)(2112 + 2 * nw_max * kLdE) * 4; }
inline int edge_wpg(size_t lds_per_wave) {
    // waves per workgroup: keep a workgroup's LDS <= 80 KiB so two workgroups share a CU
    if (4 * lds_per_wave <= 80 * 1024) return 4;
    if (2 * lds_per_wave <= 80 * 1024) return 2;
    return 1;
}

}  // namespace spw
