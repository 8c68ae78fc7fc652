// C-ABI entry points of libspwgnn_hip.so: workspace layout and launch sequences.
#include <cmath>
#include <cstring>
#include <cstdlib>
#include "kernels.h"
#include <vector>
#include "../../include/spwgnn.h"
static_assert(SPWGNN_MATH_F32 == spw::MATH_F32 && SPWGNN_MATH_X6 == spw::MATH_X6 && SPWGNN_MATH_BF16 == spw::MATH_BF16,
              "math ids");

namespace spw {

static inline int64_t up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }

// ---------------------------------------------------------------- workspace layout -----------
struct Ws {
    int64_t total = 0;  // bytes
    int S, training;
    int64_t RN, RE, NB;
    // floats offsets (bytes / 4) — every array starts on 256 bytes
    int64_t pk;
    int64_t cw;                                      // node: c_o·Wo1c (x6/bf16 node forward)
    int64_t zo1, co, P, a, o1, U, V, H2s;           // node
    int64_t A, z1, z2, z3, cr;                       // edge
    int64_t ed;                                      // per-edge (dx, dy) float2 (training)
    int64_t mask1, mask2, zmask;                     // u32
    int64_t dx, do1, g, G3, dU, dV, dP, dco, dzo2, dzo1;   // node (bwd)
    int64_t dA, dz4, dz3, dz2, dz1;                  // edge (bwd)
    int64_t H1, DH2;                                 // per step: h1 (fwd) and dh2pre (bwd) rows for the W2 gradient
    int64_t slab, bce;
    int64_t slab_floats, slot_floats;   // weight-gradient slabs: kWgSlots slots of slot_floats
    PackSlots ps;
    int64_t x6;                                      // split-bf16 weight images (uint4 units below)
    int64_t x6off[X6_COUNT];
    int sP() const { return training ? S + 1 : 2; }
    int sStep() const { return training ? S : 1; }
    // node arrays are chunk-major (104 / 152 floats per row): a step's rows are RN/32 blocks
    int64_t P_at(int s) const { return P + (int64_t)(training ? s : (s & 1)) * RN * kRowN; }
    int64_t U_at(int s) const { return U + (int64_t)(training ? s : 0) * RN * kRowE; }
    int64_t V_at(int s) const { return V + (int64_t)(training ? s : 0) * RN * kRowE; }
    int64_t H2s_at(int s) const { return H2s + (int64_t)(training ? s : 0) * RN * kRowE; }
    int64_t a_at(int s) const { return a + (int64_t)s * RN * kRowN; }
    int64_t o1_at(int s) const { return o1 + (int64_t)s * RN * kRowN; }
    int64_t m1_at(int s) const { return mask1 + (int64_t)s * NB * kLdE; }
    int64_t m2_at(int s) const { return mask2 + (int64_t)s * NB * kM2Blk; }
    int64_t dx_at(int s) const { return dx + (int64_t)s * RN * kRowN; }
    int64_t do1_at(int s) const { return do1 + (int64_t)s * RN * kRowN; }
    int64_t g_at(int s) const { return g + (int64_t)s * RN * kRowN; }
    int64_t G3_at(int s) const { return G3 + (int64_t)s * RN * kRowE; }
    int64_t dU_at(int s) const { return dU + (int64_t)s * RN * kRowE; }
    int64_t dV_at(int s) const { return dV + (int64_t)s * RN * kRowE; }
    int64_t dP_at(int k) const { return dP + (int64_t)(k & 1) * RN * kRowN; }
    int64_t H1_at(int s) const { return H1 + (int64_t)s * NB * kCmBlk; }
    int64_t DH2_at(int s) const { return DH2 + (int64_t)s * NB * kCmBlk; }
};

static constexpr int kMaxChunks = 256;   // slabs per weight gradient (the ws kernels: one per CU)
static constexpr int kWgSlots = kMaxReduce; // weight gradients per backward, reduced by one batched launch
static constexpr int kW2gWgs = 256;   // W2 gradient: one workgroup per CU (MI355X: 256 CUs)
// batched weight gradients (k_wgrad_ws_batch): the jobs share one grid, so a job need not fill the chip
// by itself — a workgroup takes ≥ kWsMinStages 32-row stages (its 160×160 slab, written here and read
// by the reduction, stays small against its operands) while a job keeps ≥ kWsMinWgs workgroups
static constexpr int kWsMinStages = 32;
static constexpr int kWsMinWgs = 32;
// ... and a small job (a small batch's: fewer than kWsMinWgs·kWsSmallStages stages) gives each
// workgroup ≥ kWsSmallStages stages: every workgroup writes a whole 160×160 slab (100 KB) that the
// reduction reads back, ≈ 2.5 stages' worth of operand bytes — one stage per workgroup made the slabs
// most of the small step's weight-gradient traffic (Keras fit at batch 32: ≈ 360 slabs, 36 MB)
#ifndef SPWGNN_WS_SMALL_STAGES
#define SPWGNN_WS_SMALL_STAGES 4
#endif
static constexpr int kWsSmallStages = SPWGNN_WS_SMALL_STAGES;
// Diagnosis switches (A/B of superseded kernels, per-kernel math) exist only in -DSPWGNN_DIAG builds;
// the shipping library has no environment-dependent code path.
static bool getenv_flag(const char* name) {
#ifdef SPWGNN_DIAG
    const char* e = getenv(name);
    return e && *e && *e != '0';
#else
    (void)name;
    return false;
#endif
}

static Ws make_ws(int64_t n_nodes, int64_t n_eblocks, int S, int training) {
    Ws w;
    w.S = S;
    w.training = training;
    w.RN = up(std::max<int64_t>(n_nodes, 1), 32);
    w.NB = n_eblocks;
    w.RE = n_eblocks * 32;
    int64_t cur = 0;  // floats
    auto take = [&](int64_t nfl) {
        int64_t o = cur;
        cur += up(nfl, 64);
        return o;
    };
    // packs
    int64_t poff = 0;
    for (int id = 0; id < PK_COUNT; ++id) {
        w.ps.off[id] = poff;
        poff += up((int64_t)pack_rows(id) * pack_cols(id), 64);
    }
    w.ps.total = poff;
    w.pk = take(poff);
    {   // x6 images (uint4 = 4 floats each)
        int64_t o = 0;
        for (int id = 0; id < X6_COUNT; ++id) {
            w.x6off[id] = o;
            o += x6_chain_uint4(kX6Specs[id].nt_out, x6_nkb(kX6Specs[id]));
        }
        w.x6 = take(o * 4);
    }
    const int64_t nN = w.RN * kRowN, nE = w.RN * kRowE, eE = w.RE * kLdE;
    w.co = take(nN);
    w.cw = take(nN);
    w.P = take(nN * w.sP());
    w.U = take(nE * w.sStep());
    w.V = take(nE * w.sStep());
    w.H2s = take(nE * w.sStep());
    const int64_t eCM = w.NB * kCmBlk;   // chunk-major edge rows
    w.A = take(eCM);
    if (training) {
        w.zo1 = take(nN);
        w.a = take(nN * S);
        w.o1 = take(nN * S);
        w.z1 = take(eCM);
        w.ed = take(w.RE * 2);
        w.z2 = take(eCM);
        w.z3 = take(eCM);
        w.cr = take(eCM);
        w.mask1 = take(w.NB * kLdE * S);
        w.zmask = take(w.NB * 4 * 3 * 64);
        w.mask2 = take(w.NB * kM2Blk * S);
        w.dx = take(nN * S);
        w.do1 = take(nN * S);
        w.g = take(nN * S);
        w.G3 = take(nE * S);
        w.dU = take(nE * S);
        w.dV = take(nE * S);
        w.dP = take(nN * 2);
        w.dco = take(nN);
        w.dzo2 = take(nN);
        w.dzo1 = take(nN);
        w.dA = take(eE);
        w.dz4 = take(eCM);
        w.dz3 = take(eCM);
        w.dz2 = take(eCM);
        w.dz1 = take(eCM);
        // a slot holds ≥ 256 160×160 slabs (one per CU for the ws kernels) and up to 1024 for the
        // row-chunked kernels of large batches (chunks of ≥ 512 rows)
        const int64_t rows = std::max(w.RE, w.RN) * S;
        const int64_t slot_chunks = std::min<int64_t>(1024, std::max<int64_t>(kMaxChunks, (rows + 511) / 512));
        w.slot_floats = slot_chunks * 160 * 160;
        w.slab_floats = (int64_t)kWgSlots * w.slot_floats;
        w.slab = take(w.slab_floats);
    } else {
        w.ed = -1;
        w.zo1 = w.a = w.o1 = w.z1 = w.z2 = w.z3 = w.cr = w.mask1 = w.mask2 = w.zmask = -1;
        w.dx = w.do1 = w.g = w.G3 = w.dU = w.dV = w.dP = w.dco = w.dzo2 = w.dzo1 = -1;
        w.dA = w.dz4 = w.dz3 = w.dz2 = w.dz1 = w.slab = w.H1 = w.DH2 = -1;
        w.slab_floats = w.slot_floats = 0;
    }
    w.total = cur * 4;
    return w;
}

// ---------------------------------------------------------------- weight packs ---------------
static void build_packs(const Ws& w, PrepArgs& pa) {
    const ParamTable& pt = param_table();
    auto T = [&](int id) { return pt.t[id]; };
    auto mk = [&](int pid, int tid, int src_rows, int src_cols, int row0, int transpose, int perm) {
        PackDesc d{};
        d.dst_off = w.ps.off[pid];
        d.src_off = T(tid).offset;
        d.rows = pack_rows(pid);
        d.cols = pack_cols(pid);
        d.src_rows = src_rows;
        d.src_cols = src_cols;
        d.src_ld = T(tid).cols;
        d.src_row0 = row0;
        d.transpose = transpose;
        d.perm = perm;
        // A operands of the transposed-orientation MLP chains are k4-blocked (gemm_blocks.h);
        // W2/W2ᵀ (LDS images built by the edge kernels), rm.0/om.0 and the biases stay row-major
        d.k4 = !(pid == PK_W2 || pid == PK_W2T || pid == PK_RM0 || pid == PK_OM0 || pack_rows(pid) == 1);
        d.bias_row = -1;
        pa.desc[pid] = d;
    };
    // forward [in][out]
    mk(PK_RM1, T_RM1K, 150, 150, 0, 0, 0);
    mk(PK_RM2, T_RM2K, 150, 150, 0, 0, 0);
    mk(PK_RM3, T_RM3K, 150, 150, 0, 0, 0);
    mk(PK_W1A, T_RMP0K, 150, 150, 0, 0, 0);
    mk(PK_OM1, T_OM1K, 100, 100, 0, 0, 0);
    mk(PK_W1B, T_RMP0K, 100, 150, 150, 0, 0);
    mk(PK_W1C, T_RMP0K, 100, 150, 250, 0, 0);
    mk(PK_W2, T_RMP1K, 150, 150, 0, 0, 0);
    mk(PK_W3A, T_RMP2K, 150, 100, 0, 0, 0);
    pa.desc[PK_W3A].bias_row = 150;             // row 150 = rmp.2 bias (the degree column multiplies it)
    pa.desc[PK_W3A].bias_off = T(T_RMP2B).offset;
    mk(PK_WO1C, T_OMP0K, 100, 100, 0, 0, 0);
    mk(PK_WO1A, T_OMP0K, 100, 100, 100, 0, 0);
    mk(PK_WO1P, T_OMP0K, 100, 100, 200, 0, 0);
    mk(PK_WO2, T_OMP1K, 100, 101, 0, 0, 1);
    // backward transposes: dst[r][c] = src[c + row0][perm? (r)]; (transpose: source row = c, source col = r)
    mk(PK_W2T, T_RMP1K, 150, 150, 0, 1, 0);
    mk(PK_W1BT, T_RMP0K, 100, 150, 150, 1, 0);
    mk(PK_W1CT, T_RMP0K, 100, 150, 250, 1, 0);
    mk(PK_WO2T, T_OMP1K, 100, 101, 0, 1, 1);
    mk(PK_WO1CT, T_OMP0K, 100, 100, 0, 1, 0);
    mk(PK_WO1AT, T_OMP0K, 100, 100, 100, 1, 0);
    mk(PK_WO1PT, T_OMP0K, 100, 100, 200, 1, 0);
    mk(PK_W3T, T_RMP2K, 150, 100, 0, 1, 0);
    mk(PK_W1AT, T_RMP0K, 150, 150, 0, 1, 0);
    mk(PK_RM3T, T_RM3K, 150, 150, 0, 1, 0);
    mk(PK_RM2T, T_RM2K, 150, 150, 0, 1, 0);
    mk(PK_RM1T, T_RM1K, 150, 150, 0, 1, 0);
    mk(PK_OM1T, T_OM1K, 100, 100, 0, 1, 0);
    // biases (rows = 1)
    mk(PB_RM1, T_RM1B, 1, 150, 0, 0, 0);
    mk(PB_RM2, T_RM2B, 1, 150, 0, 0, 0);
    mk(PB_RM3, T_RM3B, 1, 150, 0, 0, 0);
    mk(PB_W1A, T_RMP0B, 1, 150, 0, 0, 0);
    mk(PB_W2, T_RMP1B, 1, 150, 0, 0, 0);
    mk(PB_OM1, T_OM1B, 1, 100, 0, 0, 0);
    mk(PB_O1, T_OMP0B, 1, 100, 0, 0, 0);
    mk(PB_O2P, T_OMP1B, 1, 101, 0, 0, 1);
    mk(PK_RM0, T_RM0K, 2, 150, 0, 0, 0);
    mk(PK_OM0, T_OM0K, 2, 100, 0, 0, 0);
    mk(PB_RM0, T_RM0B, 1, 150, 0, 0, 0);
    mk(PB_OM0, T_OM0B, 1, 100, 0, 0, 0);
}

struct Ctx {
    const Ws& w;
    char* base;
    float* f(int64_t off) const { return off < 0 ? nullptr : reinterpret_cast<float*>(base) + off; }
    uint32_t* u(int64_t off) const { return off < 0 ? nullptr : reinterpret_cast<uint32_t*>(base) + off; }
    const float* pk(int id) const { return reinterpret_cast<const float*>(base) + w.pk + w.ps.off[id]; }
    const uint4* x6(int id) const { return reinterpret_cast<const uint4*>(reinterpret_cast<const float*>(base) + w.x6) + w.x6off[id]; }
};

static int32_t validate(const spwgnn_batch* b, const spwgnn_run* r) {
    if (!b || !r) return SPWGNN_E_ARG;
    if (b->n_nodes < 1 || b->n_wtiles < 1 || b->n_eblocks < 1) return SPWGNN_E_SHAPE;
    if (b->nw_max < 1 || b->nw_max > kNwMaxLimit) return SPWGNN_E_SHAPE;
    if (r->mp_steps < 1 || r->mp_steps > 64) return SPWGNN_E_SHAPE;
    if (!b->pos || !b->wtile || !b->edge_src || !b->edge_dst || !b->blk_csr) return SPWGNN_E_ARG;
    if (r->dropout < 0.f || r->dropout >= 1.f) return SPWGNN_E_ARG;
    if (r->math != SPWGNN_MATH_F32 && r->math != SPWGNN_MATH_X6 && r->math != SPWGNN_MATH_BF16) return SPWGNN_E_ARG;
    if (r->training && r->dropout > 0.f && (!b->node_tower || !b->node_local)) return SPWGNN_E_ARG;
    return SPWGNN_OK;
}

// Per-kernel x6 selection for A/B diagnosis: SPWGNN_X6_KERNELS (bit mask of kX6*, default all)
// narrows math == MATH_X6 (or MATH_BF16) to some kernels; the others run in f32 math.
enum : int { kX6EncEdge = 1, kX6EdgeFwd = 2, kX6NodeFwd = 4, kX6NodeBwd = 8, kX6EdgeBwd = 16, kX6EncEdgeBwd = 32,
             kX6Wgrad = 64 };
static int kmath(const spwgnn_run* r, int bit) {
#ifdef SPWGNN_DIAG
    static const int mask = [] {
        const char* e = getenv("SPWGNN_X6_KERNELS");
        return e ? (int)strtol(e, nullptr, 0) : -1;
    }();
#else
    constexpr int mask = -1;
#endif
    return (r->math != MATH_F32 && (mask & bit)) ? r->math : MATH_F32;
}

// The rm.1 / om.1 weight gradients rebuild their operands z1 = relu(rm.0(d)) and zo1 = relu(om.0(y, w))
// on the staging waves of k_wgrad_ws from the per-edge d (8 bytes) and the node positions, so the
// encoders store d instead of the 608-byte z1 rows and no zo1 rows.
static bool z1_rebuilt(const spwgnn_run* r) {
    return r->training && kmath(r, kX6Wgrad) != MATH_F32 && !getenv_flag("SPWGNN_WG_OLD");
}

struct Prof {
    const spwgnn_run* r;
    hipStream_t st;
    mutable int k = 0;
    hipError_t before(int kid) const {
        if (r->prof_kernel != kid || !r->prof_events || k >= r->prof_count) return hipSuccess;
        return hipEventRecord(static_cast<hipEvent_t>(r->prof_events[2 * k]), st);
    }
    hipError_t after(int kid) const {
        if (r->prof_kernel != kid || !r->prof_events || k >= r->prof_count) return hipSuccess;
        hipError_t e = hipEventRecord(static_cast<hipEvent_t>(r->prof_events[2 * k + 1]), st);
        ++k;
        return e;
    }
};

#define SPW_CHECK(x)                                  \
    do {                                              \
        hipError_t e_ = (x);                          \
        if (e_ != hipSuccess) return (int32_t)e_;     \
    } while (0)

// dA = Σ_s dh1pre_s: rebuilt once after the step loop (k_dA_x6 / k_dA_team) instead of being
// accumulated into HBM by every step's edge backward — float atomics bounded that kernel (A/B on one
// box: x6 step 28.11 → 27.39 ms, bf16 config 3 71.5 → 69.3 ms), and so do plain read-add-writes in
// the rebuild's order (bitwise the same dA; headline 25.7 → 28.9 ms, round 4) — DESIGN.md §3f.
// SPWGNN_DA_RMW (diagnosis builds only) selects the read-add-write form for A/B.
static bool rebuild_dA(const spwgnn_run* r, const spwgnn_batch* b) {
    const int m = kmath(r, kX6EdgeBwd);
    return b->nw_max <= 16 && m != MATH_F32 && !(m == MATH_X6 && !team_blocks(b->n_wtiles) && getenv_flag("SPWGNN_DA_RMW"));
}

// bf16 math (training) stores the encoder-side edge arrays that only ever feed MFMA operands — z2, z3,
// c_r, dz4..dz1 and dA — as bf16 (exact: the operands are rounded to bf16 anyway), and the step-invariant
// A as bf16 (rounded once before h1 = relu(A + U + V)). Every kernel that writes or
// reads them must run in bf16 math for the layouts to agree.
static bool store_b16(const spwgnn_run* r, const spwgnn_batch* b) {
    return r->training && r->math == MATH_BF16 && kmath(r, kX6EncEdge) == MATH_BF16 &&
           kmath(r, kX6EncEdgeBwd) == MATH_BF16 && kmath(r, kX6Wgrad) == MATH_BF16 && rebuild_dA(r, b) &&
           !getenv_flag("SPWGNN_WG_OLD");
}

// ... and, when every kernel that writes or reads them runs its wide (non-team) form, the node-side
// per-step arrays that only ever feed MFMA operands: H2s (node forward's W3 product, W3 gradient),
// o1 (omp.1 gradient; the node backward reads only its sign), dU, dV (node backward's W1bᵀ/W1cᵀ
// products, W1b/W1c gradients), g (W3 gradient) and dx (omp.1 gradient) — exact as above.
static bool store_b16_node(const spwgnn_run* r, const spwgnn_batch* b) {
    return store_b16(r, b) && kmath(r, kX6EdgeFwd) == MATH_BF16 && kmath(r, kX6NodeFwd) == MATH_BF16 &&
           kmath(r, kX6NodeBwd) == MATH_BF16 && kmath(r, kX6EdgeBwd) == MATH_BF16 && b->nw_max <= 16 &&
           !team_blocks(b->n_wtiles) && !team_blocks((b->n_nodes + 31) / 32) && !getenv_flag("SPWGNN_NODE_F32");
}

// U = P·W1b and V = P·W1c in bf16 math (training): rounded to bf16 when stored (oracle/bf16.py,
// DESIGN.md §3ze), and stored as bf16 exactly when the node-side arrays are (every writer and reader a
// wide kernel: the node forward, the object encoder, the N16 edge forward, k_w2grad_tile).
static int uv_storage(const spwgnn_run* r, const spwgnn_batch* b) {
    if (!r->training || r->math != MATH_BF16) return kUvF32;
    return store_b16_node(r, b) ? kUvB16 : kUvRound;
}

// Whether a forward / backward takes the fused small-batch step loops. One place for
// the gate: run_forward, run_backward and spwgnn_fused_path (the bench's kernel attribution) use it.
static bool fwd_fused_taken(const spwgnn_run* r, const spwgnn_batch* b) {
    const bool one_math = r->math == kmath(r, kX6EncEdge) && r->math == kmath(r, kX6EdgeFwd) &&
                          r->math == kmath(r, kX6NodeFwd);
    return one_math && fwd_fused_team(b->n_wtiles, b->nw_max, b->n_eblocks, b->n_nodes, r->math) &&
           !(b->flags & SPWGNN_BATCH_RECV_BLOCKS) && !store_b16_node(r, b) && !getenv_flag("SPWGNN_NO_FWD_FUSED");
}
static bool bwd_fused_taken(const spwgnn_run* r, const spwgnn_batch* b) {
    const bool one_math = r->math == kmath(r, kX6NodeBwd) && r->math == kmath(r, kX6EdgeBwd) &&
                          r->math == kmath(r, kX6EncEdgeBwd);
    return one_math && rebuild_dA(r, b) && fwd_fused_team(b->n_wtiles, b->nw_max, b->n_eblocks, b->n_nodes, r->math) &&
           !(b->flags & SPWGNN_BATCH_RECV_BLOCKS) && !store_b16_node(r, b) && !getenv_flag("SPWGNN_NO_BWD_FUSED");
}

static int32_t run_forward(const float* params, const spwgnn_batch* b, const spwgnn_run* r, const Ws& w,
                           char* base, float* logits, hipStream_t st) {
    Ctx c{w, base};
    PrepArgs pa{};
    pa.params = params;
    pa.pk = c.f(w.pk);
    build_packs(w, pa);
    // packs and, for the split-bf16 maths, the x6 images: one launch (one of the ≈ 20 of a small step)
    PrepX6Args xa{};
    if (r->math != MATH_F32) {
        xa.img = reinterpret_cast<uint4*>(c.f(w.x6));
        for (int id = 0; id < X6_PREP_COUNT; ++id) {
            const X6Spec& sp = kX6Specs[id];
            X6Desc& d = xa.d[id];
            d.pack = sp.pack;
            d.nt_out = sp.nt_out;
            d.nkb = x6_nkb(sp);
            d.kh = sp.kh;
            d.ht = sp.ht;
            d.dst = w.x6off[id];
            // an image reads pack elements (k < rows, col < cols) only
            if ((sp.kh ? 2 * sp.kh : 16 * sp.nkb) > pack_rows(sp.pack) || 32 * sp.nt_out > pack_cols(sp.pack))
                return SPWGNN_E_SHAPE;
        }
    }
    if (const spwgnn_prologue* p = r->prologue) {   // a replayed step's first work, in this launch
        if (p->copy_bytes < 0 || p->copy_bytes % 16 || (p->copy_bytes && (!p->copy_src || !p->copy_dst)) ||
            reinterpret_cast<uintptr_t>(p->copy_src) % 16 || reinterpret_cast<uintptr_t>(p->copy_dst) % 16 ||
            (p->key && (!p->step || p->mode < SPWGNN_STEP_KEY_COUNTER || p->mode > SPWGNN_STEP_KEY_SPLITMIX)))
            return SPWGNN_E_ARG;
        pa.pro.src = static_cast<const uint4*>(p->copy_src);
        pa.pro.dst = static_cast<uint4*>(p->copy_dst);
        pa.pro.n16 = p->copy_bytes / 16;
        pa.pro.key = p->key;
        pa.pro.step = p->step;
        pa.pro.mode = p->mode;
        pa.pro.rank = p->rank;
        pa.pro.seed = p->seed;
        pa.pro_row = 1;
    }
    SPW_CHECK(launch_prep(pa, r->math != MATH_F32 ? &xa : nullptr, st));
    const bool drop = r->training && r->dropout > 0.f;
    const uint32_t thresh = (uint32_t)std::min(4294967295.0, std::floor((double)r->dropout * 4294967296.0));
    const float scale = drop ? 1.0f / (1.0f - r->dropout) : 1.0f;
    const int uv16 = uv_storage(r, b);

    EncNodeArgs en{};
    en.n_nodes = b->n_nodes;
    en.pos = b->pos;
    en.prop = b->prop;
    en.node_tower = b->node_tower;
    en.node_local = b->node_local;
    en.w_om0 = c.pk(PK_OM0);
    en.b_om0 = c.pk(PB_OM0);
    en.w_om1 = c.pk(PK_OM1);
    en.b_om1 = c.pk(PB_OM1);
    en.w1b = c.pk(PK_W1B);
    en.w1c = c.pk(PK_W1C);
    if (r->math != MATH_F32) {
        en.x_om1 = c.x6(X6_OM1);
        en.xh_om1 = c.x6(X6_OM1_H);
        en.x_w1b = c.x6(X6_W1B);
        en.x_w1c = c.x6(X6_W1C);
    }
    en.zo1 = z1_rebuilt(r) ? nullptr : c.f(w.zo1);
    en.co = c.f(w.co);
    en.P0 = c.f(w.P_at(0));
    en.U0 = c.f(w.U_at(0));
    en.V0 = c.f(w.V_at(0));
    en.uv16 = uv16;
    en.dropout_on = drop;
    en.thresh = thresh;
    en.scale = scale;
    en.seed = r->seed;
    en.seed_dev = r->seed_dev;

    EncEdgeArgs ee{};
    ee.n_eblocks = b->n_eblocks;
    ee.pos = b->pos;
    ee.esrc = b->edge_src;
    ee.edst = b->edge_dst;
    ee.node_tower = b->node_tower;
    ee.node_local = b->node_local;
    ee.w_rm0 = c.pk(PK_RM0);
    ee.b_rm0 = c.pk(PB_RM0);
    ee.w_rm1 = c.pk(PK_RM1);
    ee.b_rm1 = c.pk(PB_RM1);
    ee.w_rm2 = c.pk(PK_RM2);
    ee.b_rm2 = c.pk(PB_RM2);
    ee.w_rm3 = c.pk(PK_RM3);
    ee.b_rm3 = c.pk(PB_RM3);
    ee.w_w1a = c.pk(PK_W1A);
    ee.b_w1a = c.pk(PB_W1A);
    if (r->math != MATH_F32) {
        ee.x_rm1 = c.x6(X6_RM1);
        ee.x_rm2 = c.x6(X6_RM2);
        ee.x_rm3 = c.x6(X6_RM3);
        ee.x_w1a = c.x6(X6_W1A);
    }
    ee.z1 = z1_rebuilt(r) ? nullptr : c.f(w.z1);
    ee.ed = z1_rebuilt(r) ? reinterpret_cast<float2*>(c.f(w.ed)) : nullptr;
    ee.z2 = c.f(w.z2);
    ee.z3 = c.f(w.z3);
    ee.cr = c.f(w.cr);
    ee.A = c.f(w.A);
    ee.zmask = r->training ? c.u(w.zmask) : nullptr;
    ee.b16 = store_b16(r, b);
    ee.dropout_on = drop;
    ee.thresh = thresh;
    ee.scale = scale;
    ee.seed = r->seed;
    ee.seed_dev = r->seed_dev;
    const int S = r->mp_steps;
    auto edge_args = [&](int s) {
        EdgeFwdArgs ef{};
        ef.n_wtiles = b->n_wtiles;
        ef.nw_max = b->nw_max;
        ef.wpg = 4;
        ef.wtile = b->wtile;
        ef.esrc = b->edge_src;
        ef.edst = b->edge_dst;
        ef.csr = reinterpret_cast<const uint32_t*>(b->blk_csr);
        ef.A = c.f(w.A);
        ef.U = c.f(w.U_at(s));
        ef.V = c.f(w.V_at(s));
        ef.w2 = c.pk(PK_W2);
        ef.b2 = c.pk(PB_W2);
        ef.x_w2 = r->math != MATH_F32 ? c.x6(X6_W2) : nullptr;
        ef.H2s = c.f(w.H2s_at(s));
        ef.mask1 = r->training ? c.u(w.m1_at(s)) : nullptr;
        ef.h1_out = nullptr;   // the W2 gradient recomputes h1 (XM_H1)
        ef.a_b16 = store_b16(r, b);
        ef.n16 = store_b16_node(r, b);
        ef.uv16 = uv16;
        ef.n_nodes = b->n_nodes;
        ef.recv_blocks = (b->flags & SPWGNN_BATCH_RECV_BLOCKS) && kmath(r, kX6EdgeFwd) == MATH_X6 &&
                         b->n_eblocks == b->n_nodes && !getenv_flag("SPWGNN_RB_ONEHOT");
        ef.mask2 = r->training ? c.u(w.m2_at(s)) : nullptr;
        return ef;
    };
    auto node_args = [&](int s) {
        NodeFwdArgs nf{};
        nf.n_nodes = b->n_nodes;
        nf.H2s = c.f(w.H2s_at(s));
        nf.P = c.f(w.P_at(s));
        nf.co = c.f(w.co);
        nf.cw_out = (s == 0) ? c.f(w.cw) : nullptr;
        nf.cw_in = (s > 0) ? c.f(w.cw) : nullptr;
        nf.a_out = r->training ? c.f(w.a_at(s)) : nullptr;
        nf.o1_out = r->training ? c.f(w.o1_at(s)) : nullptr;
        nf.Pn = c.f(w.P_at(s + 1));
        nf.logits = (s == S - 1) ? logits : nullptr;
        nf.U = (s + 1 < S) ? c.f(w.U_at(s + 1)) : nullptr;
        nf.V = (s + 1 < S) ? c.f(w.V_at(s + 1)) : nullptr;
        nf.w3a = c.pk(PK_W3A);
        nf.wo1c = c.pk(PK_WO1C);
        nf.wo1a = c.pk(PK_WO1A);
        nf.wo1p = c.pk(PK_WO1P);
        nf.wo2 = c.pk(PK_WO2);
        nf.w1b = c.pk(PK_W1B);
        nf.w1c = c.pk(PK_W1C);
        nf.bo1 = c.pk(PB_O1);
        nf.bo2p = c.pk(PB_O2P);
        if (r->math != MATH_F32) {
            nf.x_w3a = c.x6(X6_W3A);
            nf.x_wo1c = c.x6(X6_WO1C);
            nf.x_wo1a = c.x6(X6_WO1A);
            nf.x_wo1p = c.x6(X6_WO1P);
            nf.x_wo2 = c.x6(X6_WO2);
            nf.xh_w3a = c.x6(X6_W3A_H);
            nf.xh_wo1c = c.x6(X6_WO1C_H);
            nf.xh_wo1a = c.x6(X6_WO1A_H);
            nf.xh_wo1p = c.x6(X6_WO1P_H);
            nf.xh_wo2 = c.x6(X6_WO2_H);
            nf.x_w1b = c.x6(X6_W1B);
            nf.x_w1c = c.x6(X6_W1C);
        }
        nf.n16 = store_b16_node(r, b);
        nf.uv16 = uv16;
        return nf;
    };
    if (fwd_fused_taken(r, b)) {
        // small batch: the encoders and all S steps in one launch (timed as the relation encoder)
        FwdFusedArgs fa{};
        fa.ee = ee;
        fa.en = en;
        fa.ef = edge_args(0);
        fa.nf = node_args(0);
        fa.S = S;
        fa.training = r->training;
        fa.rowsN = w.RN * kRowN;
        fa.rowsE = w.RN * kRowE;
        fa.m1_step = r->training ? w.m1_at(1) - w.m1_at(0) : 0;
        fa.m2_step = r->training ? w.m2_at(1) - w.m2_at(0) : 0;
        fa.logits = logits;
        // the encoders side by side in their own launch (a workgroup per block / node block) beat
        // running them one after the other inside each tile's workgroup
        fa.encoders = getenv_flag("SPWGNN_FUSED_ENC");
        Prof p0{r, st};
        SPW_CHECK(p0.before(SPWGNN_K_ENC_EDGE));
        if (!fa.encoders) SPW_CHECK(launch_enc_pair_team(ee, en, r->math, ee.z1 || ee.ed, st));
        SPW_CHECK(p0.after(SPWGNN_K_ENC_EDGE));
        Prof p1{r, st};
        SPW_CHECK(p1.before(SPWGNN_K_EDGE_FWD));
        SPW_CHECK(launch_fwd_fused_team(fa, r->math, ee.z1 || ee.ed, st));
        SPW_CHECK(p1.after(SPWGNN_K_EDGE_FWD));
        return SPWGNN_OK;
    }
    if (r->math == kmath(r, kX6EncEdge) && enc_pair_team(b->n_eblocks, b->n_nodes, r->math) &&
        !getenv_flag("SPWGNN_NO_ENC_PAIR")) {
        // small batch: both encoders in one launch (timed as the relation encoder)
        Prof p0{r, st};
        SPW_CHECK(p0.before(SPWGNN_K_ENC_EDGE));
        SPW_CHECK(launch_enc_pair_team(ee, en, r->math, ee.z1 || ee.ed, st));
        SPW_CHECK(p0.after(SPWGNN_K_ENC_EDGE));
    } else {
        {
            Prof pn{r, st};
            SPW_CHECK(pn.before(SPWGNN_K_ENC_NODE));
            SPW_CHECK(launch_enc_node(en, r->math, st));
            SPW_CHECK(pn.after(SPWGNN_K_ENC_NODE));
        }
        Prof p0{r, st};
        SPW_CHECK(p0.before(SPWGNN_K_ENC_EDGE));
        SPW_CHECK(launch_enc_edge(ee, kmath(r, kX6EncEdge), st));
        SPW_CHECK(p0.after(SPWGNN_K_ENC_EDGE));
    }

    Prof prof{r, st};
    for (int s = 0; s < S; ++s) {
        const EdgeFwdArgs ef = edge_args(s);
        SPW_CHECK(prof.before(SPWGNN_K_EDGE_FWD));
        SPW_CHECK(launch_edge_fwd(ef, kmath(r, kX6EdgeFwd), st));
        SPW_CHECK(prof.after(SPWGNN_K_EDGE_FWD));
        const NodeFwdArgs nf = node_args(s);
        SPW_CHECK(prof.before(SPWGNN_K_NODE_FWD));
        SPW_CHECK(launch_node_fwd(nf, kmath(r, kX6NodeFwd), st));
        SPW_CHECK(prof.after(SPWGNN_K_NODE_FWD));
    }
    return SPWGNN_OK;
}

struct WgSpec {
    int xmode = XM_ROW, ymode = YM_ROW;
    const float* x = nullptr;
    int x_ld = 0, x_width = 0, x_ones = -1;
    int64_t x_count = 1, x_stride = 0;
    const float* y = nullptr;
    int y_ld = 0, y_width = 0;
    int64_t y_count = 1, y_stride = 0;
    int64_t rows = 0;
    int kx_pad = 0, ny_pad = 0;
    // reduce target
    int tk = -1, tb = -1, k_rows = 0, k_row0 = 0, bias_row = -1, perm = 0;
    bool recompute = false;   // XM_H1 / YM_DH2 context below
    int b16 = 0;              // kB16X / kB16Y: bf16-stored operands (bf16 math, store_b16)
    const float2* xd = nullptr;          // z1 rebuilt from d (k_wgrad_ws XD 1)
    const float4* xp = nullptr;          // zo1 rebuilt from the node positions (XD 2)
    const float *w0 = nullptr, *b0 = nullptr;
};

// Each weight gradient writes its per-chunk slabs into its own slot; the ordered chunk sums of all
// of them run as one batched launch at the end of the backward (launch_wgrad_reduce_all).
static int32_t run_wgrad(const Ctx& c, const spwgnn_batch* b, const WgSpec& g, float* grads, int math, hipStream_t st,
                         ReduceBatch& rb, const Prof* prof = nullptr, WsBatch* wsb = nullptr,
                         Pos3Batch* p3 = nullptr) {
    const Ws& w = c.w;
    if (g.rows <= 0) return SPWGNN_OK;
    if (rb.n >= kWgSlots) return SPWGNN_E_ARG;
    float* const slab = c.f(w.slab) + (int64_t)rb.n * w.slot_floats;
    // the row-chunked kernels: chunks of ≥ 512 rows, but at least one per CU (256) while a chunk
    // keeps ≥ one 32-row block — small batches spread over the chip instead of walking a few
    // chunks serially; at most 1024 chunks and what the slot holds
    const int64_t slot_chunks = w.slot_floats / ((int64_t)g.kx_pad * g.ny_pad);
    int64_t chunks = std::max<int64_t>((g.rows + 32 * 16 - 1) / (32 * 16), std::min<int64_t>((g.rows + 31) / 32, 256));
    chunks = std::max<int64_t>(1, std::min<int64_t>(chunks, std::min<int64_t>(1024, slot_chunks)));
    int64_t rpc = up((g.rows + chunks - 1) / chunks, 32);
    chunks = (g.rows + rpc - 1) / rpc;
    WgradArgs a{};
    a.rows = g.rows;
    a.rows_per_chunk = rpc;
    a.xmode = g.xmode;
    a.ymode = g.ymode;
    a.kx_pad = g.kx_pad;
    a.ny_pad = g.ny_pad;
    a.x_ptr = g.x;
    a.x_ld = g.x_ld;
    a.x_width = g.x_width;
    a.x_ones = g.x_ones;
    a.x_count = g.x_count;
    a.x_stride = g.x_stride;
    a.y_ptr = g.y;
    a.y_ld = g.y_ld;
    a.y_width = g.y_width;
    a.y_count = g.y_count;
    a.y_stride = g.y_stride;
    a.pos = b->pos;
    a.esrc = b->edge_src;
    a.edst = b->edge_dst;
    a.slab = slab;
    if (g.recompute) {
        a.A = c.f(w.A);
        a.U = c.f(w.U);
        a.V = c.f(w.V);
        a.G3 = c.f(w.G3);
        a.mask2 = c.u(w.mask2);
        a.RE = w.RE;
        a.RN = w.RN;
        a.S = (int)(g.rows / w.RE);
        a.a_b16 = (g.b16 & kB16A) != 0;
        a.uv16 = (g.b16 & kB16UV) != 0;
        a.wtile = b->wtile;
        a.n_wtiles = b->n_wtiles;
        a.nw_max = b->nw_max;
        a.w2_tile = !getenv_flag("SPWGNN_W2G_GATHER");   // A/B switch: the per-edge gather kernel
    }
    // stored chunk-major operands in x6 math: the warp-specialized kernel, one workgroup per CU
    if (math != MATH_F32 && g.xmode == XM_CM && (g.ymode == YM_CM || g.ymode == YM_ROW) &&
        !getenv_flag("SPWGNN_WG_OLD")) {
        WgWsArgs wa{};
        wa.x = g.x;
        wa.y = g.y;
        wa.slab = slab;
        wa.count = g.x_count;
        wa.S = g.rows / g.x_count;
        wa.nbs = (g.x_count + 31) / 32;
        wa.x_sb = g.x_stride / 32;
        wa.y_sb = g.y_stride / 32;
        wa.x_ones = g.x_ones;
        wa.xd = g.xd;
        wa.xp = g.xp;
        wa.w0 = g.w0;
        wa.b0 = g.b0;
        const int64_t nst = wa.nbs * wa.S;
        int64_t wgs = std::min<int64_t>(nst, kW2gWgs);
        if (wsb) {
            wgs = std::min<int64_t>(wgs, std::max<int64_t>(kWsMinWgs, (nst + kWsMinStages - 1) / kWsMinStages));
            wgs = std::min<int64_t>(wgs, (nst + kWsSmallStages - 1) / kWsSmallStages);
        }
        wa.stages_per_wg = (nst + wgs - 1) / wgs;
        wgs = (nst + wa.stages_per_wg - 1) / wa.stages_per_wg;
        chunks = wgs;
        const bool mask = !(g.kx_pad == 160 && g.ny_pad == 160);   // node arrays: rows ≥ count masked
        if (wsb) {   // queued: every k_wgrad_ws gradient of the backward runs in one launch
            const int v = wgrad_ws_variant(wa, g.kx_pad, g.ny_pad, g.ymode == YM_ROW, mask, math, g.b16);
            if (v == WSV_NONE || wsb->n >= kMaxWsJobs) return SPWGNN_E_ARG;
            WsJob& j = wsb->j[wsb->n++];
            j.a = wa;
            j.variant = v;
            j.wg0 = wsb->wgs;
            j.gn = j.gi = 0;
            wsb->wgs += (int)wgs;
        } else {
            if (prof) SPW_CHECK(prof->before(SPWGNN_K_WGRAD_WS));
            SPW_CHECK(launch_wgrad_ws(wa, (int)wgs, g.kx_pad, g.ny_pad, g.ymode == YM_ROW, mask, math, st, g.b16));
            if (prof) SPW_CHECK(prof->after(SPWGNN_K_WGRAD_WS));
        }
    } else if (math != MATH_F32 && (g.xmode == XM_NODE_O || (g.xmode == XM_EDGE_D && g.xd))) {
        // the 3-column first-layer gradients: a vector-ALU stream over Y (k_wgrad_pos3)
        const bool node = g.xmode == XM_NODE_O;
        Pos3Args pa{};
        pa.y = g.y;
        pa.pos = reinterpret_cast<const float4*>(b->pos);
        pa.ed = g.xd;
        pa.esrc = b->edge_src;
        pa.slab = slab;
        pa.count = g.rows;
        pa.nblk = (g.rows + 31) / 32;
        const int64_t wgs = std::max<int64_t>(1, std::min<int64_t>(pa.nblk, std::min<int64_t>(512, slot_chunks)));
        pa.blk_per_wg = (pa.nblk + wgs - 1) / wgs;
        chunks = (pa.nblk + pa.blk_per_wg - 1) / pa.blk_per_wg;
        if (!p3) return SPWGNN_E_ARG;
        if (node) { p3->n = pa; p3->cn = (int)chunks; }
        else { p3->e = pa; p3->ce = (int)chunks; p3->b16e = (g.b16 & kB16Y) != 0; }
    } else {
    // the x6 W2 gradient: one warp-specialized workgroup per CU over contiguous edge-block ranges
    const bool ws = g.recompute && math != MATH_F32 && (math == MATH_BF16 || !getenv_flag("SPWGNN_W2G_OLD"));
    int64_t bpw = 0;
    if (ws) {
        const int64_t nblk = w.RE / 32;
        const int64_t wgs = std::min<int64_t>(nblk, kW2gWgs);
        bpw = (nblk + wgs - 1) / wgs;
        chunks = (nblk + bpw - 1) / bpw;
    }
    // a small x6 batch: the W2 gradient runs inside the batched weight-gradient launch
    const bool w2_in_batch = ws && math == MATH_X6 && wsb && team_blocks(b->n_eblocks) && !getenv_flag("SPWGNN_NO_W2_MERGE");
    if (prof && g.recompute && !w2_in_batch) SPW_CHECK(prof->before(SPWGNN_K_WGRAD_W2));
    if (w2_in_batch) {
        wsb->w2 = a;
        wsb->w2_bpw = bpw;
        wsb->w2_wgs = (int)chunks;
    } else if (ws)
        SPW_CHECK(launch_w2grad_ws(a, (int)chunks, bpw, math, st));
    else if (math == MATH_BF16)
        SPW_CHECK(launch_wgrad_bf16(a, (int)chunks, st, g.b16));
    else if (g.b16)
        return SPWGNN_E_ARG;
    else
        SPW_CHECK(launch_wgrad(a, (int)chunks, math, st));
    if (prof && g.recompute && !w2_in_batch) SPW_CHECK(prof->after(SPWGNN_K_WGRAD_W2));
    }
    const ParamTable& pt = param_table();
    ReduceArgs& ra = rb.r[rb.n++];
    ra = ReduceArgs{};
    ra.slab = slab;
    ra.chunks = (int)chunks;
    ra.kx_pad = g.kx_pad;
    ra.ny_pad = g.ny_pad;
    ra.out = grads;
    ra.kernel_off = g.tk >= 0 ? pt.t[g.tk].offset : -1;
    ra.kernel_rows = g.k_rows;
    ra.kernel_cols = g.tk >= 0 ? pt.t[g.tk].cols : pt.t[g.tb].cols;
    ra.kernel_row0 = g.k_row0;
    ra.bias_off = g.tb >= 0 ? pt.t[g.tb].offset : -1;
    ra.bias_row = g.bias_row;
    ra.perm = g.perm;
    return SPWGNN_OK;
}

// Jobs [first, first + n) of the batch read one operand in common (the node rows P / do1): run them
// as an interleaved group (k_wgrad_ws_batch) when their row ranges match — the same workgroup count,
// a multiple of the 8 XCDs, over the same stage partition; otherwise they stay in sequence.
static void ws_group(WsBatch* wsb, int first, int n) {
    if (!wsb || n < 2 || first < 0 || first + n > wsb->n || getenv_flag("SPWGNN_WS_NOGROUP")) return;
    const WsJob& j0 = wsb->j[first];
    const int w0 = (first + 1 < wsb->n ? wsb->j[first + 1].wg0 : wsb->wgs) - j0.wg0;
    if (w0 <= 0 || w0 % 8) return;
    for (int i = 1; i < n; ++i) {
        const WsJob& ji = wsb->j[first + i];
        const int wi = (first + i + 1 < wsb->n ? wsb->j[first + i + 1].wg0 : wsb->wgs) - ji.wg0;
        if (wi != w0 || ji.a.stages_per_wg != j0.a.stages_per_wg || ji.a.nbs != j0.a.nbs || ji.a.S != j0.a.S) return;
    }
    for (int i = 0; i < n; ++i) {
        wsb->j[first + i].gn = n;
        wsb->j[first + i].gi = i;
    }
}

int32_t run_backward(const float* params, const spwgnn_batch* b, const spwgnn_run* r, const Ws& w, char* base,
                     const float* dlogits, float* grads, float* dprop, hipStream_t st, const BceArgs* bce = nullptr) {
    (void)params;  // the packed copies made by the forward on this workspace are used
    Ctx c{w, base};
    const int S = r->mp_steps;
    const bool rebuild = rebuild_dA(r, b);
    const bool b16 = store_b16(r, b);
    const bool n16 = store_b16_node(r, b);
    const int64_t nN = b->n_nodes;
    const float scale = (r->dropout > 0.f) ? 1.0f / (1.0f - r->dropout) : 1.0f;
    // the reductions write the 22 Keras tensors' elements, not every float of the flat buffer: the
    // remaining ranges (alignment gaps; tensors no job of this batch writes) are zeroed by the same
    // reduction launch (tests/test_gpu_parity.py::test_backward_writes_every_gradient; a NaN-filled
    // buffer comes out equal to a zero-filled one)
    Prof prof{r, st};

    auto node_args = [&](int s) {
        const bool first = (s == S - 1);
        NodeBwdArgs nb{};
        nb.n_nodes = b->n_nodes;
        nb.first = first;
        nb.tail = 0;
        nb.dPin = first ? nullptr : c.f(w.dP_at(s + 1));
        nb.dU = first ? nullptr : c.f(w.dU_at(s + 1));
        nb.dV = first ? nullptr : c.f(w.dV_at(s + 1));
        nb.Pn = c.f(w.P_at(s + 1));
        nb.o1 = c.f(w.o1_at(s));
        nb.a = c.f(w.a_at(s));
        nb.dlogits = dlogits;
        nb.dx = c.f(w.dx_at(s));
        nb.do1 = c.f(w.do1_at(s));
        nb.g = c.f(w.g_at(s));
        nb.G3 = c.f(w.G3_at(s));
        nb.dPout = c.f(w.dP_at(s));
        nb.dco = c.f(w.dco);
        nb.dco_accumulate = !first;
        nb.dco_sum = kmath(r, kX6NodeBwd) != MATH_F32;
        nb.w1bt = c.pk(PK_W1BT);
        nb.w1ct = c.pk(PK_W1CT);
        nb.wo2t = c.pk(PK_WO2T);
        nb.wo1ct = c.pk(PK_WO1CT);
        nb.wo1at = c.pk(PK_WO1AT);
        nb.wo1pt = c.pk(PK_WO1PT);
        nb.w3t = c.pk(PK_W3T);
        if (r->math != MATH_F32) {
            nb.x_w1bt = c.x6(X6_W1BT);
            nb.x_w1ct = c.x6(X6_W1CT);
            nb.x_wo2t = c.x6(X6_WO2T);
            nb.x_wo1ct = c.x6(X6_WO1CT);
            nb.x_wo1at = c.x6(X6_WO1AT);
            nb.x_wo1pt = c.x6(X6_WO1PT);
            nb.xh_w1bt = c.x6(X6_W1BT_H);
            nb.xh_w1ct = c.x6(X6_W1CT_H);
            nb.xh_wo2t = c.x6(X6_WO2T_H);
            nb.xh_wo1ct = c.x6(X6_WO1CT_H);
            nb.xh_wo1at = c.x6(X6_WO1AT_H);
            nb.xh_wo1pt = c.x6(X6_WO1PT_H);
            nb.x_w3t = c.x6(X6_W3T);
        }
        nb.n16 = n16;
        return nb;
    };
    auto edge_args = [&](int s) {
        EdgeBwdArgs eb{};
        eb.n_wtiles = b->n_wtiles;
        eb.nw_max = b->nw_max;
        eb.wpg = b->nw_max <= 16 ? 4 : edge_wpg(edge_bwd_lds_per_wave(b->nw_max));
        eb.dA_accumulate = s != S - 1;
        eb.no_dA = rebuild;
        eb.wtile = b->wtile;
        eb.esrc = b->edge_src;
        eb.edst = b->edge_dst;
        eb.csr = reinterpret_cast<const uint32_t*>(b->blk_csr);
        eb.mask1 = c.u(w.m1_at(s));
        eb.mask2 = c.u(w.m2_at(s));
        eb.dh2_out = nullptr;  // the W2 gradient recomputes dh2pre (YM_DH2)
        eb.G3 = c.f(w.G3_at(s));
        eb.w2t = c.pk(PK_W2T);
        eb.x_w2t = r->math != MATH_F32 ? c.x6(X6_W2T) : nullptr;
        eb.dA = c.f(w.dA);
        eb.dU = c.f(w.dU_at(s));
        eb.dV = c.f(w.dV_at(s));
        eb.n16 = n16;
        return eb;
    };
    NodeBwdArgs tl{};
    if (dprop) {
        tl.n_nodes = b->n_nodes;
        tl.first = 0;
        tl.tail = 1;
        tl.dPin = c.f(w.dP_at(0));
        tl.dU = c.f(w.dU_at(0));
        tl.dV = c.f(w.dV_at(0));
        tl.dprop = dprop;
        tl.w1bt = c.pk(PK_W1BT);
        tl.w1ct = c.pk(PK_W1CT);
        if (r->math != MATH_F32) {
            tl.x_w1bt = c.x6(X6_W1BT);
            tl.x_w1ct = c.x6(X6_W1CT);
            tl.xh_w1bt = c.x6(X6_W1BT_H);
            tl.xh_w1ct = c.x6(X6_W1CT_H);
        }
        tl.n16 = n16;
    }
    DaArgs da{};
    if (rebuild) {
        da.n_eblocks = b->n_eblocks;
        da.S = S;
        da.g3_step = w.G3_at(1) - w.G3_at(0);
        da.m1_step = w.m1_at(1) - w.m1_at(0);
        da.m2_step = w.m2_at(1) - w.m2_at(0);
        da.edst = b->edge_dst;
        da.mask1 = c.u(w.mask1);
        da.mask2 = c.u(w.mask2);
        da.G3 = c.f(w.G3);
        da.dA = c.f(w.dA);
        da.x_w2t = c.x6(X6_W2T);
        da.b16 = b16;
    }
    EncEdgeBwdArgs eeb{};
    eeb.n_eblocks = b->n_eblocks;
    eeb.b16 = b16;
    eeb.dA = c.f(w.dA);
    eeb.zmask = c.u(w.zmask);
    eeb.w1at = c.pk(PK_W1AT);
    eeb.rm3t = c.pk(PK_RM3T);
    eeb.rm2t = c.pk(PK_RM2T);
    eeb.rm1t = c.pk(PK_RM1T);
    if (r->math != MATH_F32) {
        eeb.x_w1at = c.x6(X6_W1AT);
        eeb.x_rm3t = c.x6(X6_RM3T);
        eeb.x_rm2t = c.x6(X6_RM2T);
        eeb.x_rm1t = c.x6(X6_RM1T);
    }
    eeb.dz4 = c.f(w.dz4);
    eeb.dz3 = c.f(w.dz3);
    eeb.dz2 = c.f(w.dz2);
    eeb.dz1 = c.f(w.dz1);
    eeb.scale = scale;
    EncNodeBwdArgs enb{};
    enb.n_nodes = b->n_nodes;
    enb.dco = c.f(w.dco);
    enb.co = c.f(w.co);
    enb.zo1 = z1_rebuilt(r) ? nullptr : c.f(w.zo1);
    enb.pos = b->pos;
    enb.w_om0 = c.pk(PK_OM0);
    enb.b_om0 = c.pk(PB_OM0);
    enb.om1t = c.pk(PK_OM1T);
    enb.wo1ct = kmath(r, kX6NodeBwd) != MATH_F32 ? c.pk(PK_WO1CT) : nullptr;
    enb.do1 = c.f(w.do1_at(0));
    enb.do1_step = w.do1_at(1) - w.do1_at(0);
    enb.S = S;
    enb.dzo2 = c.f(w.dzo2);
    enb.dzo1 = c.f(w.dzo1);
    enb.scale = scale;
    if (kmath(r, kX6NodeBwd) != MATH_F32) {
        enb.x_wo1ct = c.x6(X6_WO1CT);
        enb.x_om1t = c.x6(X6_OM1T);
        enb.xh_wo1ct = c.x6(X6_WO1CT_H);
        enb.xh_om1t = c.x6(X6_OM1T_H);
    }

    // two weight-gradient groups (spwgnn_run.grads_early_event): the node-side and W2/W3 gradients
    // first, the event, then dA, the relation encoder's backward and the encoder-side gradients
    const bool split = r->grads_early_event != nullptr;
    int32_t e = SPWGNN_OK;
    const bool fused = bwd_fused_taken(r, b);
    // spwgnn_bce_backward: on the fused loop (one loss workgroup) the loop computes dlogits itself and
    // the loss sums ride in the last reduction launch; anywhere else the loss launch runs first
    const bool bce_inline = bce && fused && bce->blocks == 1;
    if (bce && !bce_inline) SPW_CHECK(launch_bce(*bce, st));
    auto edge_encoder_bwd = [&]() -> int32_t {   // dA rebuild + relation encoder backward (wide kernels)
        if (rebuild) {
            SPW_CHECK(prof.before(SPWGNN_K_DA));
            SPW_CHECK(launch_dA(da, kmath(r, kX6EdgeBwd), st));
            SPW_CHECK(prof.after(SPWGNN_K_DA));
        }
        SPW_CHECK(prof.before(SPWGNN_K_ENC_EDGE_BWD));
        SPW_CHECK(launch_enc_edge_bwd(eeb, kmath(r, kX6EncEdgeBwd), st));
        SPW_CHECK(prof.after(SPWGNN_K_ENC_EDGE_BWD));
        return SPWGNN_OK;
    };
    if (fused) {
        // small batch: the step loop, dA and both encoder backwards in one launch (timed as the node backward)
        BwdFusedArgs fa{};
        fa.nb = node_args(0);
        fa.nb.dU = c.f(w.dU_at(1));   // step 0's incoming dU/dV (BwdFusedArgs)
        fa.nb.dV = c.f(w.dV_at(1));
        if (bce_inline) {
            fa.nb.bce_logits = bce->logits;
            fa.nb.bce_targets = bce->targets;
            fa.nb.bce_dlogits = bce->dlogits;
            fa.nb.bce_n = bce->n;
        }
        fa.tail = tl;
        fa.has_tail = dprop != nullptr;
        fa.eb = edge_args(0);
        fa.da = da;
        fa.eeb = eeb;
        fa.enb = enb;
        fa.S = S;
        fa.rowsN = w.RN * kRowN;
        fa.rowsE = w.RN * kRowE;
        fa.m1_step = w.m1_at(1) - w.m1_at(0);
        fa.m2_step = w.m2_at(1) - w.m2_at(0);
        fa.encoders = getenv_flag("SPWGNN_FUSED_ENC");
        fa.dA_in_loop = !getenv_flag("SPWGNN_DA_PAIR");
        SPW_CHECK(prof.before(SPWGNN_K_NODE_BWD));
        SPW_CHECK(launch_bwd_fused_team(fa, r->math, st));
        SPW_CHECK(prof.after(SPWGNN_K_NODE_BWD));
        if (!fa.encoders) {
            SPW_CHECK(prof.before(SPWGNN_K_ENC_EDGE_BWD));
            SPW_CHECK(launch_bwd_enc_pair_team(da, eeb, enb, r->math, !fa.dA_in_loop, st));
            SPW_CHECK(prof.after(SPWGNN_K_ENC_EDGE_BWD));
        }
    } else {
        for (int s = S - 1; s >= 0; --s) {
            const NodeBwdArgs nb = node_args(s);
            SPW_CHECK(prof.before(SPWGNN_K_NODE_BWD));
            SPW_CHECK(launch_node_bwd(nb, kmath(r, kX6NodeBwd), st));
            SPW_CHECK(prof.after(SPWGNN_K_NODE_BWD));
            const EdgeBwdArgs eb = edge_args(s);
            SPW_CHECK(prof.before(SPWGNN_K_EDGE_BWD));
            SPW_CHECK(launch_edge_bwd(eb, kmath(r, kX6EdgeBwd), st));
            SPW_CHECK(prof.after(SPWGNN_K_EDGE_BWD));
        }
        if (dprop) SPW_CHECK(launch_node_bwd(tl, kmath(r, kX6NodeBwd), st));
        if (!split && (e = edge_encoder_bwd())) return e;
        SPW_CHECK(prof.before(SPWGNN_K_ENC_NODE_BWD));
        SPW_CHECK(launch_enc_node_bwd(enb, kmath(r, kX6NodeBwd), st));
        SPW_CHECK(prof.after(SPWGNN_K_ENC_NODE_BWD));
    }

    // ---- weight gradients ----
    const int64_t RE = w.RE, RN = w.RN;
    auto edge_row = [&](WgSpec& g, int64_t xoff, int64_t yoff, int tk, int tb) {
        g.x = c.f(xoff); g.x_ld = kLdE; g.x_width = kFE; g.x_ones = kFE; g.x_count = RE; g.x_stride = 0;
        g.y = c.f(yoff); g.y_ld = kLdE; g.y_width = kFE; g.y_count = RE; g.y_stride = 0;
        g.rows = RE; g.kx_pad = 160; g.ny_pad = 160;
        g.tk = tk; g.tb = tb; g.k_rows = kFE; g.k_row0 = 0; g.bias_row = kFE;
    };
    ReduceBatch rb{};   // every gradient's reduction (its slab slot = its index here)
    WsBatch wsb{}, wsb2{};   // the batched launch (split: the early group's, then the late group's)
    const bool unbatched = getenv_flag("SPWGNN_WS_UNBATCHED");   // A/B: one launch per gradient
    WsBatch* wsp = unbatched ? nullptr : &wsb;
    Pos3Batch p3{};
    auto wg = [&](const WgSpec& g) { return run_wgrad(c, b, g, grads, kmath(r, kX6Wgrad), st, rb, &prof, wsp, &p3); };
    auto g_rm0 = [&]() {   // rm.0: X = [d | 1]
        WgSpec g; g.xmode = XM_EDGE_D; g.ymode = YM_CM; g.kx_pad = 32; g.ny_pad = 160; g.rows = RE;
        g.y = c.f(w.dz1); g.y_ld = kLdE; g.y_width = kFE; g.y_count = RE;
        g.tk = T_RM0K; g.tb = T_RM0B; g.k_rows = 2; g.bias_row = 2;
        g.b16 = b16 ? kB16Y : 0;   // Y = dz1
        if (z1_rebuilt(r)) g.xd = reinterpret_cast<const float2*>(c.f(w.ed));   // k_wgrad_pos3 reads d
        return wg(g);
    };
    // encoder layers: chunk-major activations and gradients; W1a: X = c_r (chunk-major), Y = dA (rows)
    auto cm_xy = [&](WgSpec& g) { g.xmode = XM_CM; g.ymode = YM_CM; };
    const int b16xy = b16 ? (kB16X | kB16Y) : 0;
    auto g_rm123_w1a = [&]() -> int32_t {
        {
            WgSpec g; edge_row(g, w.z1, w.dz2, T_RM1K, T_RM1B); cm_xy(g);
            if (z1_rebuilt(r)) {
                g.xd = reinterpret_cast<const float2*>(c.f(w.ed));
                g.w0 = c.pk(PK_RM0);
                g.b0 = c.pk(PB_RM0);
            }
            g.b16 = b16 ? kB16Y : 0;   // X rebuilt from d; Y = dz2
            if ((e = wg(g))) return e;
        }
        { WgSpec g; edge_row(g, w.z2, w.dz3, T_RM2K, T_RM2B); cm_xy(g); g.b16 = b16xy; if ((e = wg(g))) return e; }
        { WgSpec g; edge_row(g, w.z3, w.dz4, T_RM3K, T_RM3B); cm_xy(g); g.b16 = b16xy; if ((e = wg(g))) return e; }
        { WgSpec g; edge_row(g, w.cr, w.dA, T_RMP0K, T_RMP0B); g.xmode = XM_CM; g.b16 = b16xy; if ((e = wg(g))) return e; }
        return SPWGNN_OK;
    };
    auto g_w2 = [&]() {   // rmp.1 (W2, b2): X = [h1 | 1], Y = dh2pre, both recomputed from the chunk-major
        // A and node rows (U, V, G3) and the h2>0 mask, over all steps (row = s·RE + e)
        WgSpec g; edge_row(g, -1, -1, T_RMP1K, T_RMP1B);
        g.xmode = XM_H1; g.ymode = YM_DH2;
        g.x_count = g.y_count = g.rows = RE * S;
        g.recompute = true;
        g.b16 = (b16 ? kB16A : 0) | (n16 ? kB16UV : 0);   // U, V rows as the forward stored them (uv_storage)
        return wg(g);
    };
    auto node_xy = [&](WgSpec& g, int64_t xoff, int xld, int xw, int xones, int64_t xstride, int64_t yoff, int yld,
                       int yw, int kxp, int nyp) {
        g.x = c.f(xoff); g.x_ld = xld; g.x_width = xw; g.x_ones = xones; g.x_count = nN; g.x_stride = xstride;
        g.y = c.f(yoff); g.y_ld = yld; g.y_width = yw; g.y_count = nN; g.y_stride = RN;
        g.rows = nN * S; g.kx_pad = kxp; g.ny_pad = nyp;
        g.xmode = XM_CM; g.ymode = YM_CM;   // chunk-major node rows
    };
    auto g_node = [&]() -> int32_t {
        const int grp0 = wsp ? wsp->n : 0;   // W1b, W1c, omp.0 P part (X = P), omp.0 effect part (Y = do1): one group
        {   // rmp.0 rows 150..249 (W1b): Σ_s P_sᵀ dU_s
            WgSpec g; node_xy(g, w.P, kLdN, kFN, -1, RN, w.dU, kLdE, kFE, 128, 160);
            g.tk = T_RMP0K; g.k_rows = kFN; g.k_row0 = 150;
            g.b16 = n16 ? kB16Y : 0;
            if ((e = wg(g))) return e;
        }
        {   // rmp.0 rows 250..349 (W1c)
            WgSpec g; node_xy(g, w.P, kLdN, kFN, -1, RN, w.dV, kLdE, kFE, 128, 160);
            g.tk = T_RMP0K; g.k_rows = kFN; g.k_row0 = 250;
            g.b16 = n16 ? kB16Y : 0;
            if ((e = wg(g))) return e;
        }
        {   // omp.0 rows 200..299 (P part)
            WgSpec g; node_xy(g, w.P, kLdN, kFN, -1, RN, w.do1, kLdN, kFN, 128, 128);
            g.tk = T_OMP0K; g.k_rows = kFN; g.k_row0 = 200;
            if ((e = wg(g))) return e;
        }
        {   // omp.0 rows 100..199 (effect part)
            WgSpec g; node_xy(g, w.a, kLdN, kFN, -1, RN, w.do1, kLdN, kFN, 128, 128);
            g.tk = T_OMP0K; g.k_rows = kFN; g.k_row0 = 100;
            if ((e = wg(g))) return e;
        }
        if (wsp) ws_group(wsp, grp0, wsp->n - grp0);
        {   // rmp.2 (W3, b3): X = [H2s | deg]
            WgSpec g; node_xy(g, w.H2s, kLdE, kFE + 1, -1, RN, w.g, kLdN, kFN, 160, 128);
            g.tk = T_RMP2K; g.tb = T_RMP2B; g.k_rows = kFE; g.bias_row = kDegCol;
            g.b16 = n16 ? (kB16X | kB16Y) : 0;
            if ((e = wg(g))) return e;
        }
        {   // omp.0 rows 0..99 (c_o part, broadcast over steps) + bias
            WgSpec g; node_xy(g, w.co, kLdN, kFN, kFN, 0, w.do1, kLdN, kFN, 128, 128);
            g.tk = T_OMP0K; g.tb = T_OMP0B; g.k_rows = kFN; g.k_row0 = 0; g.bias_row = kFN;
            if (kmath(r, kX6NodeBwd) != MATH_F32) {   // c_oᵀ·Σ_s do1_s: Σ do1 stored by k_enc_node_bwd
                g.y = c.f(w.dco);
                g.rows = nN;
                g.y_stride = 0;
            }
            if ((e = wg(g))) return e;
        }
        {   // omp.1 (Wo2, bo2), x' column order → Keras order
            WgSpec g; node_xy(g, w.o1, kLdN, kFN, kFN, RN, w.dx, kLdN, kFN + 1, 128, 128);
            g.tk = T_OMP1K; g.tb = T_OMP1B; g.k_rows = kFN; g.bias_row = kFN; g.perm = 1;
            g.b16 = n16 ? (kB16X | kB16Y) : 0;
            if ((e = wg(g))) return e;
        }
        return SPWGNN_OK;
    };
    auto g_om0 = [&]() {   // om.0: X = [y, w | 1]
        WgSpec g; g.xmode = XM_NODE_O; g.ymode = YM_CM; g.kx_pad = 32; g.ny_pad = 128; g.rows = nN;
        g.y = c.f(w.dzo1); g.y_ld = kLdN; g.y_width = kFN; g.y_count = nN;
        g.tk = T_OM0K; g.tb = T_OM0B; g.k_rows = 2; g.bias_row = 2;
        return wg(g);
    };
    auto g_om1 = [&]() {   // om.1
        WgSpec g; node_xy(g, w.zo1, kLdN, kFN, kFN, 0, w.dzo2, kLdN, kFN, 128, 128);
        g.rows = nN; g.y_stride = 0;
        if (z1_rebuilt(r)) {
            g.xp = reinterpret_cast<const float4*>(b->pos);
            g.w0 = c.pk(PK_OM0);
            g.b0 = c.pk(PB_OM0);
        }
        g.tk = T_OM1K; g.tb = T_OM1B; g.k_rows = kFN; g.bias_row = kFN;
        return wg(g);
    };
    // the batched launch of `batch` (+ a small batch's rm.0 / om.0 gradients as trailing workgroups)
    auto launch_ws = [&](WsBatch& batch, bool with_p3) -> int32_t {
        const bool p3_in_batch = with_p3 && (batch.n > 0 || batch.w2_wgs > 0) && team_blocks(b->n_eblocks) &&
                                 !getenv_flag("SPWGNN_NO_POS3_MERGE");
        if (with_p3 && !p3_in_batch) SPW_CHECK(launch_wgrad_pos3(p3, st));
        if (batch.n > 0 || batch.w2_wgs > 0) {
            SPW_CHECK(prof.before(SPWGNN_K_WGRAD_WS));
            SPW_CHECK(launch_wgrad_ws_batch(batch, kmath(r, kX6Wgrad), st, p3_in_batch ? &p3 : nullptr));
            SPW_CHECK(prof.after(SPWGNN_K_WGRAD_WS));
        }
        return SPWGNN_OK;
    };
    // the reductions of the gradients whose tensors lie in [t_lo, t_hi), and the zeroing of the float
    // ranges of those tensors no such reduction writes (alignment gaps, uncovered tensor rows). More
    // ranges than the launch carries (kMaxZero) or no reduction: one memset of those tensors instead
    // (stream-ordered before the reduction, which then writes its ranges)
    auto reduce = [&](int t_lo, int t_hi, bool last) -> int32_t {
        const ParamTable& pt = param_table();
        const int64_t lo = pt.t[t_lo].offset, hi = t_hi < kNumTensors ? pt.t[t_hi].offset : pt.total;
        ReduceBatch sub{};
        if (last && bce_inline) {   // the loss sums: one more row of this launch
            sub.bce_row = 1;
            sub.bce = *bce;
            sub.bce.dlogits = nullptr;   // written by the step loop
        }
        for (int k = 0; k < rb.n; ++k) {
            const int64_t off = rb.r[k].kernel_off >= 0 ? rb.r[k].kernel_off : rb.r[k].bias_off;
            if (off >= lo && off < hi) sub.r[sub.n++] = rb.r[k];
        }
        sub.nzero = 0;
        bool overflow = false;
        auto zero = [&](int64_t off, int64_t len) {
            if (len <= 0) return;
            if (sub.nzero > 0 && sub.zoff[sub.nzero - 1] + sub.zlen[sub.nzero - 1] == off) {   // merge
                sub.zlen[sub.nzero - 1] += (int32_t)len;
            } else if (sub.nzero < kMaxZero) {
                sub.zoff[sub.nzero] = off;
                sub.zlen[sub.nzero++] = (int32_t)len;
            } else {
                overflow = true;
            }
        };
        constexpr int kMaxRows = 512;   // the largest Keras tensor has 350 rows (rmp.0 kernel)
        uint8_t row[kMaxRows];
        for (int t = t_lo; t < t_hi && !overflow; ++t) {
            const TensorDesc& d = pt.t[t];
            if (d.rows > kMaxRows) return SPWGNN_E_ARG;
            const int64_t end = t + 1 < kNumTensors ? pt.t[t + 1].offset : pt.total;
            memset(row, 0, d.rows);   // rows (kernels) or the one bias row written by some job
            for (int k = 0; k < sub.n; ++k) {
                const ReduceArgs& ra = sub.r[k];
                if (d.rows > 1 && ra.kernel_off == d.offset)
                    for (int q = 0; q < ra.kernel_rows; ++q)
                        if (ra.kernel_row0 + q < d.rows) row[ra.kernel_row0 + q] = 1;
                if (d.rows == 1 && ra.bias_off == d.offset) row[0] = 1;
            }
            for (int q = 0; q < d.rows; ++q)
                if (!row[q]) zero(d.offset + (int64_t)q * d.cols, d.cols);
            zero(d.offset + (int64_t)d.rows * d.cols, end - d.offset - (int64_t)d.rows * d.cols);
        }
        if (overflow || (sub.n == 0 && sub.nzero > 0)) {
            SPW_CHECK(hipMemsetAsync(grads + lo, 0, (hi - lo) * sizeof(float), st));
            sub.nzero = 0;
        }
        SPW_CHECK(launch_wgrad_reduce_all(sub, st));
        return SPWGNN_OK;
    };
    if (!split) {
        if ((e = g_rm0())) return e;
        if ((e = g_rm123_w1a())) return e;
        if ((e = g_w2())) return e;
        if ((e = g_node())) return e;
        if ((e = g_om0())) return e;
        if ((e = g_om1())) return e;
        if ((e = launch_ws(wsb, true))) return e;
        return reduce(0, kNumTensors, true);
    }
    // split: the early group needs only the step loop and the node encoder's backward (Σ do1, dzo2)
    if ((e = g_w2())) return e;
    if ((e = g_node())) return e;
    if ((e = g_om1())) return e;
    if ((e = launch_ws(wsb, false))) return e;
    if ((e = reduce(T_RMP1K, kNumTensors, false))) return e;
    SPW_CHECK(hipEventRecord(static_cast<hipEvent_t>(r->grads_early_event), st));
    if (!fused && (e = edge_encoder_bwd())) return e;
    wsp = unbatched ? nullptr : &wsb2;
    if ((e = g_rm0())) return e;
    if ((e = g_om0())) return e;
    if ((e = g_rm123_w1a())) return e;
    if ((e = launch_ws(wsb2, true))) return e;
    return reduce(0, T_RMP1K, true);
}

}  // namespace spw

using namespace spw;

extern "C" {

int64_t spwgnn_workspace_bytes(int32_t n_nodes, int32_t n_eblocks, int32_t mp_steps, int32_t training) {
    if (n_nodes < 1 || n_eblocks < 1 || mp_steps < 1) return -1;
    return make_ws(n_nodes, n_eblocks, mp_steps, training ? 1 : 0).total;
}

int32_t spwgnn_fused_path(const spwgnn_batch* batch, const spwgnn_run* run) {
    const int32_t stt = validate(batch, run);
    if (stt) return stt;
    return (fwd_fused_taken(run, batch) ? 1 : 0) | (run->training && bwd_fused_taken(run, batch) ? 2 : 0);
}

int32_t spwgnn_host_device_ptr(const void* host, void** dev) {
    if (!host || !dev) return SPWGNN_E_ARG;
    void* p = nullptr;
    const hipError_t e = hipHostGetDevicePointer(&p, const_cast<void*>(host), 0);
    if (e != hipSuccess) {
        (void)hipGetLastError();   // not this thread's next launch error
        return (int32_t)e;
    }
    if (!p) return SPWGNN_E_ARG;
    *dev = p;
    return SPWGNN_OK;
}

int32_t spwgnn_team_max_blocks(int32_t set) {
    return team_max_blocks(set);
}

int32_t spwgnn_forward(const float* params, const spwgnn_batch* batch, const spwgnn_run* run, void* workspace,
                       int64_t workspace_bytes, float* logits, spwgnn_stream_t stream) {
    int32_t stt = validate(batch, run);
    if (stt) return stt;
    if (!params || !workspace || !logits) return SPWGNN_E_ARG;
    Ws w = make_ws(batch->n_nodes, batch->n_eblocks, run->mp_steps, run->training ? 1 : 0);
    if (workspace_bytes < w.total) return SPWGNN_E_WORKSPACE;
    return run_forward(params, batch, run, w, static_cast<char*>(workspace), logits,
                       static_cast<hipStream_t>(stream));
}

int32_t spwgnn_backward(const float* params, const spwgnn_batch* batch, const spwgnn_run* run, void* workspace,
                        int64_t workspace_bytes, const float* dlogits, float* grads, float* dprop,
                        spwgnn_stream_t stream) {
    int32_t stt = validate(batch, run);
    if (stt) return stt;
    if (!run->training) return SPWGNN_E_NOTRAIN;
    if (!params || !workspace || !dlogits || !grads) return SPWGNN_E_ARG;
    Ws w = make_ws(batch->n_nodes, batch->n_eblocks, run->mp_steps, 1);
    if (workspace_bytes < w.total) return SPWGNN_E_WORKSPACE;
    return run_backward(params, batch, run, w, static_cast<char*>(workspace), dlogits, grads, dprop,
                        static_cast<hipStream_t>(stream));
}

int32_t spwgnn_bce_backward(const float* params, const spwgnn_batch* batch, const spwgnn_run* run, void* workspace,
                            int64_t workspace_bytes, const float* logits, const float* targets, int64_t n,
                            float* out3, float* dlogits, void* bce_scratch, const double* weights3, double* total3,
                            float* grads, float* dprop, spwgnn_stream_t stream) {
    int32_t stt = validate(batch, run);
    if (stt) return stt;
    if (!run->training) return SPWGNN_E_NOTRAIN;
    if (!params || !workspace || !grads || !logits || !targets || !out3 || !dlogits || !bce_scratch || n < 1 ||
        (!weights3) != (!total3))
        return SPWGNN_E_ARG;
    Ws w = make_ws(batch->n_nodes, batch->n_eblocks, run->mp_steps, 1);
    if (workspace_bytes < w.total) return SPWGNN_E_WORKSPACE;
    BceArgs a{};   // as spwgnn_bce_accumulate builds it
    a.w3 = weights3;
    a.tot3 = total3;
    a.logits = logits;
    a.targets = targets;
    a.n = n;
    a.dlogits = dlogits;
    a.partial = static_cast<float*>(bce_scratch);
    a.out3 = out3;
    a.blocks = (int)std::min<int64_t>(256, (n + 255) / 256);
    return run_backward(params, batch, run, w, static_cast<char*>(workspace), dlogits, grads, dprop,
                        static_cast<hipStream_t>(stream), &a);
}

int64_t spwgnn_bce_scratch_bytes(int64_t n) {
    (void)n;
    return 256 * 2 * sizeof(float);
}

static int32_t bce_launch(const float* logits, const float* targets, int64_t n, float* out3, float* dlogits,
                          void* scratch, const double* weights3, double* total3, spwgnn_stream_t stream) {
    if (!logits || !targets || !out3 || !scratch || n < 1) return SPWGNN_E_ARG;
    BceArgs a{};
    a.w3 = weights3;
    a.tot3 = total3;
    a.logits = logits;
    a.targets = targets;
    a.n = n;
    a.dlogits = dlogits;
    a.partial = static_cast<float*>(scratch);
    a.out3 = out3;
    a.blocks = (int)std::min<int64_t>(256, (n + 255) / 256);
    hipError_t e = launch_bce(a, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? SPWGNN_OK : (int32_t)e;
}

int32_t spwgnn_bce(const float* logits, const float* targets, int64_t n, float* out3, float* dlogits, void* scratch,
                   spwgnn_stream_t stream) {
    return bce_launch(logits, targets, n, out3, dlogits, scratch, nullptr, nullptr, stream);
}

int32_t spwgnn_bce_accumulate(const float* logits, const float* targets, int64_t n, float* out3, float* dlogits,
                              void* scratch, const double* weights3, double* total3, spwgnn_stream_t stream) {
    if (!weights3 || !total3) return SPWGNN_E_ARG;
    return bce_launch(logits, targets, n, out3, dlogits, scratch, weights3, total3, stream);
}

static float adam_lr_t(float lr, float beta1, float beta2, double t) {
    return (float)(lr * std::sqrt(1.0 - std::pow((double)beta2, t)) / (1.0 - std::pow((double)beta1, t)));
}

int32_t spwgnn_adam_lr_table(float lr, float beta1, float beta2, int32_t n, float* out) {
    if (!out || n < 2) return SPWGNN_E_ARG;
    out[0] = 0.f;   // step 0 never runs (steps count from 1)
    for (int32_t t = 1; t < n; ++t) out[t] = adam_lr_t(lr, beta1, beta2, (double)t);
    return SPWGNN_OK;
}

int32_t spwgnn_adam_dev(float* params, const float* grads, float* m, float* v, int64_t n, const int32_t* step_dev,
                        const float* lr_table, int32_t table_len, float beta1, float beta2, float eps, float l2,
                        float grad_scale, spwgnn_stream_t stream) {
    if (!params || !grads || !m || !v || n < 1 || !step_dev || !lr_table || table_len < 2) return SPWGNN_E_ARG;
    AdamArgs a{};
    a.p = params;
    a.g = grads;
    a.m = m;
    a.v = v;
    a.n = n;
    a.step_dev = step_dev;
    a.lr_table = lr_table;
    a.table_len = table_len;
    a.b1 = beta1;
    a.b2 = beta2;
    a.eps = eps;
    a.l2 = l2;
    a.gscale = grad_scale;
    hipError_t e = launch_adam(a, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? SPWGNN_OK : (int32_t)e;
}

int32_t spwgnn_step_advance(uint64_t* key_dev, int32_t* step_dev, int32_t mode, uint64_t seed, int32_t rank,
                            spwgnn_stream_t stream) {
    if (!key_dev || !step_dev || mode < SPWGNN_STEP_KEY_COUNTER || mode > SPWGNN_STEP_KEY_SPLITMIX) return SPWGNN_E_ARG;
    hipError_t e = launch_step_advance(key_dev, step_dev, mode, seed, rank, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? SPWGNN_OK : (int32_t)e;
}

int32_t spwgnn_adam(float* params, const float* grads, float* m, float* v, int64_t n, int32_t step, float lr,
                    float beta1, float beta2, float eps, float l2, float grad_scale, spwgnn_stream_t stream) {
    if (!params || !grads || !m || !v || n < 1 || step < 1) return SPWGNN_E_ARG;
    AdamArgs a{};
    a.p = params;
    a.g = grads;
    a.m = m;
    a.v = v;
    a.n = n;
    const double t = step;
    a.lr_t = adam_lr_t(lr, beta1, beta2, t);
    a.b1 = beta1;
    a.b2 = beta2;
    a.eps = eps;
    a.l2 = l2;
    a.gscale = grad_scale;
    hipError_t e = launch_adam(a, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? SPWGNN_OK : (int32_t)e;
}

int32_t spwgnn_accumulate_out3(const float* out3, const double* weights3, double* total3, spwgnn_stream_t stream) {
    if (!out3 || !weights3 || !total3) return SPWGNN_E_ARG;
    hipError_t e = launch_accumulate_out3(out3, weights3, total3, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? SPWGNN_OK : (int32_t)e;
}

int32_t spwgnn_copy_in(const void* host, void* dev, int64_t bytes, spwgnn_stream_t stream) {
    if (!host || !dev || bytes < 0 || bytes % 16 || reinterpret_cast<uintptr_t>(host) % 16 ||
        reinterpret_cast<uintptr_t>(dev) % 16)
        return SPWGNN_E_ARG;
    if (bytes == 0) return SPWGNN_OK;
    hipError_t e = launch_copy_in(host, dev, bytes / 16, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? SPWGNN_OK : (int32_t)e;
}

int32_t spwgnn_sigmoid(const float* logits, float* probs, int64_t n, spwgnn_stream_t stream) {
    if (!logits || !probs || n < 1) return SPWGNN_E_ARG;
    hipError_t e = launch_sigmoid(logits, probs, n, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? SPWGNN_OK : (int32_t)e;
}

int32_t spwgnn_tower_readout(const float* logits, const int32_t* tower_offsets, int32_t n_towers, int32_t mode,
                             float* out, spwgnn_stream_t stream) {
    if (!logits || !tower_offsets || !out || n_towers < 1 || mode < SPWGNN_READOUT_SUM_PROB ||
        mode > SPWGNN_READOUT_MEAN_LOGIT)
        return SPWGNN_E_ARG;
    hipError_t e = launch_tower_readout(logits, tower_offsets, n_towers, mode, out, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? SPWGNN_OK : (int32_t)e;
}

}  // extern "C"
