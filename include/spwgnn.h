/*
 * spwgnn.h — C-ABI of libspwgnn_hip.so, the MI355X (gfx950) propagation-network engine.
 *
 * The reference (irmakguzey/SPWGNN) has no FFI: its hot path is a Keras graph built by
 * PropagationNetwork.getModel (src/Networks.py:16-104) over MLP blocks (src/Blocks.py:12-91),
 * driven by model.fit (src/main.py:92-98) and model.predict (src/JengaBuilder.py:328-329,
 * src/TowerCreator.py:430-431). Each entry point below replaces one piece of that graph; the
 * cited lines say which. Everything is plain C: raw pointers, sizes, an int status. All device
 * memory is caller-owned; the library never allocates and never synchronises, so every
 * launch function is hipGraph-capturable on the caller's stream.
 *
 * Status codes: 0 = ok, SPWGNN_E_* below, or a positive hipError_t from a failed launch.
 */
#ifndef SPWGNN_H
#define SPWGNN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPWGNN_ABI_VERSION 6   /* 6: spwgnn_bce_backward; 5: spwgnn_team_max_blocks, spwgnn_host_device_ptr, spwgnn_plan_order, spwgnn_run.grads_early_event; 4: spwgnn_run.prologue; 3: spwgnn_batch.flags, receiver-block plans */

#define SPWGNN_OK 0
#define SPWGNN_E_ARG (-1)           /* bad argument (null pointer, negative size, …)          */
#define SPWGNN_E_SHAPE (-2)         /* shape outside what the kernels support                 */
#define SPWGNN_E_RELATION (-3)      /* relation matrix column is not one-hot / both-or-neither */
#define SPWGNN_E_WORKSPACE (-4)     /* workspace smaller than spwgnn_workspace_bytes()        */
#define SPWGNN_E_CAPACITY (-5)      /* caller-provided output array too small                 */
#define SPWGNN_E_NOTRAIN (-6)       /* backward on a workspace run with training == 0         */

typedef void* spwgnn_stream_t;      /* a hipStream_t (NULL = default stream) */

/* ---------------------------------------------------------------- parameters ------------ */
/* The 22 Keras weight tensors of rm, om, rmp, omp (Networks.py:46-50, Blocks.py:20-28/60-68)
 * live in ONE flat fp32 buffer, Keras layout (kernel = [in][out] row-major, bias = [out]),
 * each tensor starting on a 64-float boundary. 209,501 real parameters. */
typedef struct spwgnn_param_info {
    const char* name;   /* e.g. "rmp.0.kernel" */
    int64_t offset;     /* in floats from the start of the flat buffer */
    int32_t rows;       /* kernel: in-features; bias: 1 */
    int32_t cols;       /* out-features */
} spwgnn_param_info;

int32_t spwgnn_version(void);
/* sizeof the ABI structs as this library was compiled (bindings check their own layouts against it):
 * which = 0 spwgnn_batch, 1 spwgnn_run, 2 spwgnn_plan_sizes, 3 spwgnn_param_info; -1 otherwise. */
int32_t spwgnn_struct_size(int32_t which);
const char* spwgnn_strerror(int32_t status);
int32_t spwgnn_param_tensor_count(void);
int64_t spwgnn_param_count(void);                 /* padded flat length (floats)       */
int64_t spwgnn_param_real_count(void);            /* 209,501                           */
int32_t spwgnn_param_tensor(int32_t index, spwgnn_param_info* out);

/* ------------------------------------------------------------- host-side input builders -- */
/* Dense relation matrices → compact edge list. Replaces the one-hot batch_dot gathers of
 * Networks.py:27-33/:84-85 and the segment-sum of :88 at the input boundary: a column k
 * of (Rs, Rr) that is one-hot in both is edge k (sender, receiver); an all-zero column is an
 * inactive relation (it never reaches an output, Networks.py:88); a column one-hot in Rs only
 * also never reaches an output and is dropped; anything else → SPWGNN_E_RELATION.
 * Rs, Rr: host fp32 [B][N][E], E = N(N-1). Output edges are tower-major, slot order (the
 * sender-major enumeration of main.py:72-81). src/dst are GLOBAL node ids (b*N + local). */
int32_t spwgnn_dense_to_edges(const float* Rs, const float* Rr, int32_t B, int32_t N,
                              int32_t* src, int32_t* dst, int32_t* slot, int64_t capacity,
                              int64_t* n_edges, int32_t* tower_edge_count);

/* Work plan for the edge kernels: towers are packed into wave-tiles of whole towers with at
 * most nw_max nodes; each wave-tile's edges are cut into 32-edge blocks (last one padded with
 * -1). blk_csr holds, per block, the block's edge slots sorted by local receiver and by local
 * sender (deterministic segment sums). Two phases: sizes, then fill. Host memory. src/dst may
 * be NULL when no tower has an edge (single-box towers, or no relation under the threshold). */
typedef struct spwgnn_plan_sizes {
    int32_t n_wtiles;
    int32_t n_eblocks;
    int32_t nw_max;     /* max nodes in any wave-tile (<= requested nw_max) */
} spwgnn_plan_sizes;

int32_t spwgnn_plan_size(int32_t n_towers, const int32_t* tower_nodes, const int32_t* tower_edges,
                         int32_t nw_max, spwgnn_plan_sizes* out);
int32_t spwgnn_plan_fill(int32_t n_towers, const int32_t* tower_nodes, const int32_t* tower_edges,
                         const int32_t* src, const int32_t* dst, int32_t nw_max,
                         const spwgnn_plan_sizes* sizes, int32_t* wtile /* [n_wtiles][4] */,
                         int32_t* edge_src /* [n_eblocks*32] */, int32_t* edge_dst,
                         int32_t* edge_id /* [n_eblocks*32] original edge index or -1 */,
                         uint8_t* blk_csr /* [n_eblocks][128] */);
/* A tower ORDER for ragged batches (the plan packs whole towers in the order given): towers by
 * decreasing edge count, each into the open wave-tile (<= nw_max nodes) whose last 32-edge block has
 * room for its edges, else a new tile; order[k] = the k-th tower, each tile's towers consecutive.
 * Planned in this order a batch needs no more blocks than in its own order and usually far fewer
 * (BASELINE config 4's ragged 4-16-box thresholded towers: 67 % -> 78 % block fill).
 * The caller permutes its towers (node rows, edge lists, targets, propagation) and keeps each
 * tower's original id for the dropout key (TowerBatch tower_ids). Deterministic. Host memory. */
int32_t spwgnn_plan_order(int32_t n_towers, const int32_t* tower_nodes, const int32_t* tower_edges, int32_t nw_max,
                          int32_t* order);

/* The same plan with each tower's blocks sized for tower_edge_cap[t] >= tower_edges[t] edges
 * (e.g. N(N-1), every relation slot): the wave-tiles and block counts then depend only on the
 * tower sizes and capacities, so batches of the same shape share one plan geometry and one
 * captured hipGraph (the unused capacity is padding, index -1, which matches no node). */
int32_t spwgnn_plan_size_cap(int32_t n_towers, const int32_t* tower_nodes, const int32_t* tower_edge_cap,
                             int32_t nw_max, spwgnn_plan_sizes* out);
int32_t spwgnn_plan_fill_cap(int32_t n_towers, const int32_t* tower_nodes, const int32_t* tower_edges,
                             const int32_t* tower_edge_cap, const int32_t* src, const int32_t* dst, int32_t nw_max,
                             const spwgnn_plan_sizes* sizes, int32_t* wtile, int32_t* edge_src, int32_t* edge_dst,
                             int32_t* edge_id, uint8_t* blk_csr);

/* Receiver blocks: every node of a wave-tile owns ONE 32-edge block that holds its in-edges (≤ 32
 * per node; input order within a receiver; nodes without in-edges get an all-padding block), so
 * wtile[w] = (first block, #nodes, first node, #nodes) and block first_block + j feeds node
 * first_node + j alone. Set SPWGNN_BATCH_RECV_BLOCKS in spwgnn_batch.flags for such a plan: the
 * x6 edge forward then sums each block's messages as one column sum instead of a one-hot product
 * (large fully connected towers, BASELINE config 5). Every other kernel takes either layout. */
int32_t spwgnn_plan_size_recv(int32_t n_towers, const int32_t* tower_nodes, int32_t nw_max, spwgnn_plan_sizes* out);
int32_t spwgnn_plan_fill_recv(int32_t n_towers, const int32_t* tower_nodes, const int32_t* tower_edges,
                              const int32_t* src, const int32_t* dst, int32_t nw_max, const spwgnn_plan_sizes* sizes,
                              int32_t* wtile, int32_t* edge_src, int32_t* edge_dst, int32_t* edge_id,
                              uint8_t* blk_csr);

/* ------------------------------------------------------------------- device batch ------- */
#define SPWGNN_BATCH_RECV_BLOCKS 1   /* spwgnn_batch.flags: the plan is a receiver-block plan */
typedef struct spwgnn_batch {
    int32_t n_towers;
    int32_t n_nodes;        /* Σ N over towers */
    int32_t n_wtiles;
    int32_t n_eblocks;
    int32_t nw_max;
    int32_t flags;          /* SPWGNN_BATCH_* (0: a plan of spwgnn_plan_fill / _fill_cap)      */
    const float* pos;           /* [n_nodes][4]: objects (x, y, w)/170 + 0 pad (Networks.py:22)   */
    const float* prop;          /* [n_nodes][100] 'propagation' input (Networks.py:29); NULL = 0  */
    const int32_t* node_tower;  /* [n_nodes] tower id (dropout key)                                */
    const int32_t* node_local; /* [n_nodes] node index inside its tower (dropout key)             */
    const int32_t* wtile;       /* [n_wtiles][4] first block, #blocks, first node, #nodes         */
    const int32_t* edge_src;    /* [n_eblocks*32] global sender, -1 = padding                     */
    const int32_t* edge_dst;    /* [n_eblocks*32] global receiver, -1 = padding                   */
    const uint8_t* blk_csr;     /* [n_eblocks][128]                                                */
} spwgnn_batch;

/* A replayed training step's first work, folded into the forward's first launch (spwgnn_run.prologue):
 * the batch upload of spwgnn_copy_in (copy_bytes from copy_src — pinned, device-mapped — to copy_dst;
 * both 16-byte aligned, copy_bytes a multiple of 16; 0 = none) and the key/step advance of
 * spwgnn_step_advance (key NULL = none; mode SPWGNN_STEP_KEY_*). The same effects as those two calls
 * issued before the forward, two launches fewer; the forward's own kernels run after them. */
typedef struct spwgnn_prologue {
    const void* copy_src;
    void* copy_dst;
    int64_t copy_bytes;
    uint64_t* key;
    int32_t* step;
    int32_t mode;
    int32_t rank;
    uint64_t seed;
} spwgnn_prologue;

typedef struct spwgnn_run {
    int32_t mp_steps;   /* propagation steps; the reference hard-codes 5 (Networks.py:83)      */
    int32_t training;   /* 1: keep activations for backward + apply dropout                      */
    float dropout;      /* Dropout rate on the two encodings (Networks.py:77-78); 0 = off      */
    int32_t math;       /* SPWGNN_MATH_*: how the fp32 matrix products run on the matrix cores   */
    uint64_t seed;      /* dropout mask key                                                       */
    /* Optional timing hook (bench/profiling): for each launch of kernel `prof_kernel`
     * (SPWGNN_K_*), the library records caller-created hipEvent_t prof_events[2k] before and
     * prof_events[2k+1] after launch k (k < prof_count) on the call's stream. 0 = off. */
    int32_t prof_kernel;
    int32_t prof_count;
    void** prof_events;
    /* Replayable steps (hipGraph): when non-NULL the dropout key is read from this device word at
     * run time instead of `seed`, so a captured step draws new masks on every replay once
     * spwgnn_step_advance has moved the key on. NULL = use `seed`. */
    const uint64_t* seed_dev;
    /* spwgnn_forward only: work to run first (above); NULL = none. Read at call time. */
    const spwgnn_prologue* prologue;
    /* spwgnn_backward only: a hipEvent_t (NULL = none). When set, the weight gradients are issued in
     * two groups and this event is recorded on the call's stream as soon as the EARLY range of the
     * flat gradient buffer is final: from the offset of "rmp.1.kernel" to the end (rmp.1, rmp.2, omp.0,
     * omp.1 — they need only the propagation-step loop). The dA rebuild, the relation encoder's backward
     * and the late range (rm, om, rmp.0) follow. A data-parallel caller all-reduces the early range on
     * another stream after hipStreamWaitEvent, overlapped with the rest of the backward.
     * Same results as without the event. */
    void* grads_early_event;
} spwgnn_run;

/* Matrix-product arithmetic. F32 and X6 give fp32-class results:
 *   F32  v_mfma_f32_*_f32: one fp32 fma chain per output (the f32 MFMA rate, 157 TF)
 *   X6   each fp32 operand split into three bf16 parts, six bf16 MFMA products per fp32 product,
 *        fp32 accumulation (6/16 of the f32 MFMA cost; error O(2^-24) per product)
 *   BF16 operands rounded to bf16, one bf16 MFMA product, fp32 accumulation; in training the
 *        stored A, U, V (the three terms of h1) rounded to bf16 once (BASELINE configs 3-4 are
 *        quoted in bf16; error O(2^-9) per product — not the fp32 parity path)                */
#define SPWGNN_MATH_F32 0
#define SPWGNN_MATH_X6 1
#define SPWGNN_MATH_BF16 2

#define SPWGNN_K_NONE 0
#define SPWGNN_K_EDGE_FWD 1
#define SPWGNN_K_NODE_FWD 2
#define SPWGNN_K_EDGE_BWD 3
#define SPWGNN_K_NODE_BWD 4
#define SPWGNN_K_ENC_EDGE 5
#define SPWGNN_K_ENC_EDGE_BWD 6
#define SPWGNN_K_WGRAD_W2 7
#define SPWGNN_K_DA 8          /* dA = Σ_s dh1pre_s rebuilt after the backward step loop (bf16 math) */
#define SPWGNN_K_WGRAD_WS 9    /* every stored-operand weight gradient (k_wgrad_ws family, split-bf16 maths) */
#define SPWGNN_K_ENC_NODE 10
#define SPWGNN_K_ENC_NODE_BWD 11

/* Workspace bytes for (n_nodes, n_eblocks, mp_steps, training). */
int64_t spwgnn_workspace_bytes(int32_t n_nodes, int32_t n_eblocks, int32_t mp_steps, int32_t training);

/* Which launches a forward / backward of this batch and run takes (no device work): bit 0 = the
 * forward's fused small-batch step loop, bit 1 = the backward's; < 0 = an error
 * status. Profilers attribute kernel time and FLOPs by it instead of restating the library's gate. */
int32_t spwgnn_fused_path(const spwgnn_batch* batch, const spwgnn_run* run);

/* Batches of at most this many 32-row blocks (edge blocks, node blocks, wave-tiles; counted per
 * launch) run the latency-oriented team kernels, larger ones the wide kernels the large-batch step
 * runs (both compute the same products in the same order). Default 512 (the
 * reference's batch 32 is ~30 blocks). set >= 0 sets the limit for the process and returns the
 * previous one; set < 0 only returns it. 0 puts every batch on the wide kernels (parity tests of the
 * large-batch path at oracle-sized batches). Read when a call plans its launches. */
int32_t spwgnn_team_max_blocks(int32_t set);

/* Forward: the whole graph of Networks.py:31-96 → per-node logits z (the model output is
 * sigmoid(z), Networks.py:94). logits: [n_nodes] device fp32. */
int32_t spwgnn_forward(const float* params, const spwgnn_batch* batch, const spwgnn_run* run,
                       void* workspace, int64_t workspace_bytes, float* logits,
                       spwgnn_stream_t stream);

/* Backward of the last spwgnn_forward on the same workspace (training == 1): dlogits [n_nodes]
 * → grads (flat, same layout as params; overwritten) and, if dprop != NULL, d/d propagation
 * [n_nodes][100]. Replaces TF autodiff of the graph (Networks.py:102 compile → fit). */
int32_t spwgnn_backward(const float* params, const spwgnn_batch* batch, const spwgnn_run* run,
                        void* workspace, int64_t workspace_bytes, const float* dlogits,
                        float* grads, float* dprop, spwgnn_stream_t stream);

/* Keras binary_crossentropy on sigmoid(logits) (Networks.py:102), mean over n:
 * out3 = {loss, sum of correct (binary_accuracy numerator), n}; dlogits = dloss/dlogit.
 * scratch: >= spwgnn_bce_scratch_bytes(n) device bytes. Deterministic. */
int64_t spwgnn_bce_scratch_bytes(int64_t n);
int32_t spwgnn_bce(const float* logits, const float* targets, int64_t n, float* out3,
                   float* dlogits, void* scratch, spwgnn_stream_t stream);
/* spwgnn_bce plus spwgnn_accumulate_out3 in the same launch: total3[k] += (double)out3[k] *
 * weights3[k] after out3 is written (model.fit's per-batch progress sums, main.py:92-98). */
int32_t spwgnn_bce_accumulate(const float* logits, const float* targets, int64_t n, float* out3,
                              float* dlogits, void* scratch, const double* weights3, double* total3,
                              spwgnn_stream_t stream);
/* ABI 6: spwgnn_bce (weights3 = total3 = NULL) or spwgnn_bce_accumulate, then spwgnn_backward on the
 * dlogits it wrote — one call, the same results bit for bit (logits: the forward's output on this
 * workspace). Where the backward runs its fused small-batch loop and the loss fits one workgroup
 * (n <= 256, the reference's batch 32), the loop computes dlogits itself (still stored to dlogits)
 * and the loss sums ride in the backward's last launch: a training step needs no loss launch of its
 * own (Keras fit, main.py:92-98). Replaces the Keras loss + autodiff pair of Networks.py:102. */
int32_t spwgnn_bce_backward(const float* params, const spwgnn_batch* batch, const spwgnn_run* run,
                            void* workspace, int64_t workspace_bytes, const float* logits,
                            const float* targets, int64_t n, float* out3, float* dlogits, void* bce_scratch,
                            const double* weights3, double* total3, float* grads, float* dprop,
                            spwgnn_stream_t stream);

/* Keras-2.x Adam (Networks.py:101: lr=5e-4, decay=0): in-place on the flat buffer.
 * g' = grad_scale*grad + 2*l2*param; lr_t = lr*sqrt(1-b2^t)/(1-b1^t);
 * m = b1 m + (1-b1) g'; v = b2 v + (1-b2) g'^2; p -= lr_t m/(sqrt(v)+eps). step = t >= 1. */
int32_t spwgnn_adam(float* params, const float* grads, float* m, float* v, int64_t n, int32_t step,
                    float lr, float beta1, float beta2, float eps, float l2, float grad_scale,
                    spwgnn_stream_t stream);

/* Replayable (hipGraph-captured) training steps: the per-step scalars live on the device.
 * spwgnn_step_advance (one thread, stream-ordered) starts a step: *step_dev += 1 and the dropout
 * key *key_dev becomes, for mode
 *   SPWGNN_STEP_KEY_COUNTER   *key_dev + 1  (the Keras front end's per-step seed counter), or
 *   SPWGNN_STEP_KEY_SPLITMIX  splitmix64 chain of (seed, step before the increment, rank, 0)
 *                             (spwgnn_amd.trainer.dropout_key — the Trainer's key).
 * spwgnn_adam_dev is spwgnn_adam with the step read from *step_dev and lr_t = lr_table[step]
 * (table_len entries, clamped), the table filled on the host by spwgnn_adam_lr_table with the
 * expression spwgnn_adam evaluates, so replayed and eager steps agree bit for bit. */
#define SPWGNN_STEP_KEY_COUNTER 0
#define SPWGNN_STEP_KEY_SPLITMIX 1
int32_t spwgnn_step_advance(uint64_t* key_dev, int32_t* step_dev, int32_t mode, uint64_t seed, int32_t rank,
                            spwgnn_stream_t stream);
int32_t spwgnn_adam_lr_table(float lr, float beta1, float beta2, int32_t n, float* out_host);
int32_t spwgnn_adam_dev(float* params, const float* grads, float* m, float* v, int64_t n, const int32_t* step_dev,
                        const float* lr_table, int32_t table_len, float beta1, float beta2, float eps, float l2,
                        float grad_scale, spwgnn_stream_t stream);

/* Epoch sums of model.fit's progress line (main.py:92-98): total3[k] += (double)out3[k] * weights3[k]
 * for k < 3 (out3 = spwgnn_bce's [loss, correct, n]; weights (n, 1, 1) make Σ loss·n) — one launch,
 * replayable, no host sync. */
int32_t spwgnn_accumulate_out3(const float* out3, const double* weights3, double* total3, spwgnn_stream_t stream);

/* Sigmoid readout (Networks.py:93-96) for predict(): probs[i] = 1/(1+exp(-logits[i])). */
int32_t spwgnn_sigmoid(const float* logits, float* probs, int64_t n, spwgnn_stream_t stream);

/* dev[0, bytes) ← host[0, bytes) by a kernel on `stream` (not a DMA copy): `host` must be pinned,
 * device-mapped memory (hipHostMalloc), both pointers 16-byte aligned, bytes a multiple of 16. A
 * replayed small-batch step makes it its first node, so the batch upload rides inside the graph. */
int32_t spwgnn_copy_in(const void* host, void* dev, int64_t bytes, spwgnn_stream_t stream);
/* The device address of pinned, device-mapped host memory (hipHostGetDevicePointer through the HIP
 * runtime this library runs on — the one the caller's allocator used), for spwgnn_copy_in and
 * spwgnn_prologue.copy_src. 0, or the hipError_t of a host range that is not device-mapped. */
int32_t spwgnn_host_device_ptr(const void* host, void** dev);

/* Per-tower readout over contiguous node ranges [tower_offsets[t], tower_offsets[t+1]):
 *   SUM_PROB   out[t] = Σ sigmoid(z)  — the stability sum of JengaBuilder.remove_to_demolish /
 *              TowerCreator.drop_to_demolish (JengaBuilder.py:252-256, TowerCreator.py:298-301),
 *              evaluated for a whole batch of candidate towers in one call;
 *   MEAN_PROB  the optional GlobalBlock-style mean pool (not in the reference);
 *   SUM_LOGIT / MEAN_LOGIT on the logits.
 * Summed sequentially in node order (deterministic). tower_offsets: n_towers + 1 int32, device. */
enum {
    SPWGNN_READOUT_SUM_PROB = 0,
    SPWGNN_READOUT_MEAN_PROB = 1,
    SPWGNN_READOUT_SUM_LOGIT = 2,
    SPWGNN_READOUT_MEAN_LOGIT = 3
};
int32_t spwgnn_tower_readout(const float* logits, const int32_t* tower_offsets, int32_t n_towers, int32_t mode,
                             float* out, spwgnn_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* SPWGNN_H */
