// Host-side pieces of libspwgnn_hip.so: parameter table, dense→edge conversion, wave-tile plan.
// Pure C++ (no device code) so the CPU test suite can exercise it without a GPU.
#include <cstdint>
#include <cstring>
#include <vector>
#include <algorithm>

#include "../../include/spwgnn.h"
#include "spwgnn_layout.h"

namespace spw {

const ParamTable& param_table() {
    static const ParamTable t = [] {
        ParamTable pt{};
        // Networks.py:46-50 — (input width, layer widths) per MLP, Keras layer order.
        struct Spec { const char* mlp; int fin; int n; int w[4]; };
        const Spec specs[4] = {{"rm", 2, 4, {150, 150, 150, 150}},
                               {"om", 2, 2, {100, 100, 0, 0}},
                               {"rmp", 350, 3, {150, 150, 100, 0}},
                               {"omp", 300, 2, {100, 101, 0, 0}}};
        static char names[kNumTensors][32];
        int64_t off = 0;
        int idx = 0;
        int64_t real = 0;
        for (const Spec& s : specs) {
            int prev = s.fin;
            for (int i = 0; i < s.n; ++i) {
                for (int kb = 0; kb < 2; ++kb) {
                    TensorDesc& d = pt.t[idx];
                    std::snprintf(names[idx], sizeof(names[idx]), "%s.%d.%s", s.mlp, i, kb == 0 ? "kernel" : "bias");
                    d.name = names[idx];
                    d.rows = kb == 0 ? prev : 1;
                    d.cols = s.w[i];
                    d.offset = off;
                    int64_t sz = (int64_t)d.rows * d.cols;
                    real += sz;
                    off += (sz + 63) / 64 * 64;
                    ++idx;
                }
                prev = s.w[i];
            }
        }
        pt.total = off;
        pt.real = real;
        return pt;
    }();
    return t;
}

}  // namespace spw

using namespace spw;

extern "C" {

int32_t spwgnn_version(void) { return SPWGNN_ABI_VERSION; }

int32_t spwgnn_struct_size(int32_t which) {
    switch (which) {
        case 0: return (int32_t)sizeof(spwgnn_batch);
        case 1: return (int32_t)sizeof(spwgnn_run);
        case 2: return (int32_t)sizeof(spwgnn_plan_sizes);
        case 3: return (int32_t)sizeof(spwgnn_param_info);
        default: return -1;
    }
}

const char* spwgnn_strerror(int32_t st) {
    switch (st) {
        case SPWGNN_OK: return "ok";
        case SPWGNN_E_ARG: return "spwgnn: bad argument";
        case SPWGNN_E_SHAPE: return "spwgnn: shape not supported by the kernels";
        case SPWGNN_E_RELATION: return "spwgnn: relation column is not one-hot (or receiver without sender)";
        case SPWGNN_E_WORKSPACE: return "spwgnn: workspace too small";
        case SPWGNN_E_CAPACITY: return "spwgnn: output capacity too small";
        case SPWGNN_E_NOTRAIN: return "spwgnn: backward needs a forward run with training=1";
        default: return st > 0 ? "spwgnn: HIP runtime error (status = hipError_t)" : "spwgnn: unknown error";
    }
}

int32_t spwgnn_param_tensor_count(void) { return kNumTensors; }
int64_t spwgnn_param_count(void) { return param_table().total; }
int64_t spwgnn_param_real_count(void) { return param_table().real; }

int32_t spwgnn_param_tensor(int32_t index, spwgnn_param_info* out) {
    if (!out || index < 0 || index >= kNumTensors) return SPWGNN_E_ARG;
    const TensorDesc& d = param_table().t[index];
    out->name = d.name;
    out->offset = d.offset;
    out->rows = d.rows;
    out->cols = d.cols;
    return SPWGNN_OK;
}

// main.py:66-81 / JengaBuilder.py:313-326 build Rs/Rr; Networks.py:32-33,84-85,88 consume them.
int32_t spwgnn_dense_to_edges(const float* Rs, const float* Rr, int32_t B, int32_t N, int32_t* src,
                              int32_t* dst, int32_t* slot, int64_t capacity, int64_t* n_edges,
                              int32_t* tower_edge_count) {
    if (!Rs || !Rr || !n_edges || B < 0 || N < 1) return SPWGNN_E_ARG;
    const int64_t E = (int64_t)N * (N - 1);
    int64_t cnt = 0;
    for (int32_t b = 0; b < B; ++b) {
        const float* rs = Rs + (int64_t)b * N * E;
        const float* rr = Rr + (int64_t)b * N * E;
        int32_t tcnt = 0;
        for (int64_t k = 0; k < E; ++k) {
            int s = -1, r = -1, ns = 0, nr = 0;
            for (int i = 0; i < N; ++i) {
                float a = rs[(int64_t)i * E + k], c = rr[(int64_t)i * E + k];
                if (a != 0.f) {
                    if (a != 1.f) return SPWGNN_E_RELATION;
                    s = i;
                    ++ns;
                }
                if (c != 0.f) {
                    if (c != 1.f) return SPWGNN_E_RELATION;
                    r = i;
                    ++nr;
                }
            }
            if (ns > 1 || nr > 1) return SPWGNN_E_RELATION;
            if (nr == 1 && ns == 0) return SPWGNN_E_RELATION;  // receiver with a zero sender row
            if (nr == 0) continue;                              // inactive relation: never summed
            if (src) {
                if (cnt >= capacity) return SPWGNN_E_CAPACITY;
                src[cnt] = b * N + s;
                dst[cnt] = b * N + r;
                if (slot) slot[cnt] = (int32_t)k;
            }
            ++cnt;
            ++tcnt;
        }
        if (tower_edge_count) tower_edge_count[b] = tcnt;
    }
    *n_edges = cnt;
    return SPWGNN_OK;
}

// Towers → wave-tiles of whole towers (≤ nw_max nodes each, in order) and 32-edge blocks per tile;
// a tile's block count follows the edge counts in `blk_edges` (actual counts, or capacities).
static int32_t plan_pack(int32_t n_towers, const int32_t* tower_nodes, const int32_t* blk_edges,
                         int32_t nw_max, std::vector<int32_t>* tile_first_tower, int32_t* n_blocks_out,
                         int32_t* nw_used) {
    if (n_towers < 0 || !tower_nodes || !blk_edges || nw_max < 1 || nw_max > kNwMaxLimit) return SPWGNN_E_ARG;
    int32_t nb = 0, used = 0;
    int32_t t = 0;
    while (t < n_towers) {
        if (tower_nodes[t] > nw_max || tower_nodes[t] < 1) return SPWGNN_E_SHAPE;
        int32_t nodes = 0, edges = 0, t0 = t;
        while (t < n_towers && nodes + tower_nodes[t] <= nw_max) {
            nodes += tower_nodes[t];
            edges += blk_edges[t];
            ++t;
        }
        if (tile_first_tower) tile_first_tower->push_back(t0);
        nb += std::max(1, (edges + 31) / 32);
        used = std::max(used, nodes);
    }
    if (tile_first_tower) tile_first_tower->push_back(n_towers);
    *n_blocks_out = nb;
    *nw_used = used;
    return SPWGNN_OK;
}

// A tower order that packs ragged towers into fewer 32-edge blocks (spwgnn_plan_order). Towers are
// placed by decreasing edge count; each joins the open wave-tile whose last block its edges fit
// without a new block (the tightest such slot, then the tightest node fit), else opens a new tile.
// The order lists each tile's towers consecutively, tiles in opening order, so plan_pack's in-order
// packing rebuilds those tiles or merges neighbours — never more blocks: ceil(a+b) <= ceil(a)+ceil(b).
static int32_t plan_order_impl(int32_t n_towers, const int32_t* tower_nodes, const int32_t* tower_edges,
                               int32_t nw_max, int32_t* order) {
    if (n_towers < 0 || (n_towers > 0 && (!tower_nodes || !tower_edges || !order)) || nw_max < 1 ||
        nw_max > kNwMaxLimit)
        return SPWGNN_E_ARG;
    std::vector<int32_t> by_edges(n_towers);
    for (int32_t t = 0; t < n_towers; ++t) {
        if (tower_nodes[t] < 1 || tower_nodes[t] > nw_max) return SPWGNN_E_SHAPE;
        if (tower_edges[t] < 0) return SPWGNN_E_ARG;
        by_edges[t] = t;
    }
    std::stable_sort(by_edges.begin(), by_edges.end(),
                     [&](int32_t a, int32_t b) { return tower_edges[a] > tower_edges[b]; });
    // open tiles by (free nodes, free slots of the last block): stacks of tile ids
    constexpr int kSlots = 32;
    std::vector<std::vector<int32_t>> open((size_t)(nw_max + 1) * (kSlots + 1));
    auto key = [&](int nf, int sf) { return (size_t)nf * (kSlots + 1) + sf; };
    std::vector<int32_t> tile_nodes, tile_edges;
    std::vector<std::vector<int32_t>> tile_towers;
    for (const int32_t t : by_edges) {
        const int n = tower_nodes[t], e = tower_edges[t];
        int tid = -1;
        if (e <= kSlots) {
            for (int sf = e; sf <= kSlots && tid < 0; ++sf)
                for (int nf = n; nf <= nw_max; ++nf) {
                    std::vector<int32_t>& b = open[key(nf, sf)];
                    if (!b.empty()) {
                        tid = b.back();
                        b.pop_back();
                        break;
                    }
                }
        }
        if (tid < 0) {
            tid = (int32_t)tile_nodes.size();
            tile_nodes.push_back(0);
            tile_edges.push_back(0);
            tile_towers.emplace_back();
        }
        tile_nodes[tid] += n;
        tile_edges[tid] += e;
        tile_towers[tid].push_back(t);
        const int nb = std::max(1, (tile_edges[tid] + kSlots - 1) / kSlots);
        const int nf = nw_max - tile_nodes[tid], sf = nb * kSlots - tile_edges[tid];
        if (nf > 0) open[key(nf, sf)].push_back(tid);   // a full tile takes no tower
    }
    int32_t k = 0;
    for (const auto& tt : tile_towers)
        for (const int32_t t : tt) order[k++] = t;
    return SPWGNN_OK;
}

static int32_t plan_size_impl(int32_t n_towers, const int32_t* tower_nodes, const int32_t* blk_edges,
                              int32_t nw_max, spwgnn_plan_sizes* out) {
    if (!out) return SPWGNN_E_ARG;
    std::vector<int32_t> first;
    int32_t nb = 0, used = 0;
    int32_t st = plan_pack(n_towers, tower_nodes, blk_edges, nw_max, &first, &nb, &used);
    if (st) return st;
    out->n_wtiles = (int32_t)first.size() - 1;
    out->n_eblocks = nb;
    out->nw_max = used;
    return SPWGNN_OK;
}

static int32_t plan_fill_impl(int32_t n_towers, const int32_t* tower_nodes, const int32_t* tower_edges,
                              const int32_t* blk_edges, const int32_t* src, const int32_t* dst, int32_t nw_max,
                              const spwgnn_plan_sizes* sizes, int32_t* wtile, int32_t* edge_src,
                              int32_t* edge_dst, int32_t* edge_id, uint8_t* blk_csr) {
    if (!sizes || !wtile || !edge_src || !edge_dst || !blk_csr || !tower_edges) return SPWGNN_E_ARG;
    std::vector<int32_t> first;
    int32_t nb = 0, used = 0;
    int32_t st = plan_pack(n_towers, tower_nodes, blk_edges, nw_max, &first, &nb, &used);
    if (st) return st;
    const int32_t ntiles = (int32_t)first.size() - 1;
    if (ntiles != sizes->n_wtiles || nb != sizes->n_eblocks) return SPWGNN_E_ARG;
    // prefix sums of nodes, edges and block-sizing edges per tower
    std::vector<int64_t> node_off(n_towers + 1, 0), edge_off(n_towers + 1, 0), cap_off(n_towers + 1, 0);
    for (int32_t t = 0; t < n_towers; ++t) {
        if (tower_edges[t] < 0 || tower_edges[t] > blk_edges[t]) return SPWGNN_E_ARG;
        node_off[t + 1] = node_off[t] + tower_nodes[t];
        edge_off[t + 1] = edge_off[t] + tower_edges[t];
        cap_off[t + 1] = cap_off[t] + blk_edges[t];
    }
    if (edge_off[n_towers] > 0 && (!src || !dst)) return SPWGNN_E_ARG;   // no list needed without edges
    int32_t blk = 0;
    for (int32_t w = 0; w < ntiles; ++w) {
        const int32_t t0 = first[w], t1 = first[w + 1];
        const int64_t n0 = node_off[t0], n1 = node_off[t1];
        const int64_t e0 = edge_off[t0], e1 = edge_off[t1];
        const int32_t nblk = std::max<int32_t>(1, (int32_t)((cap_off[t1] - cap_off[t0] + 31) / 32));
        wtile[4 * w + 0] = blk;
        wtile[4 * w + 1] = nblk;
        wtile[4 * w + 2] = (int32_t)n0;
        wtile[4 * w + 3] = (int32_t)(n1 - n0);
        int32_t te = t0;   // tower owning edge e (walks alongside e: edges are tower-major)
        for (int32_t b = 0; b < nblk; ++b, ++blk) {
            uint8_t* csr = blk_csr + (int64_t)blk * 128;
            // csr[0:32] recv order, [32:64] recv local node, [64:96] send order, [96:128] send node
            int32_t lsrc[32], ldst[32];
            int nvalid = 0;
            for (int i = 0; i < 32; ++i) {
                const int64_t e = e0 + (int64_t)b * 32 + i;
                const int64_t o = (int64_t)blk * 32 + i;
                if (e < e1) {
                    while (e >= edge_off[te + 1]) ++te;
                    const int32_t s = src[e], d = dst[e];
                    // an edge must stay inside its own tower (not merely inside the packed wave-tile)
                    if (s < node_off[te] || s >= node_off[te + 1] || d < node_off[te] || d >= node_off[te + 1])
                        return SPWGNN_E_RELATION;
                    edge_src[o] = s;
                    edge_dst[o] = d;
                    if (edge_id) edge_id[o] = (int32_t)e;
                    lsrc[i] = (int32_t)(s - n0);
                    ldst[i] = (int32_t)(d - n0);
                    ++nvalid;
                } else {
                    edge_src[o] = -1;
                    edge_dst[o] = -1;
                    if (edge_id) edge_id[o] = -1;
                    lsrc[i] = ldst[i] = 255;
                }
            }
            for (int pass = 0; pass < 2; ++pass) {
                const int32_t* key = pass == 0 ? ldst : lsrc;
                int order[32];
                for (int i = 0; i < 32; ++i) order[i] = i;
                std::stable_sort(order, order + 32, [&](int a, int b) { return key[a] < key[b]; });
                uint8_t* o = csr + pass * 64;
                for (int i = 0; i < 32; ++i) {
                    o[i] = (uint8_t)order[i];
                    o[32 + i] = (uint8_t)(i < nvalid ? key[order[i]] : 255);
                }
            }
        }
    }
    return SPWGNN_OK;
}

// Receiver blocks: each node of a wave-tile owns one 32-edge block holding its in-edges (the tile's
// edges bucketed by receiver, input order kept within a receiver; ≤ 32 in-edges per node), so block
// bb of tile w feeds node wtile[w].first_node + bb alone and its receiver sum is a column sum
// (k_edge_fwd_rb_x6). Nodes without in-edges get an all-padding block (their sum row is zero).
static int32_t plan_fill_recv_impl(int32_t n_towers, const int32_t* tower_nodes, const int32_t* tower_edges,
                                   const int32_t* src, const int32_t* dst, int32_t nw_max,
                                   const spwgnn_plan_sizes* sizes, int32_t* wtile, int32_t* edge_src,
                                   int32_t* edge_dst, int32_t* edge_id, uint8_t* blk_csr) {
    if (!sizes || !wtile || !edge_src || !edge_dst || !blk_csr || !tower_edges) return SPWGNN_E_ARG;
    std::vector<int32_t> first;
    int32_t nb = 0, used = 0;
    int32_t st = plan_pack(n_towers, tower_nodes, tower_nodes, nw_max, &first, &nb, &used);
    if (st) return st;
    const int32_t ntiles = (int32_t)first.size() - 1;
    std::vector<int64_t> node_off(n_towers + 1, 0), edge_off(n_towers + 1, 0);
    for (int32_t t = 0; t < n_towers; ++t) {
        if (tower_edges[t] < 0) return SPWGNN_E_ARG;
        node_off[t + 1] = node_off[t] + tower_nodes[t];
        edge_off[t + 1] = edge_off[t] + tower_edges[t];
    }
    int64_t nblocks = 0;
    for (int32_t w = 0; w < ntiles; ++w) nblocks += node_off[first[w + 1]] - node_off[first[w]];
    if (ntiles != sizes->n_wtiles || nblocks != sizes->n_eblocks) return SPWGNN_E_ARG;
    if (edge_off[n_towers] > 0 && (!src || !dst)) return SPWGNN_E_ARG;
    int32_t blk = 0;
    std::vector<int32_t> fill;
    for (int32_t w = 0; w < ntiles; ++w) {
        const int32_t t0 = first[w], t1 = first[w + 1];
        const int64_t n0 = node_off[t0], n1 = node_off[t1];
        const int32_t nn = (int32_t)(n1 - n0);
        wtile[4 * w + 0] = blk;
        wtile[4 * w + 1] = nn;
        wtile[4 * w + 2] = (int32_t)n0;
        wtile[4 * w + 3] = nn;
        for (int64_t o = (int64_t)blk * 32; o < (int64_t)(blk + nn) * 32; ++o) {
            edge_src[o] = edge_dst[o] = -1;
            if (edge_id) edge_id[o] = -1;
        }
        fill.assign(nn, 0);
        for (int32_t t = t0; t < t1; ++t)
            for (int64_t e = edge_off[t]; e < edge_off[t + 1]; ++e) {
                const int32_t s = src[e], d = dst[e];
                if (s < node_off[t] || s >= node_off[t + 1] || d < node_off[t] || d >= node_off[t + 1])
                    return SPWGNN_E_RELATION;
                const int32_t b = (int32_t)(d - n0);
                if (fill[b] >= 32) return SPWGNN_E_SHAPE;   // > 32 in-edges: not a receiver-block batch
                const int64_t o = (int64_t)(blk + b) * 32 + fill[b]++;
                edge_src[o] = s;
                edge_dst[o] = d;
                if (edge_id) edge_id[o] = (int32_t)e;
            }
        for (int32_t b = 0; b < nn; ++b, ++blk) {
            uint8_t* csr = blk_csr + (int64_t)blk * 128;
            int32_t lsrc[32], ldst[32];
            for (int i = 0; i < 32; ++i) {
                const int64_t o = (int64_t)blk * 32 + i;
                lsrc[i] = i < fill[b] ? (int32_t)(edge_src[o] - n0) : 255;
                ldst[i] = i < fill[b] ? (int32_t)(edge_dst[o] - n0) : 255;
            }
            for (int pass = 0; pass < 2; ++pass) {
                const int32_t* key = pass == 0 ? ldst : lsrc;
                int order[32];
                for (int i = 0; i < 32; ++i) order[i] = i;
                std::stable_sort(order, order + 32, [&](int a, int c) { return key[a] < key[c]; });
                uint8_t* o = csr + pass * 64;
                for (int i = 0; i < 32; ++i) {
                    o[i] = (uint8_t)order[i];
                    o[32 + i] = (uint8_t)(i < fill[b] ? key[order[i]] : 255);
                }
            }
        }
    }
    return SPWGNN_OK;
}

int32_t spwgnn_plan_size_recv(int32_t n_towers, const int32_t* tower_nodes, int32_t nw_max, spwgnn_plan_sizes* out) {
    if (!out) return SPWGNN_E_ARG;
    std::vector<int32_t> first;
    int32_t nb = 0, used = 0;
    const int32_t st = plan_pack(n_towers, tower_nodes, tower_nodes, nw_max, &first, &nb, &used);
    if (st) return st;
    int64_t nodes = 0;
    for (int32_t t = 0; t < n_towers; ++t) nodes += tower_nodes[t];
    out->n_wtiles = (int32_t)first.size() - 1;
    out->n_eblocks = (int32_t)nodes;
    out->nw_max = used;
    return SPWGNN_OK;
}

int32_t spwgnn_plan_fill_recv(int32_t n_towers, const int32_t* tower_nodes, const int32_t* tower_edges,
                              const int32_t* src, const int32_t* dst, int32_t nw_max, const spwgnn_plan_sizes* sizes,
                              int32_t* wtile, int32_t* edge_src, int32_t* edge_dst, int32_t* edge_id,
                              uint8_t* blk_csr) {
    return plan_fill_recv_impl(n_towers, tower_nodes, tower_edges, src, dst, nw_max, sizes, wtile, edge_src, edge_dst,
                               edge_id, blk_csr);
}

int32_t spwgnn_plan_order(int32_t n_towers, const int32_t* tower_nodes, const int32_t* tower_edges, int32_t nw_max,
                          int32_t* order) {
    return plan_order_impl(n_towers, tower_nodes, tower_edges, nw_max, order);
}

int32_t spwgnn_plan_size(int32_t n_towers, const int32_t* tower_nodes, const int32_t* tower_edges,
                         int32_t nw_max, spwgnn_plan_sizes* out) {
    return plan_size_impl(n_towers, tower_nodes, tower_edges, nw_max, out);
}

int32_t spwgnn_plan_fill(int32_t n_towers, const int32_t* tower_nodes, const int32_t* tower_edges,
                         const int32_t* src, const int32_t* dst, int32_t nw_max,
                         const spwgnn_plan_sizes* sizes, int32_t* wtile, int32_t* edge_src,
                         int32_t* edge_dst, int32_t* edge_id, uint8_t* blk_csr) {
    return plan_fill_impl(n_towers, tower_nodes, tower_edges, tower_edges, src, dst, nw_max, sizes, wtile, edge_src,
                          edge_dst, edge_id, blk_csr);
}

int32_t spwgnn_plan_size_cap(int32_t n_towers, const int32_t* tower_nodes, const int32_t* tower_edge_cap,
                             int32_t nw_max, spwgnn_plan_sizes* out) {
    return plan_size_impl(n_towers, tower_nodes, tower_edge_cap, nw_max, out);
}

int32_t spwgnn_plan_fill_cap(int32_t n_towers, const int32_t* tower_nodes, const int32_t* tower_edges,
                             const int32_t* tower_edge_cap, const int32_t* src, const int32_t* dst, int32_t nw_max,
                             const spwgnn_plan_sizes* sizes, int32_t* wtile, int32_t* edge_src, int32_t* edge_dst,
                             int32_t* edge_id, uint8_t* blk_csr) {
    return plan_fill_impl(n_towers, tower_nodes, tower_edges, tower_edge_cap, src, dst, nw_max, sizes, wtile,
                          edge_src, edge_dst, edge_id, blk_csr);
}

}  // extern "C"
