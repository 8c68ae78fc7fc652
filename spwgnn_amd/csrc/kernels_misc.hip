// Weight gradients (dW = Σ_rows Xᵀ·Y, deterministic split-row slabs + ordered reduction),
// Keras BCE loss, Keras Adam, sigmoid readout.
#include "kernels.h"
#include <cstdlib>

namespace spw {

constexpr int kWgThreads = 256;   // 4 waves; the TX×TY output tiles are dealt round-robin to waves

__device__ __forceinline__ int64_t wg_phys(int64_t L, int64_t count, int64_t stride) {
    const int64_t s = L / count, n = L - s * count;
    return (stride ? s * stride : 0) + n;
}
__device__ __forceinline__ float4 f4zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
__device__ __forceinline__ void f4set(float4& v, int k, float x) {
    if (k == 0) v.x = x; else if (k == 1) v.y = x; else if (k == 2) v.z = x; else if (k == 3) v.w = x;
}
__device__ __forceinline__ float4 f4relu(float4 v) {
    return make_float4(relu(v.x), relu(v.y), relu(v.z), relu(v.w));
}
__device__ __forceinline__ float4 f4add3(float4 a, float4 b, float4 c) {
    return make_float4(a.x + b.x + c.x, a.y + b.y + c.y, a.z + b.z + c.z, a.w + b.w + c.w);
}

// Raw operand fetch, split in two phases so global-load latency overlaps the MFMAs:
//   fetch_*  : issue the loads of one float4 group into registers (no use of the data)
//   finish_* : combine the fetched registers into the staged value (after the MFMAs)
struct XRaw { float4 a, u, v; int flag; };
struct YRaw { float4 g; int flag; };

// Row mapping of a 32-row block: logical row L = r0 + rr → (step s, row n) with n < count.
// One 64-bit division per block (scalar), then a carry per row (count >= 1).
struct RowBase { int64_t s0, n0, count; };
__device__ __forceinline__ RowBase row_base(int64_t r0, int64_t count) {
    const int64_t s0 = r0 / count;
    return {s0, r0 - s0 * count, count};
}
__device__ __forceinline__ void row_at(const RowBase& b, int rr, int64_t& s, int64_t& n) {
    s = b.s0;
    n = b.n0 + rr;
    while (n >= b.count) {   // at most once when count >= 32
        n -= b.count;
        ++s;
    }
}

__device__ __forceinline__ int64_t phys_row(const RowBase& b, int rr, int64_t stride) {
    int64_t s, n;
    row_at(b, rr, s, n);
    return (stride ? s * stride : 0) + n;
}
// chunk-major rows: block = row / 32 (32-row blocks never straddle a step: RE, RN % 32 == 0);
// 160-wide operands are 152-feature blocks (KH 76), 128-wide ones 104-feature blocks (KH 52)
template <int W>
__device__ __forceinline__ const float* cm_piece(const float* base, int64_t row, int f0) {
    return base + cm_index<W == 160 ? kKhE : kKhN>(row, f0);
}

template <int XM, int W>
__device__ __forceinline__ void fetch_x(const WgradArgs& a, const RowBase& rb, int rr, int f0, bool in, XRaw& r) {
    r.flag = 0;
    if (!in) return;
    if (XM == XM_ROW) {
        r.a = *reinterpret_cast<const float4*>(a.x_ptr + phys_row(rb, rr, a.x_stride) * a.x_ld + f0);
        r.flag = 1;
    } else if (XM == XM_CM) {
        if (f0 < 2 * (W == 160 ? kKhE : kKhN)) {
            r.a = *reinterpret_cast<const float4*>(cm_piece<W>(a.x_ptr, phys_row(rb, rr, a.x_stride), f0));
            r.flag = 1;
        }
    } else if (XM == XM_EDGE_D) {
        const int64_t n = phys_row(rb, rr, 0);
        const int sidx = a.esrc[n];
        if (sidx >= 0 && f0 == 0) {
            r.a = reinterpret_cast<const float4*>(a.pos)[sidx];
            r.u = reinterpret_cast<const float4*>(a.pos)[a.edst[n]];
            r.flag = 1;
        }
    } else {  // XM_NODE_O
        if (f0 == 0) {
            r.a = reinterpret_cast<const float4*>(a.pos)[phys_row(rb, rr, 0)];
            r.flag = 1;
        }
    }
}

template <int XM>
__device__ __forceinline__ float4 finish_x(const WgradArgs& a, int f0, const XRaw& r) {
    if (XM == XM_ROW || XM == XM_CM) {
        float4 v = r.flag ? r.a : f4zero();
        if (r.flag && a.x_ones >= f0 && a.x_ones < f0 + 4) f4set(v, a.x_ones - f0, 1.f);
        return v;
    } else if (XM == XM_EDGE_D) {
        return r.flag ? make_float4(r.u.x - r.a.x, r.u.y - r.a.y, 1.f, 0.f) : f4zero();
    } else {
        return r.flag ? make_float4(r.a.y, r.a.z, 1.f, 0.f) : f4zero();
    }
}

template <int YM, int W>
__device__ __forceinline__ void fetch_y(const WgradArgs& a, const RowBase& rb, int rr, int f0, bool in, YRaw& r) {
    r.flag = 0;
    if (!in) return;
    if (YM == YM_ROW) {
        r.g = *reinterpret_cast<const float4*>(a.y_ptr + phys_row(rb, rr, a.y_stride) * a.y_ld + f0);
        r.flag = 1;
    } else if (f0 < 2 * (W == 160 ? kKhE : kKhN)) {  // YM_CM
        r.g = *reinterpret_cast<const float4*>(cm_piece<W>(a.y_ptr, phys_row(rb, rr, a.y_stride), f0));
        r.flag = 1;
    }
}

__device__ __forceinline__ float4 finish_y(const YRaw& r) { return r.flag ? r.g : f4zero(); }

// float4 group g of a 32-row block → (row rr, column group c4): row-major operands walk a row
// per thread run (coalesced along the row); chunk-major ones walk the 32 rows of a column group
// (16 bytes per row, 512 contiguous bytes per run).
template <bool CM, int G>
__device__ __forceinline__ void group_rc(int g, int& rr, int& c4) {
    if (CM) {
        c4 = g >> 5;
        rr = g & 31;
    } else {
        rr = g / G;
        c4 = g - rr * G;
    }
}

// Chunk-major operand staging: thread tid always stages row rr = tid & 31 of a 32-row block and
// the column groups c4 = (tid >> 5) + 8k (k < W/32), so the in-block offsets are fixed per thread
// and a block costs one row map plus W/32 16-byte loads (the 32 lanes of a column group read 512
// contiguous bytes).
template <int W, bool B16 = false>   // B16: bf16-stored operand (bf16 math, §3g)
struct CmStage {
    static constexpr int KH = W == 160 ? kKhE : kKhN, BLK = KH * 64, NG = W / 32;
    int off[NG];     // in-block offset of group k for in-block row 0, -1 for padding columns (≥ 2·KH)
    int ones_k, ones_c;
    float4 raw[NG];
    __device__ __forceinline__ void init(int tid, int ones) {
        const int c0 = tid >> 5;
#pragma unroll
        for (int k = 0; k < NG; ++k) {
            const int f0 = 4 * (c0 + 8 * k);
            off[k] = f0 < 2 * KH ? cm_offk<KH>(0, f0) : -1;
        }
        ones_k = (ones >= 0 && ((ones >> 2) & 7) == c0) ? (ones >> 5) : -1;
        ones_c = ones & 3;
    }
    __device__ __forceinline__ void fetch(const float* __restrict__ base, int64_t phys, bool in) {
        // the physical row's own position in its block (logical and physical 32-row blocks differ
        // when a step's row count is not a multiple of 32)
        const int64_t ib = (phys >> 5) * BLK + (phys & 31) * 4;
        const float* b = base + ib;
        const uint16_t* b16 = reinterpret_cast<const uint16_t*>(base) + ib;
#pragma unroll
        for (int k = 0; k < NG; ++k)
            raw[k] = (in && off[k] >= 0) ? (B16 ? unpack4_bf16(*reinterpret_cast<const uint2*>(b16 + off[k]))
                                                : *reinterpret_cast<const float4*>(b + off[k]))
                                         : f4zero();
    }
    // f(rr, c4, v): the staged float4 of row rr, column group c4
    template <class F>
    __device__ __forceinline__ void emit(int tid, F&& f) const {
#pragma unroll
        for (int k = 0; k < NG; ++k) {
            float4 v = raw[k];
            if (k == ones_k) f4set(v, ones_c, 1.f);   // the bias' ones column
            f(tid & 31, (tid >> 5) + 8 * k, v);
        }
    }
    __device__ __forceinline__ void write(float* S, int ld, int tid) const {
        emit(tid, [&](int rr, int c4, float4 v) { *reinterpret_cast<float4*>(S + rr * ld + 4 * c4) = v; });
    }
};

// Recomputed edge operands of the W2 gradient (XM_H1 / YM_DH2): thread tid stages edge rr = tid & 31
// of the 32-edge block and the column groups c4 = (tid >> 5) + 8k, like CmStage; the gathered node
// rows (U[src], V[dst], G3[dst]) are chunk-major, so a group's 32 lanes read ≤ 16 distinct nodes'
// contiguous pieces. X = [relu(A + U[src] + V[dst]) | 1], Y = G3[dst] ⊙ [h2 > 0].
// Rows are walked as 32-row stages t = r0/32 = (edge block b = t / S, step s = t % S): the S steps
// of an edge block are consecutive, so its A rows (the same at every step) are fetched once.
struct EdgeStage {
    static constexpr int NG = 5;
    int off[NG];                 // in-block offset of group k for row 0 (-1: padding ≥ 152)
    int ones_k, ones_c;
    float4 ra[NG], ru[NG], rv[NG];
    uint32_t mw[NG];
    bool in;
    int pre_src, pre_dst;        // edge indices of the stage after the one being fetched
    // the edge indices run one stage ahead of the gathers that depend on them
    __device__ __forceinline__ void fetch_idx(const WgradArgs& a, int64_t r0, int tid) {
        const int64_t b = (r0 >> 5) / a.S, e = 32 * b + (tid & 31);
        const int64_t ec = r0 < a.rows ? e : 0;
        pre_src = a.esrc[ec];
        pre_dst = a.edst[ec];
    }
    __device__ __forceinline__ void init(int tid, int ones) {
        const int c0 = tid >> 5;
#pragma unroll
        for (int k = 0; k < NG; ++k) {
            const int f0 = 4 * (c0 + 8 * k);
            off[k] = f0 < 2 * kKhE ? cm_offk<kKhE>(0, f0) : -1;
        }
        ones_k = (ones >= 0 && ((ones >> 2) & 7) == c0) ? (ones >> 5) : -1;
        ones_c = ones & 3;
    }
    // rows r0..r0+31 of step s: edges e0 + rr of block blk
    template <bool X>
    __device__ __forceinline__ void fetch(const WgradArgs& a, int64_t r0, int64_t r_begin, int64_t r_end, int tid) {
        const int rr = tid & 31;
        const int64_t t = r0 >> 5, b = t / a.S, s = t - b * a.S, e = 32 * b + rr;
        const int src = pre_src, dst = pre_dst;
        fetch_idx(a, r0 + 32, tid);
        in = (r0 + rr < r_end) && src >= 0;
        const int sn = in ? src : 0, dn = in ? dst : 0;
        const int64_t nstep = s * a.RN * kRowE;
        const float* pu = (X ? a.U : a.G3) + nstep + (int64_t)(dn >> 5) * kCmBlk + (dn & 31) * 4;
        if (X) {
            if (s == 0 || r0 == r_begin) {   // wave-uniform: a new edge block
                const float* pa = a.A + b * kCmBlk + rr * 4;
#pragma unroll
                for (int k = 0; k < NG; ++k) ra[k] = *reinterpret_cast<const float4*>(pa + (off[k] < 0 ? 0 : off[k]));
            }
            const float* ps = a.U + nstep + (int64_t)(sn >> 5) * kCmBlk + (sn & 31) * 4;
            const float* pv = a.V + nstep + (int64_t)(dn >> 5) * kCmBlk + (dn & 31) * 4;
#pragma unroll
            for (int k = 0; k < NG; ++k) {
                const int o = off[k] < 0 ? 0 : off[k];
                ru[k] = *reinterpret_cast<const float4*>(ps + o);
                rv[k] = *reinterpret_cast<const float4*>(pv + o);
            }
        } else {
            const uint32_t* pm = a.mask2 + (s * (a.RE >> 5) + (e >> 5)) * kM2Blk + rr * 8;
            const int c0 = tid >> 5;
#pragma unroll
            for (int k = 0; k < NG; ++k) {
                const int o = off[k] < 0 ? 0 : off[k];
                ru[k] = *reinterpret_cast<const float4*>(pu + o);
                mw[k] = pm[(4 * (c0 + 8 * k)) >> 5];   // word (edge rr, tile of f0)
            }
        }
    }
    template <bool X, class F>
    __device__ __forceinline__ void emit(int tid, F&& f) const {
        const int c0 = tid >> 5;
#pragma unroll
        for (int k = 0; k < NG; ++k) {
            float4 v = f4zero();
            if (in && off[k] >= 0) {
                if (X) {
                    v = f4relu(f4add3(ra[k], ru[k], rv[k]));
                } else {
                    const uint32_t b = mw[k] >> ((4 * (c0 + 8 * k)) & 31);
                    v = make_float4((b & 1u) ? ru[k].x : 0.f, (b & 2u) ? ru[k].y : 0.f, (b & 4u) ? ru[k].z : 0.f,
                                    (b & 8u) ? ru[k].w : 0.f);
                }
            }
            if (X && k == ones_k) f4set(v, ones_c, 1.f);   // the b2 ones column (padding rows too: dh2 = 0)
            f(tid & 31, c0 + 8 * k, v);
        }
    }
    template <bool X>
    __device__ __forceinline__ void write(float* S, int ld, int tid) const {
        emit<X>(tid, [&](int rr, int c4, float4 v) { *reinterpret_cast<float4*>(S + rr * ld + 4 * c4) = v; });
    }
};

// Operand staging shared by the wgrad kernels: every operand is fetched a 32-row block ahead into
// registers (fetch), then handed out as float4 groups (emit_x / emit_y: f(row rr, column group c4, v)).
template <int XM, int YM, int KXP, int NYP, bool YB16 = false>
struct WgStage {
    static constexpr int GX = KXP / 4, GY = NYP / 4;
    static constexpr int NGX = (32 * GX + kWgThreads - 1) / kWgThreads;   // float4 groups per thread
    static constexpr int NGY = (32 * GY + kWgThreads - 1) / kWgThreads;
    static constexpr bool XCM = XM == XM_CM, YCM = YM == YM_CM, XH1 = XM == XM_H1, YD2 = YM == YM_DH2;
    XRaw xr[(XCM || XH1) ? 1 : NGX];
    YRaw yr[(YCM || YD2) ? 1 : NGY];
    CmStage<KXP> xc;
    CmStage<NYP, YB16> yc;
    EdgeStage xe, ye;
    int64_t xcount, ycount, r_begin, r_end;
    __device__ __forceinline__ void init(const WgradArgs& a, int64_t r_begin_, int64_t r_end_, int tid) {
        r_begin = r_begin_;
        r_end = r_end_;
        if (XCM) xc.init(tid, a.x_ones);
        if (YCM) yc.init(tid, -1);
        if (XH1) {
            xe.init(tid, a.x_ones);
            xe.fetch_idx(a, r_begin, tid);
        }
        if (YD2) {
            ye.init(tid, -1);
            ye.fetch_idx(a, r_begin, tid);
        }
        xcount = (XM == XM_ROW || XM == XM_CM) ? a.x_count : a.rows;
        ycount = a.y_count;
    }
    __device__ __forceinline__ void fetch(const WgradArgs& a, int64_t r0, int tid) {
        if constexpr (XH1) {
            xe.fetch<true>(a, r0, r_begin, r_end, tid);
        } else {
            const RowBase xb = row_base(r0, xcount);
            if constexpr (XCM) {
                const int rr = tid & 31;
                xc.fetch(a.x_ptr, phys_row(xb, rr, a.x_stride), r0 + rr < r_end);
            } else {
#pragma unroll
                for (int k = 0; k < NGX; ++k) {
                    const int g = tid + k * kWgThreads;
                    int rr, c4;
                    group_rc<false, GX>(g, rr, c4);
                    fetch_x<XM, KXP>(a, xb, rr, 4 * c4, g < 32 * GX && r0 + rr < r_end, xr[k]);
                }
            }
        }
        if constexpr (YD2) {
            ye.fetch<false>(a, r0, r_begin, r_end, tid);
        } else {
            const RowBase yb = row_base(r0, ycount);
            if constexpr (YCM) {
                const int rr = tid & 31;
                yc.fetch(a.y_ptr, phys_row(yb, rr, a.y_stride), r0 + rr < r_end);
            } else {
#pragma unroll
                for (int k = 0; k < NGY; ++k) {
                    const int g = tid + k * kWgThreads;
                    int rr, c4;
                    group_rc<false, GY>(g, rr, c4);
                    fetch_y<YM, NYP>(a, yb, rr, 4 * c4, g < 32 * GY && r0 + rr < r_end, yr[k]);
                }
            }
        }
    }
    template <class F>
    __device__ __forceinline__ void emit_x(const WgradArgs& a, int tid, F&& f) const {
        if constexpr (XH1) {
            xe.emit<true>(tid, f);
        } else if constexpr (XCM) {
            xc.emit(tid, f);
        } else {
#pragma unroll
            for (int k = 0; k < NGX; ++k) {
                const int g = tid + k * kWgThreads;
                if (g < 32 * GX) {
                    int rr, c4;
                    group_rc<false, GX>(g, rr, c4);
                    f(rr, c4, finish_x<XM>(a, 4 * c4, xr[k]));
                }
            }
        }
    }
    template <class F>
    __device__ __forceinline__ void emit_y(int tid, F&& f) const {
        if constexpr (YD2) {
            ye.emit<false>(tid, f);
        } else if constexpr (YCM) {
            yc.emit(tid, f);
        } else {
#pragma unroll
            for (int k = 0; k < NGY; ++k) {
                const int g = tid + k * kWgThreads;
                if (g < 32 * GY) {
                    int rr, c4;
                    group_rc<false, GY>(g, rr, c4);
                    f(rr, c4, finish_y(yr[k]));
                }
            }
        }
    }
};

// dW[k][n] (slab per chunk) = Σ_{rows of the chunk} X[row][k] · Y[row][n] on v_mfma_f32_16x16x4_f32.
// The (KXP/16)×(NYP/16) output tiles split 2×2 over the 4 waves (5×5 tiles of 16×16 per wave at
// 160×160, so every SIMD gets the same work); per k-step (4 rows) a wave reads MX + MY fragments
// from LDS for MX·MY MFMAs. Software pipeline per 32-row block: [barrier] write the staged
// registers → LDS [barrier] issue the next block's loads → 8 k-steps of MFMAs on the LDS block.
template <int XM, int YM, int KXP, int NYP>
__global__ __launch_bounds__(kWgThreads, 2) void k_wgrad_t(WgradArgs a) {
    constexpr int MX = KXP / 32, MY = NYP / 32;    // 16×16 tiles per wave along X / Y features
    constexpr int LDX = KXP + 16, LDY = NYP + 16;  // ≡ 16 (mod 32): the 4 rows of a fragment read
                                                   // fall in alternate bank halves (no conflicts)
    __shared__ __attribute__((aligned(16))) float Xs[32 * LDX];
    __shared__ __attribute__((aligned(16))) float Ys[32 * LDY];
    const int tid = threadIdx.x, lane = tid & 63, c16 = lane & 15, kq = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wx = wave >> 1, wy = wave & 1;
    const int64_t r_begin = (int64_t)blockIdx.x * a.rows_per_chunk;
    const int64_t r_end = min(a.rows, r_begin + a.rows_per_chunk);
    f32x4 acc[MX][MY];
#pragma unroll
    for (int x = 0; x < MX; ++x)
#pragma unroll
        for (int y = 0; y < MY; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
    WgStage<XM, YM, KXP, NYP> st;
    st.init(a, r_begin, r_end, tid);
    st.fetch(a, r_begin, tid);
    for (int64_t r0 = r_begin; r0 < r_end; r0 += 32) {
        __syncthreads();
        st.emit_x(a, tid, [&](int rr, int c4, float4 v) { *reinterpret_cast<float4*>(&Xs[rr * LDX + 4 * c4]) = v; });
        st.emit_y(tid, [&](int rr, int c4, float4 v) { *reinterpret_cast<float4*>(&Ys[rr * LDY + 4 * c4]) = v; });
        __syncthreads();
        if (r0 + 32 < r_end) st.fetch(a, r0 + 32, tid);
        const float* xs = Xs + kq * LDX + 16 * MX * wx + c16;
        const float* ys = Ys + kq * LDY + 16 * MY * wy + c16;
#pragma unroll 2
        for (int k = 0; k < 8; ++k) {
            float xa[MX], yb[MY];
#pragma unroll
            for (int x = 0; x < MX; ++x) xa[x] = xs[4 * k * LDX + 16 * x];
#pragma unroll
            for (int y = 0; y < MY; ++y) yb[y] = ys[4 * k * LDY + 16 * y];
#pragma unroll
            for (int x = 0; x < MX; ++x)
#pragma unroll
                for (int y = 0; y < MY; ++y) acc[x][y] = mfma16(xa[x], yb[y], acc[x][y]);
        }
    }
    // C layout of a 16×16 tile: reg r of lane l = row 4(l>>4) + r, col l&15
    float* out = a.slab + (int64_t)blockIdx.x * KXP * NYP;
#pragma unroll
    for (int x = 0; x < MX; ++x)
#pragma unroll
        for (int y = 0; y < MY; ++y)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                out[(int64_t)(16 * (MX * wx + x) + 4 * kq + r) * NYP + 16 * (MY * wy + y) + c16] = acc[x][y][r];
}

// Split-bf16 LDS image of a staged [32 rows][W] operand: three parts (h, m, l), each [row][W] bf16,
// read back transposed with ds_read_b64_tr_b16. 16-column units (32 B) are XOR-swizzled per row so
// that the 8 rows one 32-lane half reads land on 64 distinct banks (row pitch W·2 bytes: 80 dwords
// ≡ 16 (mod 64) at W = 160 and 32 → swizzle by row bit 2; 64 dwords at W = 128 → by row & 7).
template <int W>
struct X6Img {
    static constexpr int ROWB = W * 2, PART = 32 * ROWB;
    __device__ static __forceinline__ int sigma(int r) { return (ROWB % 256 == 0) ? (r & 7) : ((r >> 2) & 1); }
    // Within a unit the four 8-byte granules are XOR-permuted by gsw(row). The staging store
    // (ds_write_b64: groups of 16 lanes = 16 consecutive rows of one 4-column group, banks mod 32)
    // is conflict-free when (row pitch, unit swizzle, granule swizzle) give 16 distinct 8-byte slots
    // mod 32 banks: at W = 128 (pitch ≡ 0) the unit swizzle contributes row bits 0-1, so the granules
    // take bits 2-3; at W = 160 (pitch ≡ 16 dwords) the pitch gives bit 0 and the unit swizzle bit 2,
    // so the granules take bits 1 and 3. (Was `row & 3` at every width: 4-way / 2-way store
    // conflicts, SQ_LDS_BANK_CONFLICT in profiles/r02_pmc_sq.json.) The granule permutation stays
    // inside a unit, so the transposed reads keep their 64 distinct banks.
    __device__ static __forceinline__ int gsw(int r) {
        if constexpr (W == 32) return r & 3;
        else if constexpr (ROWB % 256 == 0) return (r >> 2) & 3;
        else return ((r >> 1) & 1) | (((r >> 3) & 1) << 1);
    }
    __device__ static __forceinline__ int woff(int rr, int c4) {
        return rr * ROWB + 32 * ((c4 >> 2) ^ sigma(rr)) + 8 * ((c4 & 3) ^ gsw(rr));
    }
    // lane's read offset for 16-column tile t: group g = lane>>4 reads rows 4g..4g+3 (elements 0-3)
    // and 16+4g..16+4g+3 (elements 4-7, at + 16·ROWB) — the k order of the 16x16x32 operand, the
    // same for both operands of a product (row + 16 has the same sigma and gsw as row)
    __device__ static __forceinline__ int roff(int lane, int t) {
        const int li = lane & 15, row = 4 * (lane >> 4) + (li >> 2);
        return row * ROWB + 32 * (t ^ sigma(row)) + 8 * ((li & 3) ^ gsw(row));
    }
    // NP = 1 (bf16 math): the h part only
    template <int NP = 3>
    __device__ static __forceinline__ void put(char* S, int rr, int c4, float4 v) {
        uint32_t h0, m0, l0, h1, m1, l1;
        split2(v.x, v.y, h0, m0, l0);
        split2(v.z, v.w, h1, m1, l1);
        char* p = S + woff(rr, c4);
        *reinterpret_cast<uint2*>(p) = make_uint2(h0, h1);
        if constexpr (NP == 3) {
            *reinterpret_cast<uint2*>(p + PART) = make_uint2(m0, m1);
            *reinterpret_cast<uint2*>(p + 2 * PART) = make_uint2(l0, l1);
        }
    }
    template <int NP = 3>
    __device__ static __forceinline__ void get(const char* S, int off, bf16x8 (&f)[3]) {
#pragma unroll
        for (int p = 0; p < NP; ++p)
            f[p] = as_bf16x8(lds_tr16(S + p * PART + off), lds_tr16(S + p * PART + off + 16 * ROWB));
    }
};

// The same gradient in split-bf16 math (x6): operands are split once when staged (every element
// feeds MX or MY tiles), 16x16x32 bf16 MFMAs, one k-step per 32-row block: 6·MX·MY MFMAs of 16
// cycles per wave per block instead of 8·MX·MY f32 MFMAs of 32.
template <int XM, int YM, int KXP, int NYP, int OCC, int NP = 3, bool YB16 = false>
__global__ __launch_bounds__(kWgThreads, OCC) void k_wgrad_x6(WgradArgs a) {
    constexpr int MX = KXP / 32, MY = NYP / 32;
    using IX = X6Img<KXP>;
    using IY = X6Img<NYP>;
    __shared__ __attribute__((aligned(16))) char Xs[3 * IX::PART];
    __shared__ __attribute__((aligned(16))) char Ys[3 * IY::PART];
    const int tid = threadIdx.x, lane = tid & 63, c16 = lane & 15, kq = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wx = wave >> 1, wy = wave & 1;
    const int64_t r_begin = (int64_t)blockIdx.x * a.rows_per_chunk;
    const int64_t r_end = min(a.rows, r_begin + a.rows_per_chunk);
    f32x4 acc[MX][MY];
#pragma unroll
    for (int x = 0; x < MX; ++x)
#pragma unroll
        for (int y = 0; y < MY; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
    int ox[MX], oy[MY];
#pragma unroll
    for (int x = 0; x < MX; ++x) ox[x] = IX::roff(lane, MX * wx + x);
#pragma unroll
    for (int y = 0; y < MY; ++y) oy[y] = IY::roff(lane, MY * wy + y);
    WgStage<XM, YM, KXP, NYP, YB16> st;
    st.init(a, r_begin, r_end, tid);
    st.fetch(a, r_begin, tid);
    for (int64_t r0 = r_begin; r0 < r_end; r0 += 32) {
        __syncthreads();
        st.emit_x(a, tid, [&](int rr, int c4, float4 v) { IX::template put<NP>(Xs, rr, c4, v); });
        st.emit_y(tid, [&](int rr, int c4, float4 v) { IY::template put<NP>(Ys, rr, c4, v); });
        __syncthreads();
        if (r0 + 32 < r_end) st.fetch(a, r0 + 32, tid);
        bf16x8 yb[MY][3];
#pragma unroll
        for (int y = 0; y < MY; ++y) IY::template get<NP>(Ys, oy[y], yb[y]);
#pragma unroll
        for (int x = 0; x < MX; ++x) {
            bf16x8 xa[3];
            IX::template get<NP>(Xs, ox[x], xa);
#pragma unroll
            for (int y = 0; y < MY; ++y) acc[x][y] = mfma16_x6<NP>(xa, yb[y], acc[x][y]);
        }
    }
    float* out = a.slab + (int64_t)blockIdx.x * KXP * NYP;
#pragma unroll
    for (int x = 0; x < MX; ++x)
#pragma unroll
        for (int y = 0; y < MY; ++y)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                out[(int64_t)(16 * (MX * wx + x) + 4 * kq + r) * NYP + 16 * (MY * wy + y) + c16] = acc[x][y][r];
}

// W2 gradient (x6), warp-specialized: dW2 = Σ_{s,e} [h1 | 1]ᵀ · dh2pre over all (edge, step) rows,
// h1 = relu(A + U_s[src] + V_s[dst]), dh2pre = G3_s[dst] ⊙ [h2_s > 0], recomputed from chunk-major
// rows. A 512-thread workgroup per CU walks a contiguous range of edge blocks × steps (stage t =
// (edge block b0 + t / S, step t % S)). Waves 0-3 (one per SIMD) only read split images from LDS
// and run the 16x16x32 MFMAs (5×5 tiles each, 2×2 over the 160×160 output); waves 4-7 (the
// partner wave on each SIMD) gather stage t+2 into registers, build and split stage t+1 into the
// other LDS buffer, so the matrix pipe runs while the staging VALU work issues in its gaps.
// One barrier per stage; deterministic (fixed ranges and order).
constexpr int kW2gThreads = 512;
constexpr int kW2gImg = 3 * X6Img<160>::PART;   // one operand's split image (30 KB)

// A rows of 32-edge block b (fp32, or bf16 at the fp32 element index) through a buffer descriptor
// built from wave-uniform values: the lane's offsets within a block stay fixed over the stage loop,
// so a load costs no 64-bit address arithmetic on the staging wave
template <bool AB16>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t w2_rows_rsrc(const float* A, int64_t b) {
    constexpr int EB = AB16 ? 2 : 4;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(reinterpret_cast<const char*>(A) + b * kCmBlk * EB), (short)0,
                                             kCmBlk * EB, 0x00020000);
}
template <bool AB16>
__device__ __forceinline__ void w2_row_load(__amdgpu_buffer_rsrc_t r, int vo, uint2& ah, float4& af) {
    if constexpr (AB16) {
        const auto u = __builtin_amdgcn_raw_buffer_load_b64(r, vo, 0, 0);
        ah = make_uint2(u[0], u[1]);
    } else {
        const auto u = __builtin_amdgcn_raw_buffer_load_b128(r, vo, 0, 0);
        af = make_float4(__uint_as_float(u[0]), __uint_as_float(u[1]), __uint_as_float(u[2]), __uint_as_float(u[3]));
    }
}
struct W2gSet {
    float4 a[5], u[5], v[5], g[5];
    uint2 ah[5];   // A rows stored as bf16 (AB16): unpacked where they are used (build)
    uint32_t m[5];
    int in;
};

// DBG (diagnosis builds, SPWGNN_W2G_DBG): 1 no MFMAs, 2 gathers from stage 0, 4 no staging
// arithmetic, 8 matrix waves at s_setprio 1, 32 no gathers
template <int dbg, int NP = 3, bool AB16 = false>   // AB16: A stored as bf16 (bf16 math, §3g)
__device__ __forceinline__ void w2grad_ws_body(const WgradArgs& a, int64_t blk_per_wg, int bid,
                                               char (*buf)[2 * kW2gImg]) {   // [stage parity][X | Y]
    using IM = X6Img<160>;
    const int tid = threadIdx.x;
    const int S = a.S;
    const int64_t nblk = a.RE >> 5;
    const int64_t b0 = (int64_t)bid * blk_per_wg;
    const int64_t b1 = min(nblk, b0 + blk_per_wg);
    const int T = b1 > b0 ? (int)(b1 - b0) * S : 0;   // stages of this workgroup (< 2^31)
    if (tid < 256) {
        // ---------------- matrix waves ----------------
        const int lane = tid & 63, c16 = lane & 15, kq = lane >> 4;
        const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        const int wx = wave >> 1, wy = wave & 1;
        f32x4 acc[5][5];
#pragma unroll
        for (int x = 0; x < 5; ++x)
#pragma unroll
            for (int y = 0; y < 5; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
        int ox[5], oy[5];
#pragma unroll
        for (int x = 0; x < 5; ++x) ox[x] = IM::roff(lane, 5 * wx + x);
#pragma unroll
        for (int y = 0; y < 5; ++y) oy[y] = IM::roff(lane, 5 * wy + y);
        if constexpr ((dbg & 8) != 0) __builtin_amdgcn_s_setprio(1);
        __syncthreads();   // stage 0 staged
        for (int t = 0; t < T; ++t) {
            if constexpr ((dbg & 1) != 0) { __syncthreads(); continue; }
            const char* Xs = buf[t & 1];
            const char* Ys = Xs + kW2gImg;
            // fragment reads run one (x, y) group ahead of the MFMAs that use them: X0 Y0 | Y1 ·
            // (0,0) | Y2 · (0,1) | … | X1 · (0,4) | X2 · (1,*) | X3 · (2,*) | X4 · (3,*) | (4,*)
            bf16x8 yb[5][3], xa[2][3];
            IM::template get<NP>(Xs, ox[0], xa[0]);
            IM::template get<NP>(Ys, oy[0], yb[0]);
#pragma unroll
            for (int y = 0; y < 5; ++y) {
                if (y < 4) IM::template get<NP>(Ys, oy[y + 1], yb[y + 1]);
                else IM::template get<NP>(Xs, ox[1], xa[1]);
                __builtin_amdgcn_sched_barrier(0);
                acc[0][y] = mfma16_x6<NP>(xa[0], yb[y], acc[0][y]);
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int x = 1; x < 5; ++x) {
                if (x < 4) IM::template get<NP>(Xs, ox[x + 1], xa[(x + 1) & 1]);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int y = 0; y < 5; ++y) acc[x][y] = mfma16_x6<NP>(xa[x & 1], yb[y], acc[x][y]);
                __builtin_amdgcn_sched_barrier(0);
            }
            __syncthreads();
        }
        float* out = a.slab + (int64_t)bid * 160 * 160;
#pragma unroll
        for (int x = 0; x < 5; ++x)
#pragma unroll
            for (int y = 0; y < 5; ++y)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    out[(int64_t)(16 * (5 * wx + x) + 4 * kq + r) * 160 + 16 * (5 * wy + y) + c16] = acc[x][y][r];
        return;
    }
    // ---------------- staging waves ----------------
    // thread: edge rr of the 32-edge block, column groups c4 = c0 + 8k (k < 5; c4 ≥ 38 is padding)
    const int st = tid - 256, rr = st & 31, c0 = st >> 5;
    const bool k4ok = __builtin_amdgcn_readfirstlane(st >> 6) < 3;   // c0 < 6: staging waves 0-2
    int off[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) off[k] = (k < 4 || k4ok) ? cm_offk<kKhE>(0, 4 * (c0 + 8 * k)) : 0;
    int voa[5];   // byte offsets of the lane's A-row groups within a 32-edge block
#pragma unroll
    for (int k = 0; k < 5; ++k) voa[k] = (rr * 4 + off[k]) * (AB16 ? 2 : 4);
    const int64_t nstep_n = a.RN * kRowE;
    auto stage_of = [&](int t, int64_t& b, int& s) {
        const uint32_t tc = (uint32_t)(t < T ? t : T - 1);
        const uint32_t q = tc / (uint32_t)S;
        b = b0 + q;
        s = (int)(tc - q * (uint32_t)S);
    };
    auto load_idx = [&](int t, int2& idx) {
        int64_t b; int s;
        stage_of(t, b, s);
        idx.x = a.esrc[32 * b + rr];
        idx.y = a.edst[32 * b + rr];
    };
    auto fetch = [&](int t, const int2& idx, W2gSet& R) {
        if constexpr ((dbg & 32) != 0) return;
        if constexpr ((dbg & 2) != 0) t = 0;
        int64_t b; int s;
        stage_of(t, b, s);
        R.in = idx.x >= 0;
        const int sn = R.in ? idx.x : 0, dn = R.in ? idx.y : 0;
        const int64_t ns = (int64_t)s * nstep_n;
        const float* pu = a.U + ns + (int64_t)(sn >> 5) * kCmBlk + (sn & 31) * 4;
        const int64_t dno = ns + (int64_t)(dn >> 5) * kCmBlk + (dn & 31) * 4;
        const float* pv = a.V + dno;
        const float* pg = a.G3 + dno;
        uint32_t mw[5];
        load_m2(a.mask2 + ((int64_t)s * nblk + b) * kM2Blk, rr, mw);
        // A rows: buffer loads from the block's (wave-uniform) base at fixed lane offsets
        const auto rA = w2_rows_rsrc<AB16>(a.A, b);
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            w2_row_load<AB16>(rA, voa[k], R.ah[k], R.a[k]);   // re-read by the block's next steps
            R.u[k] = *reinterpret_cast<const float4*>(pu + off[k]);
            R.v[k] = *reinterpret_cast<const float4*>(pv + off[k]);
            R.g[k] = *reinterpret_cast<const float4*>(pg + off[k]);
            R.m[k] = mw[k];
        }
    };
    auto build = [&](const W2gSet& R, char* Xs) {
        if constexpr ((dbg & 4) != 0) return;
        char* Ys = Xs + kW2gImg;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            if (k == 4 && !k4ok) break;
            float4 x = f4relu(f4add3(AB16 ? unpack4_bf16(R.ah[k]) : R.a[k], R.u[k], R.v[k]));
            if (k == 4 && c0 == 5) x.z = 1.f;   // feature 150: the b2 ones column
            // dh2pre = G3 ⊙ [h2 > 0]: sign-extended single-bit fields as AND masks
            const int w = (int)(R.in ? R.m[k] : 0u);
            const float4 gv = R.g[k];
            const float4 y = make_float4(
                __int_as_float(__float_as_int(gv.x) & __builtin_amdgcn_sbfe(w, 4 * c0, 1)),
                __int_as_float(__float_as_int(gv.y) & __builtin_amdgcn_sbfe(w, 4 * c0 + 1, 1)),
                __int_as_float(__float_as_int(gv.z) & __builtin_amdgcn_sbfe(w, 4 * c0 + 2, 1)),
                __int_as_float(__float_as_int(gv.w) & __builtin_amdgcn_sbfe(w, 4 * c0 + 3, 1)));
            IM::template put<NP>(Xs, rr, c0 + 8 * k, x);
            IM::template put<NP>(Ys, rr, c0 + 8 * k, y);
        }
    };
    if (T == 0) {
        __syncthreads();
        return;
    }
    if (!k4ok) {   // padding columns 152..159 of both operands in both buffers stay zero
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            IM::template put<NP>(buf[p], rr, c0 + 32, f4zero());
            IM::template put<NP>(buf[p] + kW2gImg, rr, c0 + 32, f4zero());
        }
    }
    W2gSet R0, R1;
    int2 i0, i1;
    load_idx(0, i0);
    load_idx(1, i1);
    fetch(0, i0, R0);
    load_idx(2, i0);
    fetch(1, i1, R1);
    load_idx(3, i1);
    build(R0, buf[0]);
    __syncthreads();   // stage 0 staged
    // iteration t: gather stage t+2 (set t&1, indices loaded an iteration earlier), load the
    // indices of stage t+3, build stage t+1 (set (t+1)&1) into buffer (t+1)&1, barrier
    int t = 0;
    for (; t + 2 < T; t += 2) {
        fetch(t + 2, i0, R0);
        load_idx(t + 4, i0);
        build(R1, buf[1]);
        __syncthreads();
        fetch(t + 3, i1, R1);
        load_idx(t + 5, i1);
        build(R0, buf[0]);
        __syncthreads();
    }
    if (t + 1 < T) {   // t even: build stage t+1 from set 1
        build(R1, buf[1]);
        __syncthreads();
        ++t;
    }
    __syncthreads();   // the matrix waves' last stage
}
template <int dbg, int NP = 3, bool AB16 = false>
__global__ __launch_bounds__(kW2gThreads, 1) __attribute__((amdgpu_waves_per_eu(2, 2)))
void k_w2grad_ws(WgradArgs a, int64_t blk_per_wg) {
    __shared__ __attribute__((aligned(16))) char buf[2][2 * kW2gImg];
    w2grad_ws_body<dbg, NP, AB16>(a, blk_per_wg, blockIdx.x, buf);
}

// W2 gradient with the node rows staged in LDS per (wave-tile, step) — bf16 math. The per-edge
// gathers of U[src], V[dst], G3[dst] bound k_w2grad_ws there: diagnosis builds at config 3 (65,536
// fully connected 12-block towers) ran 8.4 ms with the gathers, 7.2 ms with every gather hitting the
// cache, 2.5 ms without them — the vector-memory instruction stream, not HBM. Here a workgroup walks
// whole wave-tiles (tile-major, then step, then 32-edge block): for each (tile, step) group the ≤ 16
// node rows of U, V and G3 are loaded once with coalesced loads (one group ahead, into registers) and
// written to an LDS node buffer (double-buffered by group parity); each edge then reads its rows
// from LDS. A rows and the h2 > 0 words stay per-stage global loads (contiguous per block). Matrix
// waves, images, products and the per-workgroup slab are k_w2grad_ws's; stages differ only in order,
// so the gradient is the same sum in a different fixed order (deterministic).
constexpr int kW2tNodes = 16;                          // ≤ 16-node wave-tiles (default plan for N ≤ 16)
constexpr int kW2tChunks = kRowE / 4;                  // 38 float4 chunks per 152-feature row
constexpr int kW2tUnits = 3 * kW2tNodes * kW2tChunks;  // U, V, G3 chunks of one group: 1824
constexpr int kW2tPf = (kW2tUnits + 255) / 256;        // per staging thread: 8

struct W2tSet {
    uint2 ah[5];
    float4 a[5];
    uint32_t m[5];
    int src, dst;
};
struct W2tIt {   // stage iterator (wave-uniform): tile ti, step s, block bb of the tile
    int ti, s, bb;
    int4 info;   // wtile[ti]: first block, blocks, first node, nodes
};

// DBG (diagnosis builds, SPWGNN_W2G_DBG with SPWGNN_DIAG; wrong results): 1 no node-row LDS reads,
// 2 no per-stage global loads (A, h2 words, indices), 4 no node-row loads/stores, 8 no staging
// stores (nor the arithmetic feeding them), 16 no MFMAs
// UV16 (kUvB16, §3ze): U and V rows stored as bf16 (each step's element index from its fp32 step start)
template <int NP, bool AB16, int DBG = 0, bool UV16 = false>
__global__ __launch_bounds__(kW2gThreads, 1) __attribute__((amdgpu_waves_per_eu(2, 2)))
void k_w2grad_tile(WgradArgs a, int64_t blk_per_wg) {
    using IM = X6Img<160>;
    constexpr int IMG = NP * IM::PART;
    __shared__ __attribute__((aligned(16))) char buf[2][2 * IMG];            // [stage parity][X | Y]
    __shared__ __attribute__((aligned(16))) float4 nodes[2][kW2tUnits];      // [group parity][arr][node][chunk]
    const int tid = threadIdx.x;
    const int S = a.S;
    const int nt = a.n_wtiles;
    const int4* wt = reinterpret_cast<const int4*>(a.wtile);
    const int64_t nblk = a.RE >> 5;
    // this workgroup's wave-tiles: those whose first block lies in [w·bpw, (w+1)·bpw)
    auto lower = [&](int64_t blk) {
        int lo = 0, hi = nt;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (wt[mid].x < blk) lo = mid + 1; else hi = mid;
        }
        return lo;
    };
    const int tlo = lower((int64_t)blockIdx.x * blk_per_wg);
    const int thi = lower((int64_t)(blockIdx.x + 1) * blk_per_wg);
    const int64_t blo = tlo < nt ? wt[tlo].x : nblk, bhi = thi < nt ? wt[thi].x : nblk;
    const int T = (int)(bhi - blo) * S;
    if (tid < 256) {
        // ---------------- matrix waves (as k_w2grad_ws) ----------------
        const int lane = tid & 63, c16 = lane & 15, kq = lane >> 4;
        const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        const int wx = wave >> 1, wy = wave & 1;
        f32x4 acc[5][5];
#pragma unroll
        for (int x = 0; x < 5; ++x)
#pragma unroll
            for (int y = 0; y < 5; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
        int ox[5], oy[5];
#pragma unroll
        for (int x = 0; x < 5; ++x) ox[x] = IM::roff(lane, 5 * wx + x);
#pragma unroll
        for (int y = 0; y < 5; ++y) oy[y] = IM::roff(lane, 5 * wy + y);
        __syncthreads();   // group 0's node rows in LDS (the staging waves' prologue barrier)
        __syncthreads();   // stage 0 staged
        for (int t = 0; t < T; ++t) {
            const char* Xs = buf[t & 1];
            const char* Ys = Xs + IMG;
            if constexpr ((DBG & 16) != 0) { __syncthreads(); continue; }
            bf16x8 yb[5][3], xa[2][3];
            IM::template get<NP>(Xs, ox[0], xa[0]);
            IM::template get<NP>(Ys, oy[0], yb[0]);
#pragma unroll
            for (int y = 0; y < 5; ++y) {
                if (y < 4) IM::template get<NP>(Ys, oy[y + 1], yb[y + 1]);
                else IM::template get<NP>(Xs, ox[1], xa[1]);
                __builtin_amdgcn_sched_barrier(0);
                acc[0][y] = mfma16_x6<NP>(xa[0], yb[y], acc[0][y]);
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int x = 1; x < 5; ++x) {
                if (x < 4) IM::template get<NP>(Xs, ox[x + 1], xa[(x + 1) & 1]);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int y = 0; y < 5; ++y) acc[x][y] = mfma16_x6<NP>(xa[x & 1], yb[y], acc[x][y]);
                __builtin_amdgcn_sched_barrier(0);
            }
            __syncthreads();
        }
        float* out = a.slab + (int64_t)blockIdx.x * 160 * 160;
#pragma unroll
        for (int x = 0; x < 5; ++x)
#pragma unroll
            for (int y = 0; y < 5; ++y)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    out[(int64_t)(16 * (5 * wx + x) + 4 * kq + r) * 160 + 16 * (5 * wy + y) + c16] = acc[x][y][r];
        return;
    }
    // ---------------- staging waves ----------------
    const int st = tid - 256, rr = st & 31, c0 = st >> 5;
    const bool k4ok = __builtin_amdgcn_readfirstlane(st >> 6) < 3;   // c0 < 6: chunk c0 + 32 < 38
    int off[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) off[k] = (k < 4 || k4ok) ? cm_offk<kKhE>(0, 4 * (c0 + 8 * k)) : 0;
    int voa[5];   // byte offsets of the lane's A-row groups within a 32-edge block
#pragma unroll
    for (int k = 0; k < 5; ++k) voa[k] = (rr * 4 + off[k]) * (AB16 ? 2 : 4);
    const int64_t nstep_n = a.RN * kRowE;
    if (T == 0) {   // the matrix waves' two barriers (they write a zero slab)
        __syncthreads();
        __syncthreads();
        return;
    }
    auto tile_info = [&](int ti) { return wt[ti < thi ? ti : thi - 1]; };
    auto advance = [&](W2tIt& it) {
        if (++it.bb >= it.info.y) {
            it.bb = 0;
            if (++it.s >= S) {
                it.s = 0;
                ++it.ti;
                it.info = tile_info(it.ti);
            }
        }
    };
    auto fetch = [&](const W2tIt& it, W2tSet& R) {
        if constexpr ((DBG & 2) != 0) {
            R.src = R.dst = rr;
#pragma unroll
            for (int k = 0; k < 5; ++k) { R.ah[k] = make_uint2(0x3f803f80u, 0u); R.a[k] = f4zero(); R.m[k] = ~0u; }
            return;
        }
        const int64_t b = (int64_t)it.info.x + it.bb;
        R.src = a.esrc[32 * b + rr];
        R.dst = a.edst[32 * b + rr];
        load_m2(a.mask2 + ((int64_t)it.s * nblk + b) * kM2Blk, rr, R.m);
        const auto rA = w2_rows_rsrc<AB16>(a.A, b);
#pragma unroll
        for (int k = 0; k < 5; ++k) w2_row_load<AB16>(rA, voa[k], R.ah[k], R.a[k]);
    };
    // one group's node rows: unit u = (arr·38 + chunk)·16 + node (node fastest: coalesced per chunk)
    float4 pf[kW2tPf];
    // UV16: per array three slots of 256 units (arr = slot / 3, a compile-time value: the bf16 U/V
    // pieces and the fp32 G3 pieces land in registers of their own type, so no load result is merged
    // with another's and the loads' wait stays in node_store)
    constexpr int kUvSlots = 3, kArrUnits = kW2tChunks * kW2tNodes;   // 608 units per array
    uint2 pfuv[2 * kUvSlots];
    float4 pfg[kUvSlots];
    auto node_fetch = [&](int ti, int s) {
        if constexpr ((DBG & 4) != 0) return;
        const int4 inf = tile_info(ti);
        const int64_t ns = (int64_t)s * nstep_n;
        if constexpr (UV16) {
#pragma unroll
            for (int k = 0; k < 3 * kUvSlots; ++k) {
                const int arr = k / kUvSlots, ua = st + 256 * (k % kUvSlots);
                const int q = ua >> 4, nd = ua & 15;
                const int64_t e = cm_index<kKhE>(inf.z + nd, 4 * q);
                if (arr < 2) {
                    pfuv[k] = make_uint2(0u, 0u);
                    if (ua < kArrUnits && nd < inf.w)
                        pfuv[k] = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>((arr == 0 ? a.U : a.V) + ns) + e);
                } else {
                    pfg[k - 2 * kUvSlots] = f4zero();
                    if (ua < kArrUnits && nd < inf.w) pfg[k - 2 * kUvSlots] = *reinterpret_cast<const float4*>(a.G3 + ns + e);
                }
            }
            return;
        }
#pragma unroll
        for (int j = 0; j < kW2tPf; ++j) {
            const int u = st + 256 * j;
            const int arr = u / (kW2tChunks * kW2tNodes), rem = u - arr * (kW2tChunks * kW2tNodes);
            const int q = rem >> 4, nd = rem & 15;
            pf[j] = f4zero();
            if (u < kW2tUnits && nd < inf.w) {
                const float* base = arr == 0 ? a.U : (arr == 1 ? a.V : a.G3);
                pf[j] = *reinterpret_cast<const float4*>(base + ns + cm_index<kKhE>(inf.z + nd, 4 * q));
            }
        }
    };
    auto node_store = [&](int par) {
        if constexpr ((DBG & 4) != 0) return;
        if constexpr (UV16) {
#pragma unroll
            for (int k = 0; k < 3 * kUvSlots; ++k) {
                const int arr = k / kUvSlots, ua = st + 256 * (k % kUvSlots);
                const int q = ua >> 4, nd = ua & 15;
                if (ua < kArrUnits)
                    nodes[par][(arr * kW2tNodes + nd) * kW2tChunks + q] =
                        arr < 2 ? unpack4_bf16(pfuv[k < 2 * kUvSlots ? k : 0]) : pfg[k < 2 * kUvSlots ? 0 : k - 2 * kUvSlots];
            }
            return;
        }
#pragma unroll
        for (int j = 0; j < kW2tPf; ++j) {
            const int u = st + 256 * j;
            const int arr = u / (kW2tChunks * kW2tNodes), rem = u - arr * (kW2tChunks * kW2tNodes);
            const int q = rem >> 4, nd = rem & 15;
            if (u < kW2tUnits) nodes[par][(arr * kW2tNodes + nd) * kW2tChunks + q] = pf[j];
        }
    };
    int gpar = 0;   // node buffer of the group being built
    auto build = [&](const W2tIt& it, const W2tSet& R, char* Xs) {
        if (it.bb == 0) {   // first stage of its group: fetch the next group's rows
            const bool more_steps = it.s + 1 < S;
            node_fetch(more_steps ? it.ti : it.ti + 1, more_steps ? it.s + 1 : 0);
        }
        char* Ys = Xs + IMG;
        const float4* nb = nodes[gpar];
        const bool in = R.src >= 0;
        const int sl = in ? R.src - it.info.z : 0, dl = in ? R.dst - it.info.z : 0;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            if (k == 4 && !k4ok) break;
            const int cg = c0 + 8 * k;
            const float4 u = (DBG & 1) ? make_float4(0.1f, 0.2f, 0.3f, 0.4f) : nb[sl * kW2tChunks + cg];
            const float4 v = (DBG & 1) ? make_float4(0.1f, 0.2f, 0.3f, 0.4f) : nb[(kW2tNodes + dl) * kW2tChunks + cg];
            const float4 gv = (DBG & 1) ? make_float4(0.1f, 0.2f, 0.3f, 0.4f) : nb[(2 * kW2tNodes + dl) * kW2tChunks + cg];
            float4 x = f4relu(f4add3(AB16 ? unpack4_bf16(R.ah[k]) : R.a[k], u, v));
            if (k == 4 && c0 == 5) x.z = 1.f;   // feature 150: the b2 ones column
            const int w = (int)(in ? R.m[k] : 0u);
            const float4 y = make_float4(
                __int_as_float(__float_as_int(gv.x) & __builtin_amdgcn_sbfe(w, 4 * c0, 1)),
                __int_as_float(__float_as_int(gv.y) & __builtin_amdgcn_sbfe(w, 4 * c0 + 1, 1)),
                __int_as_float(__float_as_int(gv.z) & __builtin_amdgcn_sbfe(w, 4 * c0 + 2, 1)),
                __int_as_float(__float_as_int(gv.w) & __builtin_amdgcn_sbfe(w, 4 * c0 + 3, 1)));
            if constexpr ((DBG & 8) == 0) {
                IM::template put<NP>(Xs, rr, cg, x);
                IM::template put<NP>(Ys, rr, cg, y);
            }
        }
        if (it.bb == it.info.y - 1) {   // last stage of its group: the next group's rows → LDS
            node_store(gpar ^ 1);
            gpar ^= 1;
        }
    };
    if (!k4ok) {   // padding columns 152..159 of both operands in both buffers stay zero
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            IM::template put<NP>(buf[p], rr, c0 + 32, f4zero());
            IM::template put<NP>(buf[p] + IMG, rr, c0 + 32, f4zero());
        }
    }
    // prologue: group 0's rows, stages 0 and 1 fetched, stage 0 built
    W2tIt ib{tlo, 0, 0, tile_info(tlo)};
    node_fetch(ib.ti, 0);
    node_store(0);
    __syncthreads();   // group 0's node rows visible to every staging wave
    W2tIt i1 = ib;
    advance(i1);
    W2tIt i2 = i1;
    advance(i2);
    W2tSet R0, R1;
    fetch(ib, R0);
    fetch(i1, R1);
    build(ib, R0, buf[0]);
    __syncthreads();   // stage 0 staged
    // iteration t: fetch stage t+2 into the set stage t used, build stage t+1, barrier
    int t = 0;
    for (; t + 2 < T; t += 2) {
        fetch(i2, R0);
        build(i1, R1, buf[1]);
        __syncthreads();
        i1 = i2;
        advance(i2);
        fetch(i2, R1);
        build(i1, R0, buf[0]);
        __syncthreads();
        i1 = i2;
        advance(i2);
    }
    if (t + 1 < T) {   // t even: build stage t+1 from set 1
        build(i1, R1, buf[1]);
        __syncthreads();
        ++t;
    }
    __syncthreads();   // the matrix waves' last stage
}

// Stored-operand weight gradients (x6), warp-specialized like k_w2grad_ws: dW[k][n] =
// Σ_rows X[row][k]·Y[row][n] with X chunk-major and Y chunk-major (YROW = 0) or row-major
// (YROW = 1, stride 160: the dA rows). Stages are 32-row blocks t = (step s, block nb) of a
// [S][nbs] grid; X block s·x_sb + nb (x_sb = 0: an operand shared by every step), Y block
// s·y_sb + nb; rows ≥ count of a step are masked (MASK). Waves 0-3 run the MFMAs on
// double-buffered split images, waves 4-7 stream the operands three stages ahead and split them.
constexpr int kWsThreads = 512;

template <int KXP, int NYP, int YROW, bool MASK>
struct WsStage {
    static constexpr int KHX = KXP == 160 ? kKhE : kKhN, KHY = NYP == 160 ? kKhE : kKhN;
    static constexpr int GX = KHX / 2, GY = YROW ? NYP / 4 : KHY / 2;   // float4 groups per row
    static constexpr int NKX = (GX + 7) / 8, NKY = (GY + 7) / 8;        // groups per staging thread
    static constexpr int IMX = 3 * X6Img<KXP>::PART, IMY = 3 * X6Img<NYP>::PART;
    static constexpr int BUF = IMX + IMY;
};
struct WsSet4 {
    float4 x[5], y[5];
    uint2 xh[5], yh[5];   // bf16-stored operands in bf16 math: the raw element pairs (no unpack)
    float2 d;
    int nvalid;
};

// XD: X = [z1 | 1] rebuilt from the per-edge (dx, dy) (XD 1), or [zo1 | 1] from the node's (y, w)
// (XD 2), with the encoders' own first-layer arithmetic (dense2 + relu on the same pack):
// bit-identical to the activations the encoders no longer store.
// B16 (bf16 math, §3g): X (kB16X) and/or Y (kB16Y) stored as bf16 with the fp32 element layout.
// The body of one workgroup `bid` of a weight gradient; smem: two stage buffers of W::BUF bytes
// (k_wgrad_ws: its own; k_wgrad_ws_batch: the largest variant's, shared by every job of the batch).
// SPWGNN_WS_DBG (diagnosis builds, wrong results, timing only): 1 staging without global loads,
// 2 staging without the split (raw bits into the three part images), 3 staging without LDS writes,
// 4 matrix waves without MFMAs (fragment reads kept), 5 matrix waves without fragment reads (MFMAs on
// constant fragments), 6 staging waves idle (barriers only)
#ifndef SPWGNN_WS_DBG
#define SPWGNN_WS_DBG 0
#endif
#ifndef SPWGNN_WS_NSET   // stage sets the staging waves keep in flight (k_wgrad_ws)
#define SPWGNN_WS_NSET 4
#endif
#ifndef SPWGNN_WS_NSET_B16   // the same in bf16 math (half the bytes per load)
#define SPWGNN_WS_NSET_B16 4
#endif
template <int KXP, int NYP, int YROW, bool MASK, int NP, int XD, int B16>
__device__ __forceinline__ void wgrad_ws_body(const WgWsArgs& a, int bid, char* smem) {
    constexpr int DBG = SPWGNN_WS_DBG;
    // bf16 math over bf16-stored operands: the stored element pairs ARE the h parts of the image
    // (rounding an exactly representable value is the identity), so they go to LDS as loaded — no
    // unpack, mask select or re-pack per element on the staging wave's VALU stream
    constexpr bool kRawX = NP == 1 && (B16 & kB16X) && XD == 0 && DBG == 0;
    constexpr bool kRawY = NP == 1 && (B16 & kB16Y) && DBG == 0;
    using W = WsStage<KXP, NYP, YROW, MASK>;
    using IX = X6Img<KXP>;
    using IY = X6Img<NYP>;
    constexpr int MX = KXP / 32, MY = NYP / 32;
    auto buf = [&](int p) { return smem + p * W::BUF; };   // (offsets, not a pointer array: keeps the LDS address space)
    const int tid = threadIdx.x;
    const int64_t t0 = (int64_t)bid * a.stages_per_wg;
    const int64_t nst = a.nbs * a.S;
    const int T = t0 < nst ? (int)min<int64_t>(a.stages_per_wg, nst - t0) : 0;
    if (tid < 256) {
        const int lane = tid & 63, c16 = lane & 15, kq = lane >> 4;
        const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        const int wx = wave >> 1, wy = wave & 1;
        f32x4 acc[MX][MY];
#pragma unroll
        for (int x = 0; x < MX; ++x)
#pragma unroll
            for (int y = 0; y < MY; ++y) acc[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
        int ox[MX], oy[MY];
#pragma unroll
        for (int x = 0; x < MX; ++x) ox[x] = IX::roff(lane, MX * wx + x);
#pragma unroll
        for (int y = 0; y < MY; ++y) oy[y] = IY::roff(lane, MY * wy + y);
        __syncthreads();
        // diagnosis forms: the products, or the fragment reads, taken away
        auto mm = [&](const bf16x8 (&xf)[3], const bf16x8 (&yf)[3], f32x4 c) {
            if constexpr (DBG == 4) {
                c[0] += __builtin_bit_cast(f32x4, xf[0])[0] + __builtin_bit_cast(f32x4, yf[0])[1];
                return c;
            } else {
                return mfma16_x6<NP>(xf, yf, c);
            }
        };
        auto getx = [&](const char* Xs, int off, bf16x8 (&f)[3]) {
            if constexpr (DBG != 5) IX::template get<NP>(Xs, off, f);
        };
        auto gety = [&](const char* Ys, int off, bf16x8 (&f)[3]) {
            if constexpr (DBG != 5) IY::template get<NP>(Ys, off, f);
        };
        bf16x8 yb[MY][3], xa[2][3];
        if constexpr (DBG == 5) {
            const uint32_t k = 0x3f803f80u ^ (uint32_t)lane;
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                xa[0][p] = xa[1][p] = as_bf16x8(make_uint4(k, k, k, k));
#pragma unroll
                for (int y = 0; y < MY; ++y) yb[y][p] = as_bf16x8(make_uint4(k, k + 1, k, k));
            }
        }
        for (int t = 0; t < T; ++t) {
            const char* Xs = buf(t & 1);
            const char* Ys = Xs + W::IMX;
            getx(Xs, ox[0], xa[0]);
            gety(Ys, oy[0], yb[0]);
#pragma unroll
            for (int y = 0; y < MY; ++y) {
                if (y + 1 < MY) gety(Ys, oy[y + 1], yb[y + 1]);
                else getx(Xs, ox[1], xa[1]);
                __builtin_amdgcn_sched_barrier(0);
                acc[0][y] = mm(xa[0], yb[y], acc[0][y]);
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int x = 1; x < MX; ++x) {
                if (x + 1 < MX) getx(Xs, ox[x + 1], xa[(x + 1) & 1]);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int y = 0; y < MY; ++y) acc[x][y] = mm(xa[x & 1], yb[y], acc[x][y]);
                __builtin_amdgcn_sched_barrier(0);
            }
            __syncthreads();
        }
        float* out = a.slab + (int64_t)bid * KXP * NYP;
#pragma unroll
        for (int x = 0; x < MX; ++x)
#pragma unroll
            for (int y = 0; y < MY; ++y)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    out[(int64_t)(16 * (MX * wx + x) + 4 * kq + r) * NYP + 16 * (MY * wy + y) + c16] = acc[x][y][r];
        return;
    }
    // ---------------- staging waves ----------------
    // chunk-major operands: thread = row rr, column groups c0 + 8k; row-major Y: 8 threads per row
    // (row yr = st >> 3, groups (st & 7) + 8k: 128 contiguous bytes per 8 lanes)
    const int st = tid - 256, rr = st & 31, c0 = st >> 5;
    const int yr = YROW ? (st >> 3) & 31 : rr, yc0 = YROW ? (st & 7) : c0;
    const int swave = __builtin_amdgcn_readfirstlane(st >> 6);
    int offx[W::NKX], offy[W::NKY];
#pragma unroll
    for (int k = 0; k < W::NKX; ++k) {
        const int c4 = c0 + 8 * k;
        offx[k] = c4 < W::GX ? cm_offk<W::KHX>(0, 4 * c4) : 0;
    }
#pragma unroll
    for (int k = 0; k < W::NKY; ++k) {
        const int c4 = yc0 + 8 * k;
        offy[k] = YROW ? 4 * c4 : (c4 < W::GY ? cm_offk<W::KHY>(0, 4 * c4) : 0);
    }
    // wave-uniform: does this staging wave own a real group at slot k (c0 = 2·swave + {0, 1})
    auto xk_ok = [&](int k) { return 2 * swave + 8 * k < W::GX; };
    auto yk_ok = [&](int k) { return YROW ? true : 2 * swave + 8 * k < W::GY; };
    const int ones_k = a.x_ones >= 0 && ((a.x_ones >> 2) & 7) == c0 ? (a.x_ones >> 5) : -1;
    const int ones_c = a.x_ones & 3;
    float4 w0r[XD ? W::NKX : 1], w1r[XD ? W::NKX : 1], b0r[XD ? W::NKX : 1];
    if (XD) {
#pragma unroll
        for (int k = 0; k < W::NKX; ++k) {
            const int f = 4 * (c0 + 8 * k);
            const bool ok = c0 + 8 * k < W::GX;
            w0r[k] = ok ? *reinterpret_cast<const float4*>(a.w0 + f) : f4zero();
            w1r[k] = ok ? *reinterpret_cast<const float4*>(a.w0 + KXP + f) : f4zero();
            b0r[k] = ok ? *reinterpret_cast<const float4*>(a.b0 + f) : f4zero();
        }
    }
    // the stage (s, nb) of the next fetch, advanced by one per call: fetch runs t = 0, 1, 2, … in order
    // and the tail re-fetches stage T − 1. (A 64-bit division per stage was ≈ 130 scalar instructions
    // in the staging wave's stream.)
    int64_t fs = t0 / a.nbs, fnb = t0 - fs * a.nbs;
    int fdone = 0;
    // operand loads as buffer loads: a stage's block base is wave-uniform (a descriptor built by the
    // scalar unit), each lane's 32-bit offset within the block is fixed for the whole loop — no 64-bit
    // address arithmetic per load on the staging wave's vector stream
    constexpr int XEB = (B16 & kB16X) ? 2 : 4, YEB = (B16 & kB16Y) ? 2 : 4;   // bytes per element
    int vox[W::NKX], voy[W::NKY];
#pragma unroll
    for (int k = 0; k < W::NKX; ++k) vox[k] = (rr * 4 + offx[k]) * XEB;
#pragma unroll
    for (int k = 0; k < W::NKY; ++k) voy[k] = (YROW ? yr * 160 + offy[k] : rr * 4 + offy[k]) * YEB;
    auto rsrc = [](const void* p, int bytes) {
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, bytes, 0x00020000);
    };
    auto fetch = [&](int t, WsSet4& R) {
        if constexpr (DBG == 1 || DBG == 6) {   // diagnosis: no global loads
            const float c = (float)(rr + t);
            R.nvalid = 32;
            R.d = make_float2(c, c + 1.f);
#pragma unroll
            for (int k = 0; k < W::NKX; ++k) R.x[k] = make_float4(c, c + 1.f, c + 2.f, c + 3.f);
#pragma unroll
            for (int k = 0; k < W::NKY; ++k) R.y[k] = make_float4(c, c - 1.f, c - 2.f, c - 3.f);
            return;
        }
        const int64_t s = fs, nb = fnb;   // stage t0 + min(t, T − 1)
        if (fdone < T - 1) {
            ++fdone;
            if (++fnb == a.nbs) {
                fnb = 0;
                ++fs;
            }
        }
        if (MASK) R.nvalid = (int)min<int64_t>(32, a.count - nb * 32);
        if constexpr (DBG == 0) {
            // stage blocks: bf16 storage keeps the fp32 step starts (the producers write through
            // per-step pointers), elements within a step at 2 bytes
            const int64_t bx = (s * a.x_sb + nb) * (W::KHX * 64), sx = s * a.x_sb * (W::KHX * 64);
            const int64_t by = YROW ? (s * a.y_sb + nb) * (32 * 160) : (s * a.y_sb + nb) * (W::KHY * 64);
            const int64_t sy = YROW ? 0 : s * a.y_sb * (W::KHY * 64);
            if (XD == 1) {
                R.d = a.xd[(s * a.x_sb + nb) * 32 + rr];
            } else if (XD == 2) {
                const float4 p = a.xp[min<int64_t>((s * a.x_sb + nb) * 32 + rr, a.count - 1)];
                R.d = make_float2(p.y, p.z);   // Networks.py:65-71: (y, width)
            } else {
                const auto rx = rsrc(reinterpret_cast<const char*>(a.x + sx) + (bx - sx) * XEB, W::KHX * 64 * XEB);
#pragma unroll
                for (int k = 0; k < W::NKX; ++k) {
                    if constexpr (XEB == 2) {
                        const auto u = __builtin_amdgcn_raw_buffer_load_b64(rx, vox[k], 0, 0);
                        const uint2 w = make_uint2(u[0], u[1]);
                        if constexpr (kRawX) R.xh[k] = w;
                        else R.x[k] = unpack4_bf16(w);
                    } else {
                        const auto u = __builtin_amdgcn_raw_buffer_load_b128(rx, vox[k], 0, 0);
                        R.x[k] = make_float4(__uint_as_float(u[0]), __uint_as_float(u[1]), __uint_as_float(u[2]), __uint_as_float(u[3]));
                    }
                }
            }
            const auto ry = rsrc(reinterpret_cast<const char*>(a.y + sy) + (by - sy) * YEB, (YROW ? 32 * 160 : W::KHY * 64) * YEB);
#pragma unroll
            for (int k = 0; k < W::NKY; ++k) {
                if constexpr (YEB == 2) {
                    const auto u = __builtin_amdgcn_raw_buffer_load_b64(ry, voy[k], 0, 0);
                    const uint2 w = make_uint2(u[0], u[1]);
                    if constexpr (kRawY) R.yh[k] = w;
                    else R.y[k] = unpack4_bf16(w);
                } else {
                    const auto u = __builtin_amdgcn_raw_buffer_load_b128(ry, voy[k], 0, 0);
                    R.y[k] = make_float4(__uint_as_float(u[0]), __uint_as_float(u[1]), __uint_as_float(u[2]), __uint_as_float(u[3]));
                }
            }
            return;
        }
        const int64_t ix = (s * a.x_sb + nb) * (W::KHX * 64) + rr * 4;   // element indices
        const int64_t iy = YROW ? ((s * a.y_sb + nb) * 32 + yr) * 160 : (s * a.y_sb + nb) * (W::KHY * 64) + rr * 4;
        const float* px = a.x + ix;
        const float* py = a.y + iy;
        // bf16 storage: a per-step array's step s starts where its fp32 step starts (the producers write
        // through per-step pointers), the element index runs within the step
        const int64_t sx = s * a.x_sb * (W::KHX * 64), sy = YROW ? 0 : s * a.y_sb * (W::KHY * 64);
        const uint16_t* hx = reinterpret_cast<const uint16_t*>(a.x + sx) + (ix - sx);
        const uint16_t* hy = reinterpret_cast<const uint16_t*>(a.y + sy) + (iy - sy);
        if (XD == 1) {
            R.d = a.xd[(s * a.x_sb + nb) * 32 + rr];
        } else if (XD == 2) {
            const float4 p = a.xp[min<int64_t>((s * a.x_sb + nb) * 32 + rr, a.count - 1)];
            R.d = make_float2(p.y, p.z);   // Networks.py:65-71: (y, width)
        } else {
#pragma unroll
            for (int k = 0; k < W::NKX; ++k) {
                if constexpr (kRawX) R.xh[k] = *reinterpret_cast<const uint2*>(hx + offx[k]);
                else if constexpr (B16 & kB16X) R.x[k] = unpack4_bf16(*reinterpret_cast<const uint2*>(hx + offx[k]));
                else R.x[k] = *reinterpret_cast<const float4*>(px + offx[k]);
            }
        }
#pragma unroll
        for (int k = 0; k < W::NKY; ++k) {
            if constexpr (kRawY) R.yh[k] = *reinterpret_cast<const uint2*>(hy + offy[k]);
            else if constexpr (B16 & kB16Y) R.y[k] = unpack4_bf16(*reinterpret_cast<const uint2*>(hy + offy[k]));
            else R.y[k] = *reinterpret_cast<const float4*>(py + offy[k]);
        }
    };
    uint32_t dbg_sink = 0u;
    // diagnosis forms of the image writes: raw bits into the parts (no split), or no LDS writes
    auto putx = [&](char* S, int row, int c4, float4 v) {
        if constexpr (DBG == 2) {
            char* p = S + IX::woff(row, c4);
            const uint2 u = make_uint2(__float_as_uint(v.x) ^ __float_as_uint(v.y), __float_as_uint(v.z) ^ __float_as_uint(v.w));
            *reinterpret_cast<uint2*>(p) = u;
            if constexpr (NP == 3) { *reinterpret_cast<uint2*>(p + IX::PART) = u; *reinterpret_cast<uint2*>(p + 2 * IX::PART) = u; }
        } else if constexpr (DBG == 3) {
            uint32_t h0, m0, l0, h1, m1, l1;
            split2(v.x, v.y, h0, m0, l0);
            split2(v.z, v.w, h1, m1, l1);
            dbg_sink ^= h0 ^ h1 ^ (NP == 3 ? (m0 ^ l0 ^ m1 ^ l1) : 0u);
        } else {
            IX::template put<NP>(S, row, c4, v);
        }
    };
    auto puty = [&](char* S, int row, int c4, float4 v) {
        if constexpr (DBG == 2) {
            char* p = S + IY::woff(row, c4);
            const uint2 u = make_uint2(__float_as_uint(v.x) ^ __float_as_uint(v.y), __float_as_uint(v.z) ^ __float_as_uint(v.w));
            *reinterpret_cast<uint2*>(p) = u;
            if constexpr (NP == 3) { *reinterpret_cast<uint2*>(p + IY::PART) = u; *reinterpret_cast<uint2*>(p + 2 * IY::PART) = u; }
        } else if constexpr (DBG == 3) {
            uint32_t h0, m0, l0, h1, m1, l1;
            split2(v.x, v.y, h0, m0, l0);
            split2(v.z, v.w, h1, m1, l1);
            dbg_sink ^= h0 ^ h1 ^ (NP == 3 ? (m0 ^ l0 ^ m1 ^ l1) : 0u);
        } else {
            IY::template put<NP>(S, row, c4, v);
        }
    };
    // the bias' ones column: its group slot is wave-uniform (a scalar branch per slot), its lane set
    // is not — one select per stage instead of one per slot and component
    const int ones_kk = a.x_ones >= 0 ? (a.x_ones >> 5) : -1;
    const bool ones_lane = ones_k >= 0;
    // row masks only on a job's last, partial row block (wave-uniform): full stages take no selects
    auto build_m = [&](const WsSet4& R, char* Xs, auto Mc) {
        constexpr bool M = MASK && decltype(Mc)::value;
        char* Ys = Xs + W::IMX;
        const bool xin = !M || rr < R.nvalid, yin = !M || yr < R.nvalid;
#pragma unroll
        for (int k = 0; k < W::NKX; ++k) {
            if (!xk_ok(k)) break;
            if constexpr (kRawX) {
                uint2 u = R.xh[k];
                if (M && !xin) u = make_uint2(0u, 0u);
                if (k == ones_kk && ones_lane) {   // the bias' ones column: bf16 1.0 = 0x3f80 in half ones_c
                    uint32_t& w = (ones_c >> 1) ? u.y : u.x;
                    const int sh = 16 * (ones_c & 1);
                    w = (w & ~(0xffffu << sh)) | ((xin ? 0x3f80u : 0u) << sh);
                }
                *reinterpret_cast<uint2*>(Xs + IX::woff(rr, c0 + 8 * k)) = u;
                continue;
            }
            float4 v;
            if (XD) {
                v.x = relu(dense2(R.d.x, R.d.y, w0r[k].x, w1r[k].x, b0r[k].x));
                v.y = relu(dense2(R.d.x, R.d.y, w0r[k].y, w1r[k].y, b0r[k].y));
                v.z = relu(dense2(R.d.x, R.d.y, w0r[k].z, w1r[k].z, b0r[k].z));
                v.w = relu(dense2(R.d.x, R.d.y, w0r[k].w, w1r[k].w, b0r[k].w));
            } else {
                v = R.x[k];
            }
            if (M && !xin) v = f4zero();
            if (k == ones_kk) {
                if (ones_lane) f4set(v, ones_c, xin ? 1.f : 0.f);
            }
            putx(Xs, rr, c0 + 8 * k, v);
        }
#pragma unroll
        for (int k = 0; k < W::NKY; ++k) {
            if (!yk_ok(k)) break;
            if constexpr (kRawY) {
                uint2 u = R.yh[k];
                if (M && !yin) u = make_uint2(0u, 0u);
                *reinterpret_cast<uint2*>(Ys + IY::woff(yr, yc0 + 8 * k)) = u;
                continue;
            }
            float4 v = R.y[k];
            if (M && !yin) v = f4zero();
            puty(Ys, yr, yc0 + 8 * k, v);
        }
    };
    auto build = [&](const WsSet4& R, char* Xs) {
        if constexpr (DBG == 6) return;
        if (MASK && R.nvalid < 32) build_m(R, Xs, std::true_type{});
        else build_m(R, Xs, std::false_type{});
    };
    if (T == 0) {
        __syncthreads();
        return;
    }
    // padding column groups (≥ GX / GY, below the image width) stay zero in both buffers
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
        for (int k = 0; k < (KXP / 4 + 7) / 8; ++k) {
            const int c4 = c0 + 8 * k;
            if (c4 >= W::GX && c4 < KXP / 4) IX::template put<NP>(buf(p), rr, c4, f4zero());
        }
        if (!YROW) {
#pragma unroll
            for (int k = 0; k < (NYP / 4 + 7) / 8; ++k) {
                const int c4 = c0 + 8 * k;
                if (c4 >= W::GY && c4 < NYP / 4) IY::template put<NP>(buf(p) + W::IMX, rr, c4, f4zero());
            }
        }
    }
    // NS stage sets in flight: at (sub-)iteration u the staging waves stream stage u + NS into set
    // u % NS (its stage u was built one iteration ago) and build stage u + 1 into buffer (u + 1) & 1,
    // so a stage's loads are issued NS − 1 iterations before their split (static set names: the
    // loop is unrolled by NS)
    constexpr int NS = NP == 1 ? SPWGNN_WS_NSET_B16 : SPWGNN_WS_NSET;
    WsSet4 R[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) fetch(k, R[k]);
    build(R[0], buf(0));
    __syncthreads();
    int t = 0;
    for (; t + NS <= T - 1; t += NS) {
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            fetch(t + k + NS, R[k]);
            build(R[(k + 1) % NS], buf((t + k + 1) & 1));
            __syncthreads();
        }
    }
#pragma unroll
    for (int k = 1; k < NS; ++k) {   // t ≡ 0 (mod NS) here: stage t + k sits in set k
        if (t < T - 1) {
            build(R[k], buf((t + 1) & 1));
            __syncthreads();
            ++t;
        }
    }
    if constexpr (DBG == 3) {   // keep the diagnosis split alive
        if (dbg_sink == 0x9e3779b9u) a.slab[0] = 0.f;
    }
    __syncthreads();
}

template <int KXP, int NYP, int YROW, bool MASK, int NP = 3, int XD = 0, int B16 = 0>
__global__ __launch_bounds__(kWsThreads, 1) __attribute__((amdgpu_waves_per_eu(2, 2)))
void k_wgrad_ws(WgWsArgs a) {
    __shared__ __attribute__((aligned(16))) char buf[2 * WsStage<KXP, NYP, YROW, MASK>::BUF];
    wgrad_ws_body<KXP, NYP, YROW, MASK, NP, XD, B16>(a, blockIdx.x, buf);
}

// Every stored-operand weight gradient of a backward in ONE launch: workgroup b runs job k's
// workgroup b − wg0[k] (job ranges in order; the job and its variant are workgroup-uniform). At the
// reference's batch 32 each gradient is a few workgroups of one or two stages, so eleven launches
// cost their ramp-up eleven times; batched they overlap.
constexpr int kWsMaxBuf = WsStage<160, 160, 0, false>::BUF;
template <int KH, bool NODE, bool B16>
__device__ __forceinline__ void wgrad_pos3_body(const Pos3Args& a, int bid, int tid);
// A small batch's rm.0 / om.0 gradients (k_wgrad_pos3) ride in the same launch: workgroups from
// b.wgs on run two of k_wgrad_pos3's 256-thread workgroups each (one per half), beside the jobs.
// ... and so does its W2 gradient (k_w2grad_ws, x6): the last b.w2_wgs workgroups.
static_assert(2 * kWsMaxBuf >= 2 * 2 * kW2gImg && kWsThreads == kW2gThreads, "W2 gradient in the batched launch");
template <int NP>
__global__ __launch_bounds__(kWsThreads, 1) __attribute__((amdgpu_waves_per_eu(2, 2)))
void k_wgrad_ws_batch(WsBatch b, Pos3Batch p3) {
    __shared__ __attribute__((aligned(16))) char smem[2 * kWsMaxBuf];
    const int w2_first = (int)gridDim.x - b.w2_wgs;
    if (NP == 3 && (int)blockIdx.x >= w2_first) {
        w2grad_ws_body<0, 3, false>(b.w2, b.w2_bpw, (int)blockIdx.x - w2_first, reinterpret_cast<char (*)[2 * kW2gImg]>(smem));
        return;
    }
    if ((int)blockIdx.x >= b.wgs) {
        const int q = 2 * ((int)blockIdx.x - b.wgs) + (int)(threadIdx.x >> 8), tid = threadIdx.x & 255;
        if (q < p3.ce) {
            if (p3.b16e) wgrad_pos3_body<kKhE, false, true>(p3.e, q, tid);
            else wgrad_pos3_body<kKhE, false, false>(p3.e, q, tid);
        } else if (q < p3.ce + p3.cn) {
            wgrad_pos3_body<kKhN, true, false>(p3.n, q - p3.ce, tid);
        }
        return;
    }
    int k = 0;
    while (k + 1 < b.n && (int)blockIdx.x >= b.j[k + 1].wg0) ++k;
    int bid = (int)blockIdx.x - b.j[k].wg0;
    if (b.j[k].gn > 1) {
        // an operand-sharing group of G jobs with the same row ranges (ws_group): slot q of the group
        // runs job q/8 mod G on its workgroup (q/8/G)·8 + q mod 8, so the G workgroups of one row
        // range sit 8 slots apart — on one XCD (workgroups go round-robin over the 8 XCDs) at the
        // same time, and the shared operand's rows come from that XCD's L2 after the first read
        const int first = k - b.j[k].gi, G = b.j[k].gn;
        const int q = (int)blockIdx.x - b.j[first].wg0, r = q >> 3;
        k = first + r % G;
        bid = (r / G) * 8 + (q & 7);
    }
    const WsJob& job = b.j[k];
    switch (job.variant) {
        case WSV_160_160: wgrad_ws_body<160, 160, 0, false, NP, 0, 0>(job.a, bid, smem); break;
        case WSV_160_160_ROW: wgrad_ws_body<160, 160, 1, false, NP, 0, 0>(job.a, bid, smem); break;
        case WSV_128_160: wgrad_ws_body<128, 160, 0, true, NP, 0, 0>(job.a, bid, smem); break;
        case WSV_160_128: wgrad_ws_body<160, 128, 0, true, NP, 0, 0>(job.a, bid, smem); break;
        case WSV_128_128: wgrad_ws_body<128, 128, 0, true, NP, 0, 0>(job.a, bid, smem); break;
        case WSV_XD_EDGE: wgrad_ws_body<160, 160, 0, false, NP, 1, 0>(job.a, bid, smem); break;
        case WSV_XD_NODE: wgrad_ws_body<128, 128, 0, true, NP, 2, 0>(job.a, bid, smem); break;
        default:
            if constexpr (NP == 1) {   // bf16 math's bf16-stored edge operands (§3g)
                switch (job.variant) {
                    case WSV_XD_EDGE_B16Y: wgrad_ws_body<160, 160, 0, false, 1, 1, kB16Y>(job.a, bid, smem); break;
                    case WSV_160_160_ROW_B16: wgrad_ws_body<160, 160, 1, false, 1, 0, kB16X | kB16Y>(job.a, bid, smem); break;
                    case WSV_160_160_B16: wgrad_ws_body<160, 160, 0, false, 1, 0, kB16X | kB16Y>(job.a, bid, smem); break;
                    case WSV_128_160_B16Y: wgrad_ws_body<128, 160, 0, true, 1, 0, kB16Y>(job.a, bid, smem); break;
                    case WSV_160_128_B16: wgrad_ws_body<160, 128, 0, true, 1, 0, kB16X | kB16Y>(job.a, bid, smem); break;
                    case WSV_128_128_B16: wgrad_ws_body<128, 128, 0, true, 1, 0, kB16X | kB16Y>(job.a, bid, smem); break;
                    default: break;
                }
            }
            break;
    }
}

// dW = Σ_c slab[c] in a fixed order (deterministic), scattered into the Keras tensors (kernel rows,
// bias row, omp.1 column permutation); blockIdx.y selects the weight gradient of the batch. A
// workgroup takes 32 elements × 8 chunk groups: thread (e, g) sums chunks g, g+8, … (four interleaved
// sums), then the 8 partial sums meet in LDS — a 256-chunk gradient is 8 dependent load rounds per
// thread instead of 64 (the reduction was latency-bound: 66 µs at config 2, 74 µs at the headline).
__device__ __forceinline__ void bce_block_final(const BceArgs& a);
__global__ __launch_bounds__(256) void k_wgrad_reduce_all(ReduceBatch rb) {
    __shared__ float part[8][32];
    if (rb.bce_row && blockIdx.y == gridDim.y - 1) {   // spwgnn_bce_backward: the loss sums
        if (blockIdx.x == 0) bce_block_final(rb.bce);
        return;
    }
    if ((int)blockIdx.y == rb.n) {   // the ranges no reduction writes: zeros
        for (int z = 0; z < rb.nzero; ++z)
            for (int e = blockIdx.x * 256 + threadIdx.x; e < rb.zlen[z]; e += gridDim.x * 256) rb.r[0].out[rb.zoff[z] + e] = 0.f;
        return;
    }
    const ReduceArgs& a = rb.r[blockIdx.y];
    const int e = threadIdx.x & 31, g = threadIdx.x >> 5;
    const int idx = blockIdx.x * 32 + e;
    const int k = idx / a.ny_pad, n = idx - k * a.ny_pad;
    const int col = a.perm ? wo2_perm(n) : n;
    const bool kern = a.kernel_off >= 0 && k < a.kernel_rows, bias = a.bias_off >= 0 && k == a.bias_row;
    const bool ok = idx < a.kx_pad * a.ny_pad && col >= 0 && col < a.kernel_cols && (kern || bias);
    const int64_t stride = (int64_t)a.kx_pad * a.ny_pad;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    if (ok) {
        const float* p = a.slab + idx;
        int c = g;
        for (; c + 24 < a.chunks; c += 32) {
            s0 += p[(c + 0) * stride];
            s1 += p[(c + 8) * stride];
            s2 += p[(c + 16) * stride];
            s3 += p[(c + 24) * stride];
        }
        for (; c < a.chunks; c += 8) s0 += p[c * stride];
    }
    part[g][e] = (s0 + s1) + (s2 + s3);
    __syncthreads();
    if (g != 0 || !ok) return;
    const float s = ((part[0][e] + part[1][e]) + (part[2][e] + part[3][e])) +
                    ((part[4][e] + part[5][e]) + (part[6][e] + part[7][e]));
    if (kern) a.out[a.kernel_off + (int64_t)(a.kernel_row0 + k) * a.kernel_cols + col] = s;
    if (bias) a.out[a.bias_off + col] = s;
}

// ------------------------------------------------------------------------------------------------
// Keras binary_crossentropy (Networks.py:102): kLogitClip and bce_dlogit in kernels.h.

// FINAL (a.blocks == 1, e.g. the reference's batch 32): the one workgroup also writes out3, the
// same double-precision division k_bce_final does over its one partial — one launch instead of two.
// With a.tot3 the thread that writes out3 also adds it into the epoch sums (k_accumulate_out3's
// arithmetic on the same float values).
__device__ inline void bce_store_out3(const BceArgs& a, float loss, float correct) {
    const float o[3] = {loss, correct, (float)a.n};
    for (int k = 0; k < 3; ++k) {
        a.out3[k] = o[k];
        if (a.tot3) a.tot3[k] += (double)o[k] * a.w3[k];
    }
}

// one workgroup (256 threads, `blk` of a.blocks) of the loss: k_bce_partial, and the extra row of the
// gradient reductions under spwgnn_bce_backward
template <bool FINAL>
__device__ __forceinline__ void bce_block(const BceArgs& a, int blk) {
    __shared__ float sl[256], sc[256];
    float ls = 0.f, cs = 0.f;
    const float inv_n = 1.0f / (float)a.n;
    for (int64_t i = (int64_t)blk * 256 + threadIdx.x; i < a.n; i += (int64_t)a.blocks * 256) {
        const float z0 = a.logits[i], t = a.targets[i];
        const float z = fminf(fmaxf(z0, -kLogitClip), kLogitClip);
        ls += fmaxf(z, 0.f) - z * t + log1pf(expf(-fabsf(z)));
        const float p = 1.f / (1.f + expf(-z0));
        cs += ((p > 0.5f ? 1.f : 0.f) == t) ? 1.f : 0.f;
        if (a.dlogits) a.dlogits[i] = bce_dlogit(z0, t, inv_n);
    }
    sl[threadIdx.x] = ls;
    sc[threadIdx.x] = cs;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) {
            sl[threadIdx.x] += sl[threadIdx.x + o];
            sc[threadIdx.x] += sc[threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        if constexpr (FINAL) {
            bce_store_out3(a, (float)((double)sl[0] / (double)a.n), (float)(double)sc[0]);
        } else {
            a.partial[2 * blk] = sl[0];
            a.partial[2 * blk + 1] = sc[0];
        }
    }
}
template <bool FINAL>
__global__ __launch_bounds__(256) void k_bce_partial(BceArgs a) {
    bce_block<FINAL>(a, blockIdx.x);
}
__device__ __forceinline__ void bce_block_final(const BceArgs& a) { bce_block<true>(a, 0); }

__global__ void k_bce_final(BceArgs a) {
    if (threadIdx.x != 0) return;
    double ls = 0.0, cs = 0.0;
    for (int b = 0; b < a.blocks; ++b) {
        ls += a.partial[2 * b];
        cs += a.partial[2 * b + 1];
    }
    bce_store_out3(a, (float)(ls / (double)a.n), (float)cs);
}

__global__ void k_adam(AdamArgs a) {
    // replayable steps: the step count lives on the device; lr_t comes from the host-built table
    // (spwgnn_adam_lr_table: the same expression spwgnn_adam evaluates, so both paths agree bitwise)
    if (a.step_dev) a.lr_t = a.lr_table[min(max(*a.step_dev, 0), a.table_len - 1)];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
        const float p = a.p[i];
        const float g = a.gscale * a.g[i] + 2.f * a.l2 * p;
        const float m = a.b1 * a.m[i] + (1.f - a.b1) * g;
        const float v = a.b2 * a.v[i] + (1.f - a.b2) * g * g;
        a.m[i] = m;
        a.v[i] = v;
        a.p[i] = p - a.lr_t * m / (sqrtf(v) + a.eps);
    }
}

// Start of a replayable training step (one thread, device_common.h step_advance_dev).
__global__ void k_step_advance(uint64_t* key, int32_t* step, int mode, uint64_t seed, int32_t rank) {
    if (threadIdx.x == 0) step_advance_dev(key, step, mode, seed, rank);
}

__global__ void k_sigmoid(const float* z, float* p, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = 1.f / (1.f + expf(-z[i]));
}

// per-tower readout (one thread per tower, node order): modes as SPWGNN_READOUT_*
__global__ void k_tower_readout(const float* __restrict__ z, const int32_t* __restrict__ off, int n_towers, int mode,
                                float* __restrict__ out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_towers) return;
    const int b = off[t], e = off[t + 1];
    float s = 0.f;
    for (int n = b; n < e; ++n) s += (mode <= 1) ? 1.f / (1.f + expf(-z[n])) : z[n];
    out[t] = ((mode & 1) && e > b) ? s / (float)(e - b) : s;
}

// ------------------------------------------------------------------------------------------------
// The two first-layer gradients whose X has three columns (rm.0: X = [pos[dst] − pos[src] | 1],
// padding edge → 0; om.0: X = [pos[n].y, pos[n].z | 1], rows ≥ count → 0), in the split-bf16 maths:
// dW[k][f] = Σ_rows X[row][k]·Y[row][f] is a 3-column contraction — 6 FLOPs per Y element against
// 4 (2 in bf16 storage) bytes of it, far below the ridge point, so it runs on the vector ALUs as a
// stream over Y (exact fp32 fmas, no split) instead of padded 32-row MFMA tiles behind two barriers
// per 32-row stage (k_wgrad_x6: config 3's rm.0 gradient 1.3 ms at 2 TB/s). A workgroup owns a
// contiguous range of 32-row blocks; thread (row i = tid & 31, piece g = tid >> 5) keeps the three
// sums of chunk-major pieces g, g + 8, ... of row i over the range (fixed order), the 32 rows of a
// piece are summed across the half-wave in a fixed butterfly, and the slab rows 0-2 (kernel rows d0,
// d1 / y, w and the bias row) go to this workgroup's chunk for k_wgrad_reduce_all. Pieces past the
// row's last one (qh ≥ NQH) re-read the last piece and are never written out.
template <int KH, bool NODE, bool B16>
__device__ __forceinline__ void wgrad_pos3_body(const Pos3Args& a, int bid, int tid) {
    constexpr int NQH = KH / 2, NK = (NQH + 7) / 8, NYP = KH == kKhE ? 160 : 128, BLK = KH * 64;
    // blocks whose loads are issued together (the loop is latency-bound): bf16 rows are half the bytes
    // per load, so twice the blocks keep the same bytes in flight
    constexpr int UB = B16 ? 8 : 4;
    const int i = tid & 31, g = tid >> 5;
    const int64_t b0 = (int64_t)bid * a.blk_per_wg, b1 = min(a.nblk, b0 + a.blk_per_wg);
    float4 s0[NK], s1[NK], s2[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) s0[k] = s1[k] = s2[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t bg = b0; bg < b1; bg += UB) {
        float x0[UB], x1[UB], x2[UB];
        float4 y[UB][NK];
        uint2 yh[UB][NK];   // B16: the stored pairs, unpacked at their fmas
#pragma unroll
        for (int u = 0; u < UB; ++u) {
            const bool in = bg + u < b1;
            const int64_t b = in ? bg + u : b1 - 1;
            const int64_t row = b * 32 + i;
            bool ok;
            if constexpr (NODE) {
                ok = in && row < a.count;
                const float4 p = a.pos[ok ? row : 0];
                x0[u] = ok ? p.y : 0.f;
                x1[u] = ok ? p.z : 0.f;
                x2[u] = ok ? 1.f : 0.f;
            } else {   // d from the encoder's stored per-edge (dx, dy): no dependent gathers
                ok = in && a.esrc[row] >= 0;
                const float2 d = a.ed[row];
                x0[u] = ok ? d.x : 0.f;
                x1[u] = ok ? d.y : 0.f;
                x2[u] = ok ? 1.f : 0.f;
            }
#pragma unroll
            for (int k = 0; k < NK; ++k) {
                const int qh = min(g + 8 * k, NQH - 1);
                const int64_t el = b * BLK + (qh * 32 + i) * 4;
                // rows past the batch are not written by every producer (the fused small-batch
                // kernels store only their towers' rows): 0·NaN must not reach the sums
                if constexpr (B16) {
                    yh[u][k] = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(a.y) + el);
                    if (!ok) yh[u][k] = make_uint2(0u, 0u);
                } else {
                    y[u][k] = *reinterpret_cast<const float4*>(a.y + el);
                    if (!ok) y[u][k] = make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < UB; ++u)
#pragma unroll
            for (int k = 0; k < NK; ++k) {
                const float4 v = B16 ? unpack4_bf16(yh[u][k]) : y[u][k];
                s0[k] = make_float4(__builtin_fmaf(x0[u], v.x, s0[k].x), __builtin_fmaf(x0[u], v.y, s0[k].y),
                                    __builtin_fmaf(x0[u], v.z, s0[k].z), __builtin_fmaf(x0[u], v.w, s0[k].w));
                s1[k] = make_float4(__builtin_fmaf(x1[u], v.x, s1[k].x), __builtin_fmaf(x1[u], v.y, s1[k].y),
                                    __builtin_fmaf(x1[u], v.z, s1[k].z), __builtin_fmaf(x1[u], v.w, s1[k].w));
                s2[k] = make_float4(__builtin_fmaf(x2[u], v.x, s2[k].x), __builtin_fmaf(x2[u], v.y, s2[k].y),
                                    __builtin_fmaf(x2[u], v.z, s2[k].z), __builtin_fmaf(x2[u], v.w, s2[k].w));
            }
    }
    auto hsum = [&](float v) {   // the 32 rows of this half-wave, fixed butterfly
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 32);
        return v;
    };
    float* out = a.slab + (int64_t)bid * 32 * NYP;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
        const int qh = g + 8 * k;
        if (qh >= NQH) continue;   // uniform per half-wave
        const float4 r0 = make_float4(hsum(s0[k].x), hsum(s0[k].y), hsum(s0[k].z), hsum(s0[k].w));
        const float4 r1 = make_float4(hsum(s1[k].x), hsum(s1[k].y), hsum(s1[k].z), hsum(s1[k].w));
        const float4 r2 = make_float4(hsum(s2[k].x), hsum(s2[k].y), hsum(s2[k].z), hsum(s2[k].w));
        if (i == 0) {
            const int f = KH * (qh & 1) + 4 * (qh >> 1);   // features f .. f+3 (chunk-major piece qh)
            *reinterpret_cast<float4*>(out + f) = r0;
            *reinterpret_cast<float4*>(out + NYP + f) = r1;
            *reinterpret_cast<float4*>(out + 2 * NYP + f) = r2;
        }
    }
}
// rm.0 (edge rows) and om.0 (node rows) in one launch: workgroups [0, ce) take the edge job
template <bool B16E>
__global__ __launch_bounds__(256) void k_wgrad_pos3(Pos3Args e, Pos3Args n, int ce) {
    if ((int)blockIdx.x < ce) wgrad_pos3_body<kKhE, false, B16E>(e, blockIdx.x, threadIdx.x);
    else wgrad_pos3_body<kKhN, true, false>(n, blockIdx.x - ce, threadIdx.x);
}
hipError_t launch_wgrad_pos3(const Pos3Batch& p, hipStream_t st) {
    if (p.ce + p.cn <= 0) return hipSuccess;
    const dim3 g(p.ce + p.cn), b(256);
    if (p.b16e) hipLaunchKernelGGL((k_wgrad_pos3<true>), g, b, 0, st, p.e, p.n, p.ce);
    else hipLaunchKernelGGL((k_wgrad_pos3<false>), g, b, 0, st, p.e, p.n, p.ce);
    return hipGetLastError();
}

hipError_t launch_wgrad(const WgradArgs& a, int chunks, int math, hipStream_t st) {
    const dim3 g(chunks), b(kWgThreads);
#define SPW_WG(XM, YM, KX, NY)                                                               \
    if (a.xmode == XM && a.ymode == YM && a.kx_pad == KX && a.ny_pad == NY) {                 \
        if (math == MATH_X6)                                                           \
            hipLaunchKernelGGL((k_wgrad_x6<XM, YM, KX, NY, (XM == XM_H1 || YM == YM_ROW) ? 1 : 2>), g, b, 0, st, a); \
        else                                                                                  \
            hipLaunchKernelGGL((k_wgrad_t<XM, YM, KX, NY>), g, b, 0, st, a);                  \
        return hipGetLastError();                                                             \
    }
    SPW_WG(XM_CM, YM_ROW, 160, 160)
    SPW_WG(XM_CM, YM_CM, 128, 160)
    SPW_WG(XM_CM, YM_CM, 160, 128)
    SPW_WG(XM_CM, YM_CM, 128, 128)
    SPW_WG(XM_EDGE_D, YM_CM, 32, 160)
    SPW_WG(XM_NODE_O, YM_CM, 32, 128)
    SPW_WG(XM_CM, YM_CM, 160, 160)
    SPW_WG(XM_H1, YM_DH2, 160, 160)
#undef SPW_WG
    return hipErrorInvalidValue;
}
// bf16 math: the two small position-operand gradients (the stored-operand ones run on k_wgrad_ws)
hipError_t launch_wgrad_bf16(const WgradArgs& a, int chunks, hipStream_t st, int b16) {
    const dim3 g(chunks), b(kWgThreads);
    if (a.xmode == XM_EDGE_D && a.ymode == YM_CM && a.kx_pad == 32 && a.ny_pad == 160 && b16 == kB16Y)
        hipLaunchKernelGGL((k_wgrad_x6<XM_EDGE_D, YM_CM, 32, 160, 2, 1, true>), g, b, 0, st, a);   // Y = dz1 (bf16)
    else if (b16)
        return hipErrorInvalidValue;
    else if (a.xmode == XM_EDGE_D && a.ymode == YM_CM && a.kx_pad == 32 && a.ny_pad == 160)
        hipLaunchKernelGGL((k_wgrad_x6<XM_EDGE_D, YM_CM, 32, 160, 2, 1>), g, b, 0, st, a);
    else if (a.xmode == XM_NODE_O && a.ymode == YM_CM && a.kx_pad == 32 && a.ny_pad == 128)
        hipLaunchKernelGGL((k_wgrad_x6<XM_NODE_O, YM_CM, 32, 128, 2, 1>), g, b, 0, st, a);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}
hipError_t launch_w2grad_ws(const WgradArgs& a, int wgs, int64_t blk_per_wg, int math, hipStream_t st) {
#ifdef SPWGNN_DIAG   // diagnosis variants (wrong results): see k_w2grad_ws's DBG bits
    static const int dbg = getenv("SPWGNN_W2G_DBG") ? atoi(getenv("SPWGNN_W2G_DBG")) : 0;
#else
    constexpr int dbg = 0;
#endif
    const dim3 g(wgs), b(kW2gThreads);
    if (a.uv16 && (math != MATH_BF16 || (dbg && dbg < 100))) return hipErrorInvalidValue;
    if (math == MATH_BF16) {
#ifdef SPWGNN_DIAG
        if (a.a_b16 && dbg && dbg < 100) {
            switch (dbg) {
                case 1: hipLaunchKernelGGL((k_w2grad_ws<1, 1, true>), g, b, 0, st, a, blk_per_wg); break;
                case 2: hipLaunchKernelGGL((k_w2grad_ws<2, 1, true>), g, b, 0, st, a, blk_per_wg); break;
                case 4: hipLaunchKernelGGL((k_w2grad_ws<4, 1, true>), g, b, 0, st, a, blk_per_wg); break;
                case 32: hipLaunchKernelGGL((k_w2grad_ws<32, 1, true>), g, b, 0, st, a, blk_per_wg); break;
                case 33: hipLaunchKernelGGL((k_w2grad_ws<33, 1, true>), g, b, 0, st, a, blk_per_wg); break;
                case 36: hipLaunchKernelGGL((k_w2grad_ws<36, 1, true>), g, b, 0, st, a, blk_per_wg); break;
                default: return hipErrorInvalidValue;
            }
            return hipGetLastError();
        }
#endif
        if (a.w2_tile && a.nw_max <= kW2tNodes) {   // node rows via LDS (k_w2grad_tile)
#ifdef SPWGNN_DIAG
            if (a.a_b16 && dbg >= 100) {   // the tile kernel's diagnosis variants: SPWGNN_W2G_DBG = 100 + bits
                switch (dbg - 100) {
#define W2T_CASE(d) case d: \
    if (a.uv16) hipLaunchKernelGGL((k_w2grad_tile<1, true, d, true>), g, b, 0, st, a, blk_per_wg); \
    else hipLaunchKernelGGL((k_w2grad_tile<1, true, d>), g, b, 0, st, a, blk_per_wg); \
    break;
                    W2T_CASE(1) W2T_CASE(2) W2T_CASE(4) W2T_CASE(8) W2T_CASE(16) W2T_CASE(3) W2T_CASE(6) W2T_CASE(7)
#undef W2T_CASE
                    default: return hipErrorInvalidValue;
                }
                return hipGetLastError();
            }
#endif
            if (a.a_b16 && a.uv16) hipLaunchKernelGGL((k_w2grad_tile<1, true, 0, true>), g, b, 0, st, a, blk_per_wg);
            else if (a.uv16) return hipErrorInvalidValue;
            else if (a.a_b16) hipLaunchKernelGGL((k_w2grad_tile<1, true>), g, b, 0, st, a, blk_per_wg);
            else hipLaunchKernelGGL((k_w2grad_tile<1, false>), g, b, 0, st, a, blk_per_wg);
            return hipGetLastError();
        }
        if (a.uv16) return hipErrorInvalidValue;   // bf16 U, V rows: the tile kernel only
        if (a.a_b16) hipLaunchKernelGGL((k_w2grad_ws<0, 1, true>), g, b, 0, st, a, blk_per_wg);
        else hipLaunchKernelGGL((k_w2grad_ws<0, 1>), g, b, 0, st, a, blk_per_wg);
        return hipGetLastError();
    }
    if (a.a_b16) return hipErrorInvalidValue;
    if (dbg == 0) {
        hipLaunchKernelGGL(k_w2grad_ws<0>, g, b, 0, st, a, blk_per_wg);
        return hipGetLastError();
    }
#ifdef SPWGNN_DIAG
    switch (dbg) {
        case 1: hipLaunchKernelGGL(k_w2grad_ws<1>, g, b, 0, st, a, blk_per_wg); break;
        case 4: hipLaunchKernelGGL(k_w2grad_ws<4>, g, b, 0, st, a, blk_per_wg); break;
        case 8: hipLaunchKernelGGL(k_w2grad_ws<8>, g, b, 0, st, a, blk_per_wg); break;
        case 33: hipLaunchKernelGGL(k_w2grad_ws<33>, g, b, 0, st, a, blk_per_wg); break;
        default: return hipErrorInvalidValue;
    }
#endif
    return hipGetLastError();
}
int wgrad_ws_variant(const WgWsArgs& a, int kx_pad, int ny_pad, int yrow, int mask, int math, int b16) {
    if (b16 && math != MATH_BF16) return WSV_NONE;
    if (a.xd) {   // the rm.1 gradient with X = [z1 | 1] rebuilt from (dx, dy)
        if (kx_pad != 160 || ny_pad != 160 || yrow || mask) return WSV_NONE;
        if (b16 == kB16Y) return WSV_XD_EDGE_B16Y;
        return b16 ? WSV_NONE : WSV_XD_EDGE;
    }
    if (a.xp) {   // the om.1 gradient with X = [zo1 | 1] rebuilt from the node positions
        if (kx_pad != 128 || ny_pad != 128 || yrow || !mask || b16) return WSV_NONE;
        return WSV_XD_NODE;
    }
    if (b16) {   // the encoder-side edge operands of bf16 math (rm.2, rm.3: X, Y; W1a: X = c_r, Y = dA rows)
        if (kx_pad == 160 && ny_pad == 160 && !mask && b16 == (kB16X | kB16Y))
            return yrow ? WSV_160_160_ROW_B16 : WSV_160_160_B16;
        // node side (§3g): W1b/W1c (Y = dU/dV), W3 (X = H2s, Y = g), omp.1 (X = o1, Y = dx)
        if (!yrow && mask) {
            if (kx_pad == 128 && ny_pad == 160 && b16 == kB16Y) return WSV_128_160_B16Y;
            if (kx_pad == 160 && ny_pad == 128 && b16 == (kB16X | kB16Y)) return WSV_160_128_B16;
            if (kx_pad == 128 && ny_pad == 128 && b16 == (kB16X | kB16Y)) return WSV_128_128_B16;
        }
        return WSV_NONE;
    }
    const bool mk = mask != 0;
    if (kx_pad == 160 && ny_pad == 160 && !mk) return yrow ? WSV_160_160_ROW : WSV_160_160;
    if (yrow) return WSV_NONE;
    if (kx_pad == 128 && ny_pad == 160 && mk) return WSV_128_160;
    if (kx_pad == 160 && ny_pad == 128 && mk) return WSV_160_128;
    if (kx_pad == 128 && ny_pad == 128 && mk) return WSV_128_128;
    return WSV_NONE;
}
// one gradient on its own launch (the per-shape kernels; SPWGNN_DIAG A/B of the batched launch)
hipError_t launch_wgrad_ws(const WgWsArgs& a, int wgs, int kx_pad, int ny_pad, int yrow, int mask, int math,
                           hipStream_t st, int b16) {
    const int v = wgrad_ws_variant(a, kx_pad, ny_pad, yrow, mask, math, b16);
    const dim3 g(wgs), b(kWsThreads);
    const bool bf = math == MATH_BF16;
    switch (v) {
#define SPW_WS(V, KX, NY, YR, MK, XD)                                                              \
        case V:                                                                                     \
            if (bf) hipLaunchKernelGGL((k_wgrad_ws<KX, NY, YR, MK, 1, XD>), g, b, 0, st, a);        \
            else hipLaunchKernelGGL((k_wgrad_ws<KX, NY, YR, MK, 3, XD>), g, b, 0, st, a);           \
            break;
        SPW_WS(WSV_160_160, 160, 160, 0, false, 0)
        SPW_WS(WSV_160_160_ROW, 160, 160, 1, false, 0)
        SPW_WS(WSV_128_160, 128, 160, 0, true, 0)
        SPW_WS(WSV_160_128, 160, 128, 0, true, 0)
        SPW_WS(WSV_128_128, 128, 128, 0, true, 0)
        SPW_WS(WSV_XD_EDGE, 160, 160, 0, false, 1)
        SPW_WS(WSV_XD_NODE, 128, 128, 0, true, 2)
#undef SPW_WS
        case WSV_XD_EDGE_B16Y: hipLaunchKernelGGL((k_wgrad_ws<160, 160, 0, false, 1, 1, kB16Y>), g, b, 0, st, a); break;
        case WSV_160_160_ROW_B16: hipLaunchKernelGGL((k_wgrad_ws<160, 160, 1, false, 1, 0, kB16X | kB16Y>), g, b, 0, st, a); break;
        case WSV_160_160_B16: hipLaunchKernelGGL((k_wgrad_ws<160, 160, 0, false, 1, 0, kB16X | kB16Y>), g, b, 0, st, a); break;
        case WSV_128_160_B16Y: hipLaunchKernelGGL((k_wgrad_ws<128, 160, 0, true, 1, 0, kB16Y>), g, b, 0, st, a); break;
        case WSV_160_128_B16: hipLaunchKernelGGL((k_wgrad_ws<160, 128, 0, true, 1, 0, kB16X | kB16Y>), g, b, 0, st, a); break;
        case WSV_128_128_B16: hipLaunchKernelGGL((k_wgrad_ws<128, 128, 0, true, 1, 0, kB16X | kB16Y>), g, b, 0, st, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
hipError_t launch_wgrad_ws_batch(const WsBatch& b, int math, hipStream_t st, const Pos3Batch* p3) {
    if (b.n <= 0 && b.w2_wgs <= 0) return p3 ? launch_wgrad_pos3(*p3, st) : hipSuccess;
    if (b.n > kMaxWsJobs || b.wgs < 0 || (b.n > 0 && b.wgs == 0) || b.w2_wgs < 0) return hipErrorInvalidValue;
    Pos3Batch none{};
    const Pos3Batch& q = p3 ? *p3 : none;
    if (b.w2_wgs && math != MATH_X6) return hipErrorInvalidValue;
    const dim3 g(b.wgs + (q.ce + q.cn + 1) / 2 + b.w2_wgs);
    if (math == MATH_BF16) hipLaunchKernelGGL(k_wgrad_ws_batch<1>, g, dim3(kWsThreads), 0, st, b, q);
    else hipLaunchKernelGGL(k_wgrad_ws_batch<3>, g, dim3(kWsThreads), 0, st, b, q);
    return hipGetLastError();
}
// Small batches (every gradient ≤ kReduceSmallChunks slabs): one thread per element sums its slabs in
// order — 100 workgroups per gradient instead of 800: at the reference's batch 32 the launch's
// workgroup dispatch, not its sums, was most of its 11 µs. Deterministic (a fixed order per element).
constexpr int kReduceSmallChunks = 64;
__global__ __launch_bounds__(256) void k_wgrad_reduce_small(ReduceBatch rb) {
    if (rb.bce_row && blockIdx.y == gridDim.y - 1) {   // spwgnn_bce_backward: the loss sums
        if (blockIdx.x == 0) bce_block_final(rb.bce);
        return;
    }
    if ((int)blockIdx.y == rb.n) {   // the ranges no reduction writes: zeros
        for (int z = 0; z < rb.nzero; ++z)
            for (int e = blockIdx.x * 256 + threadIdx.x; e < rb.zlen[z]; e += gridDim.x * 256) rb.r[0].out[rb.zoff[z] + e] = 0.f;
        return;
    }
    const ReduceArgs& a = rb.r[blockIdx.y];
    const int idx = blockIdx.x * 256 + threadIdx.x;
    const int k = idx / a.ny_pad, n = idx - k * a.ny_pad;
    const int col = a.perm ? wo2_perm(n) : n;
    const bool kern = a.kernel_off >= 0 && k < a.kernel_rows, bias = a.bias_off >= 0 && k == a.bias_row;
    if (!(idx < a.kx_pad * a.ny_pad && col >= 0 && col < a.kernel_cols && (kern || bias))) return;
    const int64_t stride = (int64_t)a.kx_pad * a.ny_pad;
    const float* p = a.slab + idx;
    float s0 = 0.f, s1 = 0.f;
    int c = 0;
    // eight slabs' loads in flight, added in the same order as two at a time (even chunks into s0, odd
    // into s1): the same bits, a quarter of the dependent load latencies (the W2 job's 32 slabs)
    for (; c + 7 < a.chunks; c += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = p[(c + u) * stride];
#pragma unroll
        for (int u = 0; u < 8; u += 2) {
            s0 += v[u];
            s1 += v[u + 1];
        }
    }
    for (; c + 1 < a.chunks; c += 2) {
        s0 += p[c * stride];
        s1 += p[(c + 1) * stride];
    }
    if (c < a.chunks) s0 += p[c * stride];
    const float s = s0 + s1;
    if (kern) a.out[a.kernel_off + (int64_t)(a.kernel_row0 + k) * a.kernel_cols + col] = s;
    if (bias) a.out[a.bias_off + col] = s;
}
hipError_t launch_wgrad_reduce_all(const ReduceBatch& rb, hipStream_t st) {
    if (rb.bce_row && (rb.bce.blocks != 1 || rb.bce.dlogits)) return hipErrorInvalidValue;   // one FINAL workgroup
    if (rb.n <= 0 && rb.nzero > 0) return hipErrorInvalidValue;   // the zero row writes through r[0].out
    if (rb.n <= 0 && !rb.bce_row) return hipSuccess;
    int maxc = 0;
    for (int k = 0; k < rb.n; ++k) maxc = rb.r[k].chunks > maxc ? rb.r[k].chunks : maxc;
    const int rows = rb.n + (rb.nzero > 0 ? 1 : 0) + (rb.bce_row ? 1 : 0);
    if (maxc <= kReduceSmallChunks)
        hipLaunchKernelGGL(k_wgrad_reduce_small, dim3((160 * 160 + 255) / 256, rows), dim3(256), 0, st, rb);
    else
        hipLaunchKernelGGL(k_wgrad_reduce_all, dim3((160 * 160 + 31) / 32, rows), dim3(256), 0, st, rb);
    return hipGetLastError();
}
hipError_t launch_bce(const BceArgs& a, hipStream_t st) {
    if (a.blocks == 1) {
        hipLaunchKernelGGL(k_bce_partial<true>, dim3(1), dim3(256), 0, st, a);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_bce_partial<false>, dim3(a.blocks), dim3(256), 0, st, a);
    hipLaunchKernelGGL(k_bce_final, dim3(1), dim3(64), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_adam(const AdamArgs& a, hipStream_t st) {
    const int64_t blocks = std::min<int64_t>((a.n + 255) / 256, 2048);
    hipLaunchKernelGGL(k_adam, dim3((unsigned)blocks), dim3(256), 0, st, a);
    return hipGetLastError();
}
hipError_t launch_step_advance(uint64_t* key, int32_t* step, int mode, uint64_t seed, int32_t rank, hipStream_t st) {
    hipLaunchKernelGGL(k_step_advance, dim3(1), dim3(64), 0, st, key, step, mode, seed, rank);
    return hipGetLastError();
}
hipError_t launch_tower_readout(const float* z, const int32_t* off, int n_towers, int mode, float* out, hipStream_t st) {
    hipLaunchKernelGGL(k_tower_readout, dim3((n_towers + 255) / 256), dim3(256), 0, st, z, off, n_towers, mode, out);
    return hipGetLastError();
}
// A replayed small-batch step's batch arrays, pinned (device-mapped) host staging → the static device
// buffer, as the step's first kernel: the loads cross PCIe once, all in flight together (a few µs),
// where a DMA copy between two replays left the GPU idle for ≈ 26 µs.
__global__ __launch_bounds__(256) void k_copy_in(const uint4* __restrict__ src, uint4* __restrict__ dst, int64_t n16) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256)
        dst[i] = ld_sys_u4(src + i);   // host staging the host rewrites between replays: system-coherent reads
}
hipError_t launch_copy_in(const void* src, void* dst, int64_t n16, hipStream_t st) {
    const int wgs = (int)std::min<int64_t>(64, (n16 + 1023) / 1024);   // ≤ 4 pieces per thread
    hipLaunchKernelGGL(k_copy_in, dim3(std::max(wgs, 1)), dim3(256), 0, st, static_cast<const uint4*>(src),
                       static_cast<uint4*>(dst), n16);
    return hipGetLastError();
}

__global__ void k_accumulate_out3(const float* out3, const double* w, double* tot) {
    const int k = threadIdx.x;
    if (k < 3) tot[k] += (double)out3[k] * w[k];
}
hipError_t launch_accumulate_out3(const float* out3, const double* w, double* tot, hipStream_t st) {
    hipLaunchKernelGGL(k_accumulate_out3, dim3(1), dim3(64), 0, st, out3, w, tot);
    return hipGetLastError();
}
hipError_t launch_sigmoid(const float* z, float* p, int64_t n, hipStream_t st) {
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 2048);
    hipLaunchKernelGGL(k_sigmoid, dim3((unsigned)std::max<int64_t>(blocks, 1)), dim3(256), 0, st, z, p, n);
    return hipGetLastError();
}

}  // namespace spw
