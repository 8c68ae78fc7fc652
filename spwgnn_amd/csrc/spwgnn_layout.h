// Shared host/device constants and the parameter table of libspwgnn_hip.
#pragma once
#include <cstdint>
#include <hip/hip_runtime.h>
#include <cstdio>

namespace spw {

// ---- model widths (Networks.py:29,46-50) ----
constexpr int kFE = 150;    // relation widths (rm hidden/out, rmp hidden)
constexpr int kFN = 100;    // object / state widths (om, effect, P, omp hidden)
constexpr int kLdE = 160;   // row stride (floats) of every 150/151-wide array  (5 MFMA tiles of 32)
constexpr int kLdN = 128;   // row stride (floats) of every 100/101-wide array  (4 MFMA tiles of 32)
constexpr int kKhE = 76;    // split-halves contraction: features [76h, 76h+76), h = lane/32 (152 = 150 + 2 zero)
constexpr int kKhN = 52;    // split-halves contraction for 100-wide inputs (104 = 100 + 4 zero)
constexpr int kNwMaxLimit = 32;   // max nodes per wave-tile (LDS node accumulators)
constexpr int kDegCol = 150;      // H2s column 150 holds the in-degree (multiplies the rmp.2 bias)

// ---- chunk-major edge rows ("CM"): a 32-edge block of 152-wide rows stored as
// [q < 19][h < 2][edge i < 32][4] — feature f = 76h + 4q + c. A wave's 16-byte-per-lane access in
// either orientation (lane = edge) is 1 KiB contiguous, where row-major rows would touch 64 lines.
// Node rows use the same scheme per 32-node block: 160-wide arrays with KH = 76 (152 features),
// 128-wide (100-feature) arrays with KH = 52 (104 features).
template <int KH>
__host__ __device__ constexpr int cm_offk(int i, int f) {
    return (((f >= KH ? f - KH : f) >> 2) * 2 + (f >= KH ? 1 : 0)) * 128 + i * 4 + (f & 3);
}
constexpr int kCmBlk = kKhE * 64;    // 4864 floats per 32-row block of a 152-feature array
constexpr int kCmBlkN = kKhN * 64;   // 3328 floats per 32-row block of a 104-feature array
constexpr int kRowE = 2 * kKhE;      // floats per row of a chunk-major 152-feature array
constexpr int kRowN = 2 * kKhN;      // floats per row of a chunk-major 104-feature array
__host__ __device__ constexpr int cm_off(int i, int f) { return cm_offk<kKhE>(i, f); }

constexpr int kNumTensors = 22;

struct TensorDesc {
    const char* name;
    int64_t offset;
    int32_t rows, cols;
};
struct ParamTable {
    TensorDesc t[kNumTensors];
    int64_t total;  // padded
    int64_t real;
};
const ParamTable& param_table();

// Tensor indices in the flat buffer (order of param_table: rm.0..3, om.0..1, rmp.0..2, omp.0..1; kernel, bias)
enum TensorId : int {
    T_RM0K = 0, T_RM0B, T_RM1K, T_RM1B, T_RM2K, T_RM2B, T_RM3K, T_RM3B,
    T_OM0K, T_OM0B, T_OM1K, T_OM1B,
    T_RMP0K, T_RMP0B, T_RMP1K, T_RMP1B, T_RMP2K, T_RMP2B,
    T_OMP0K, T_OMP0B, T_OMP1K, T_OMP1B,
};

}  // namespace spw
