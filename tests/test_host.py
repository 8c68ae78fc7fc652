"""CPU: the C-ABI library loads and exports every declared symbol; host-side input builders
(dense→edge conversion, wave-tile plan), parameter layout, and data builders vs the reference
semantics (main.py:8-23, 66-81; JengaBuilder.py:137-192)."""
import ctypes as C
import json
import os
import re

import numpy as np
import pytest

from oracle import model as O
from spwgnn_amd import _lib, data as D, params as P
from spwgnn_amd.batch import TowerBatch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol():
    hdr = open(os.path.join(ROOT, "include", "spwgnn.h")).read()
    declared = set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(spwgnn_\w+)\s*\(", hdr, re.M))
    assert len(declared) >= 15
    lib = _lib.lib()
    for name in sorted(declared):
        assert hasattr(lib, name), name
    ver = int(re.search(r"#define SPWGNN_ABI_VERSION (\d+)", hdr).group(1))
    assert lib.spwgnn_version() == ver == _lib.ABI_VERSION
    # the ctypes run struct ends with the field the header declares last
    assert _lib.RunC._fields_[-1][0] == re.search(r"(\w+);\s*\} spwgnn_run;", hdr).group(1)
    assert b"workspace" in lib.spwgnn_strerror(-4)


def test_param_table_matches_reference_layout():
    shapes = dict(O.param_shapes())
    lay = P.layout()
    assert [n for n, _, _ in lay] == [n for n, _ in O.param_shapes()]
    for name, off, shape in lay:
        assert tuple(shape) == tuple(shapes[name]), name
        assert off % 64 == 0
    assert P.real_size() == 209501  # rm 68,400 + om 10,400 + rmp 90,400 + omp 40,301
    p = O.random_params(0)
    back = P.from_flat(P.to_flat(p))
    for k in p:
        assert np.array_equal(back[k].astype(np.float32), p[k])


def _c_dense_to_edges(Rs, Rr):
    B, N, E = Rs.shape
    Rs = np.ascontiguousarray(Rs, np.float32)
    Rr = np.ascontiguousarray(Rr, np.float32)
    src = np.zeros(B * E + 1, np.int32)
    dst = np.zeros(B * E + 1, np.int32)
    slot = np.zeros(B * E + 1, np.int32)
    tec = np.zeros(B, np.int32)
    n = C.c_int64()
    st = _lib.lib().spwgnn_dense_to_edges(Rs.ctypes.data, Rr.ctypes.data, B, N, src.ctypes.data, dst.ctypes.data,
                                          slot.ctypes.data, B * E, C.byref(n), tec.ctypes.data)
    return st, src[:n.value], dst[:n.value], slot[:n.value], tec


@pytest.mark.parametrize("fully", [True, False])
def test_dense_to_edges_matches_reference_enumeration(fully):
    raw = D.synthetic_towers(16, 7, seed=3)
    Rs, Rr = O.relation_matrices(raw, None if fully else 170.0)
    st, src, dst, slot, tec = _c_dense_to_edges(Rs, Rr)
    assert st == 0
    ref = O.dense_to_edges(Rs, Rr)
    assert len(ref) == len(src) == tec.sum()
    for (b, k, s, r), cs, cd, ck in zip(ref, src, dst, slot):
        assert (cs, cd, ck) == (b * 7 + s, b * 7 + r, k)


def test_dense_to_edges_rejects_non_onehot():
    Rs, Rr = O.relation_matrices(D.synthetic_towers(2, 4, seed=1), None)
    bad = Rs.copy()
    bad[0, 1, 0] = 1.0            # two senders in one column
    assert _c_dense_to_edges(bad, Rr)[0] == -3
    bad = Rs.copy()
    bad[0, :, 2] = 0.0            # receiver without sender
    assert _c_dense_to_edges(bad, Rr)[0] == -3
    half = Rr.copy()
    half[1, :, 3] = 0.0           # sender without receiver: never summed → dropped
    st, src, _, _, tec = _c_dense_to_edges(Rs, half)
    assert st == 0 and tec[1] == 11 and tec[0] == 12


@pytest.mark.parametrize("N,nw", [(6, None), (12, None), (4, 16), (3, 10)])
def test_plan_invariants(N, nw):
    B = 11
    raw = D.synthetic_towers(B, N, seed=N)
    Rs, Rr = O.relation_matrices(raw, 170.0)
    b = TowerBatch.from_dense((raw / 170).astype(np.float32), Rs, Rr, device="cpu", nw_max=nw)
    wt = b.wtile.numpy()
    esrc, edst = b.edge_src.numpy(), b.edge_dst.numpy()
    csr = b.blk_csr.numpy()
    assert wt[:, 1].sum() == b.n_eblocks
    seen = []
    tower_of = np.repeat(np.arange(B), N)
    node_cover = np.zeros(B * N, int)
    for fb, nb, n0, nn in wt:
        node_cover[n0:n0 + nn] += 1
        assert nn <= b.nw_max
        towers = set(tower_of[n0:n0 + nn])
        assert all((tower_of == t).sum() == (tower_of[n0:n0 + nn] == t).sum() for t in towers)  # whole towers
        for blk in range(fb, fb + nb):
            s = esrc[blk * 32:(blk + 1) * 32]
            d = edst[blk * 32:(blk + 1) * 32]
            valid = s >= 0
            assert np.all(valid[:valid.sum()])            # padding only at the end
            assert np.all((s[valid] >= n0) & (s[valid] < n0 + nn)) and np.all((d[valid] >= n0) & (d[valid] < n0 + nn))
            seen += list(zip(s[valid], d[valid]))
            for base, key in ((0, d), (64, s)):
                order = csr[blk, base:base + 32]
                nodes = csr[blk, base + 32:base + 64]
                assert sorted(order) == list(range(32))
                nv = valid.sum()
                assert np.all(nodes[nv:] == 255)
                assert np.all(nodes[:nv] == key[order[:nv]] - n0)
                assert np.all(np.diff(nodes[:nv].astype(int)) >= 0)
    assert np.all(node_cover == 1)
    assert sorted(seen) == sorted(zip(b.src, b.dst))


def test_relation_matrices_vectorised_equals_reference_loop():
    raw = D.synthetic_towers(9, 6, seed=5)
    for thr in (None, 170.0, 120.0):
        a = D.relation_matrices(raw, thr)
        b = O.relation_matrices(raw, thr)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_synthetic_tower_geometry():
    raw = D.synthetic_towers(200, 6, seed=0)
    assert raw.shape == (200, 6, 3)
    assert np.all((raw[..., 2] >= 50) & (raw[..., 2] <= 300))             # JengaBuilder.py:57-58
    assert np.all(((raw[..., 1] - 110) % 80) == 0)                        # y = 70 + 40 + 80·layer
    assert np.all(raw[..., 0] > 0)


def test_calculate_stability_matches_reference_loop():
    rng = np.random.default_rng(0)
    boxes = rng.normal(0, 0.1, size=(5, 7, 4, 3)).cumsum(axis=1)
    boxes[:, :, 0] = 3.0                   # a static object → stable
    y = D.calculate_stability(boxes)
    ref = np.zeros((5, 4, 1))
    for o in range(4):                     # main.py:16-22
        for t in range(5):
            pc = sum(np.linalg.norm(boxes[t, f, o, 0:2] - boxes[t, f + 1, o, 0:2]) for f in range(0, 6))
            ref[t, o, 0] = 1.0 if pc < 0.5 else 0.0
    assert np.array_equal(y, ref)
    assert np.all(y[:, 0, 0] == 1.0)


def test_json_loader_pads_with_last_frame(tmp_path):
    data = [[[[1, 2, 50], [1, 3, 50]], [[5, 6, 70]]], [], [[[0, 0, 60]], [[9, 9, 80], [9, 8, 80], [9, 7, 80]]]]
    p = tmp_path / "jenga_model_3_2_x.txt"
    p.write_text(json.dumps(data))
    boxes = D.load_trajectories(str(p), 2)
    assert boxes.shape == (2, 2, 2, 3)               # empty dropped; F = max len of object 0 (main.py:46-47)
    assert np.array_equal(boxes[0, 1, 1], [5, 6, 70])  # padded with last frame (main.py:56-59)
    assert np.array_equal(boxes[1, :, 1, 1], [9, 8])   # truncated to F frames
    assert np.array_equal(boxes[1, 1, 0], [0, 0, 60])


def test_training_arrays_layout():
    boxes = np.repeat(D.synthetic_towers(3, 5, seed=2)[:, None], 4, axis=1)
    x, y = D.training_arrays(boxes)
    assert set(x) == {"objects", "sender_relations", "receiver_relations", "propagation"}   # main.py:92
    assert x["objects"].shape == (3, 5, 3) and x["sender_relations"].shape == (3, 5, 20)
    assert np.all(y["target"] == 1.0)                 # static trajectories are stable
    assert np.allclose(x["objects"] * 170, boxes[:, 0])


def test_removal_candidates_order():
    from spwgnn_amd.demolish import removal_candidates
    boxes = np.arange(15, dtype=np.float64).reshape(5, 3)
    c = removal_candidates(boxes)
    assert c.shape == (5, 4, 3)
    for i in range(5):
        assert np.array_equal(c[i], np.delete(boxes, i, axis=0))   # JengaBuilder.py:244-249 order


def test_bench_pmc_names_match_committed_summaries():
    """bench.py's roofline `traffic` looks kernels up by name prefix in the committed PMC summary of
    each config; a kernel rename must be caught here, not show up as a null. Every committed summary
    with a `_workload` tag is quoted only for that workload."""
    import glob
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    for path in sorted(glob.glob(os.path.join(root, "profiles", "pmc_summary*.json"))):
        with open(path) as f:
            summary = json.load(f)
        m = re.search(r"config(\d)", os.path.basename(path))
        config = int(m.group(1)) if m else 0
        meta = summary.get("_workload", {})
        wl, math = meta.get("workload"), meta.get("math") or "x6"
        kernels = ["edge_fwd"] if config == 5 else ["edge_fwd", "edge_bwd", "enc_edge", "enc_edge_bwd", "wgrad_w2"]
        # config 1 (32 towers) runs the fused small-batch launches: bench looks those up
        bench._FUSED[0] = config == 1
        if config == 1:
            kernels = list(bench.FUSED_PARTS)
        for k in kernels:
            assert bench.load_pmc(config, k, math, wl) is not None, (path, k)
        if meta:
            assert bench.load_pmc(config, kernels[0], math, wl + " (other)") is None
        assert bench.step_hbm(config, 10.0, math, wl) is not None, path


def test_bench_dominant_kernel_rule():
    """The roofline names the kernel with the largest ms per step; the weight-gradient family counts
    as one kernel only when it ran as one batched launch per backward (k_wgrad_ws_batch)."""
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    table = {"edge_fwd": {"ms_per_step": 3.7}, "dA": {"ms_per_step": 2.4},
             "wgrad_ws": {"ms_per_step": 4.6, "batched": True}}
    assert bench.dominant(table) == "wgrad_ws"
    table["wgrad_ws"]["batched"] = False
    assert bench.dominant(table) == "edge_fwd"
    assert bench.dominant({}) == "edge_fwd"


def test_bench_roofline_bound_follows_intensity():
    """The roofline's bound is the roof with the larger floor: the weight-gradient kernel (34 FLOP/B
    at x6, ridge 52) is priced against HBM, the aggregate-gradient dA (162 FLOP/B) against the matrix
    peak; the fused small-batch launches stay on the matrix roof; frac = achieved / peak either way."""
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    Ne, Nn, S = 1966080, 393216, 5
    bench._FUSED[0] = False
    r = bench.roofline("wgrad_ws", [4.5], 1, Ne, Nn, S, "x6", 0, "t")
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == bench.PEAK_HBM_GBS
    assert r["intensity_flop_per_byte"] < r["ridge_flop_per_byte"]
    assert abs(r["frac"] - r["alg_bytes_per_launch"] / 4.5e-3 / 1e9 / bench.PEAK_HBM_GBS) < 1e-3
    r = bench.roofline("dA", [2.0], 1, Ne, Nn, S, "x6", 0, "t")
    assert r["bound"] == "mfma" and r["unit"] == "TFLOP/s" and r["frac"] == r["mfma_frac"]
    bench._FUSED[0] = True
    r = bench.roofline("wgrad_ws", [0.02], 1, 4000, 400, S, "x6", 1, "t")
    assert r["bound"] == "mfma" and r["alg_bytes_per_launch"] is None
    bench._FUSED[0] = False


def test_plan_without_any_edge_and_empty_batch():
    """Single-box towers: no edge list at all (NULL src/dst through the C-ABI), one padding block
    per wave-tile; an empty batch is rejected before the library is called."""
    from spwgnn_amd import TowerBatch, data as D
    objs = [(D.synthetic_towers(1, 1, seed=i)[0] / 170).astype(np.float32) for i in range(5)]
    b = TowerBatch.ragged(objs, device="cpu")
    assert b.n_edges == 0 and b.n_eblocks == b.n_wtiles >= 1
    assert np.all(b.edge_src.numpy() == -1) and np.all(b.edge_dst.numpy() == -1)
    with pytest.raises(ValueError):
        TowerBatch.ragged([], device="cpu")


def test_plan_rejects_cross_tower_edge_inside_one_packed_tile():
    """Two 3-box towers pack into one 16-node wave-tile; an edge from tower 0 to tower 1 must still
    be rejected (the check is against the edge's own tower, not the tile)."""
    pos = np.zeros((6, 3), np.float32)
    tn = np.array([3, 3], np.int32)
    src = np.array([0, 1, 3, 2], np.int32)
    dst = np.array([1, 0, 4, 4], np.int32)      # 2 → 4 crosses towers
    with pytest.raises(_lib.SpwgnnError):
        TowerBatch.from_edges(pos, tn, src, dst, np.array([2, 2], np.int32), device="cpu", nw_max=16)
    ok = TowerBatch.from_edges(pos, tn, src[:3], np.array([1, 0, 4], np.int32), np.array([2, 1], np.int32),
                               device="cpu", nw_max=16)
    assert ok.n_wtiles == 1


# (B, validation_split) → training samples, worked by hand from Keras 2.x's
# split_at = int(num_train_samples * (1. - validation_split)):
#   7·0.8 = 5.6 → 5; 13·0.8 = 10.4 → 10; 10·0.8 = 8.000000000000002 → 8; 96·0.75 = 72;
#   5, v = 0 → 5 (no split); 3·0.5 = 1.5 → 1; 1000·0.8 = 800; 9·(1 − 0.1) = 8.1 → 8; 4·0.8 = 3.2 → 3
@pytest.mark.parametrize("B,v,want", [(7, 0.2, 5), (13, 0.2, 10), (10, 0.2, 8), (96, 0.25, 72), (5, 0.0, 5),
                                      (3, 0.5, 1), (1000, 0.2, 800), (9, 0.1, 8), (4, 0.2, 3)])
def test_keras_validation_split_matches_keras2(B, v, want):
    """Keras 2.x fit: split_at = int(B·(1 − v)) training samples, the rest is validation (main.py:96)."""
    from spwgnn_amd.keras_api import keras_split_at
    assert keras_split_at(B, v) == want


def test_ragged_batch_matches_per_tower_relations():
    """data.ragged_batch (config 4's vectorised builder) equals the per-tower loop of main.py:71-81 on
    every tower: same thresholded sender-major edges, positions /170; edge_slice rebases a sub-range."""
    pos, sz, s, d, te, raw = D.ragged_batch(300, 4, 16, seed=5)
    assert sz.min() >= 4 and sz.max() <= 16 and len(raw) == 300
    off = np.concatenate([[0], np.cumsum(sz)])
    eo = np.concatenate([[0], np.cumsum(te)])
    for t in range(300):
        n, r = sz[t], raw[t]
        m, j = np.nonzero(~np.eye(n, dtype=bool))
        k = np.linalg.norm(r[m, :2] - r[j, :2], axis=1) < D.RELATION_THRESHOLD
        assert np.array_equal(s[eo[t]:eo[t + 1]], off[t] + m[k])
        assert np.array_equal(d[eo[t]:eo[t + 1]], off[t] + j[k])
        assert np.array_equal(pos[off[t]:off[t + 1]], (r / D.RELATION_THRESHOLD).astype(np.float32))
    p2, n2, s2, d2, e2 = D.edge_slice(pos, sz, s, d, te, 100, 200)
    assert np.array_equal(s2 + off[100], s[eo[100]:eo[200]]) and np.array_equal(n2, sz[100:200])
    assert len(p2) == off[200] - off[100] and s2.min() >= 0 and d2.max() < len(p2)


def test_compact_dataset_subset_matches_per_tower_gather():
    """keras_api.CompactDataset.subset gathers the towers' edge ranges in one vectorised pass:
    same edge list as walking the towers one by one (node ids shifted by k·N for batch tower k)."""
    from spwgnn_amd import data as D
    from spwgnn_amd.keras_api import CompactDataset
    obj, Rs, Rr, prop, _ = D.synthetic_batch(40, 7, seed=4, fully_connected=False)
    ds = CompactDataset(obj, Rs, Rr, prop)
    for idx in (np.arange(40), np.random.default_rng(1).permutation(40)[:13], np.array([5])):
        b = ds.subset(idx, "cpu")
        ps, pd = [], []
        for k, t in enumerate(idx):
            e0, e1 = ds.edge_off[t], ds.edge_off[t + 1]
            ps.append(ds.src[e0:e1] + k * ds.N)
            pd.append(ds.dst[e0:e1] + k * ds.N)
        assert np.array_equal(b.src, np.concatenate(ps)) and np.array_equal(b.dst, np.concatenate(pd))


def test_batch_upload_roundtrip_cpu():
    """batch.upload packs host arrays into one staging buffer (16-byte aligned pieces) and returns
    one tensor per array with its dtype and shape."""
    from spwgnn_amd.batch import upload
    arrs = [np.arange(7, dtype=np.int32), np.ones((3, 4), np.float32) * 2.5, np.arange(5, dtype=np.uint8),
            np.zeros(0, np.int32)]
    out = upload(arrs, "cpu")
    for a, t in zip(arrs, out):
        assert t.shape == a.shape and np.array_equal(t.numpy(), a)


class _UniformRandint:
    """random.Random stand-in for `jenga_tower`: randint(a, b) from a row of uniforms, in order."""

    def __init__(self, row):
        self.row, self.k = row, 0

    def randint(self, a, b):
        v = a + min(int(np.floor(self.row[self.k] * (b - a + 1))), b - a)
        self.k += 1
        return v


@pytest.mark.parametrize("n", [1, 2, 4, 6, 9, 12, 16, 32])
def test_vectorised_jenga_builder_equals_scalar(n):
    """data.jenga_towers_from_draws (the lockstep builder the benchmark's large batches use) gives,
    tower for tower, what the scalar JengaBuilder.create_world restatement `jenga_tower` gives on the
    same draws (JengaBuilder.py:150-184), including the removed box (JengaBuilder.py:223-233)."""
    T = 300
    u = np.random.default_rng(n).random((T, D.draws_per_tower(n)))
    vec = D.jenga_towers_from_draws(u, n)
    for t in range(T):
        r = _UniformRandint(u[t])
        tower = D.jenga_tower(n + 1, r)
        tower = np.delete(tower, r.randint(0, len(tower) - 1), axis=0)
        assert r.k <= u.shape[1]
        np.testing.assert_array_equal(vec[t], tower)
    fast = D.synthetic_towers_fast(64, n, seed=3)
    assert fast.shape == (64, n, 3) and np.all(fast[..., 2] >= D.RECT_WIDTH_MIN)


def test_capacity_plan_shares_geometry_and_edge_layout():
    """spwgnn_plan_fill_cap: blocks sized for N(N-1) edges per tower, so two batches of 6-block
    towers with different relation sets get the same wave-tiles and block counts (one captured
    graph); each real edge sits where the actual-count plan puts it, the rest is padding (-1)."""
    from spwgnn_amd.batch import HostPlan
    geo = set()
    for seed in (1, 2, 3):
        obj, Rs, Rr, prop, _ = D.synthetic_batch(32, 6, seed=seed, fully_connected=False)
        e = np.array(O.dense_to_edges(Rs, Rr), np.int64).reshape(-1, 4)
        src, dst = (e[:, 0] * 6 + e[:, 2]).astype(np.int32), (e[:, 0] * 6 + e[:, 3]).astype(np.int32)
        te = np.bincount(e[:, 0], minlength=32).astype(np.int32)
        nodes = np.full(32, 6, np.int32)
        plain = HostPlan.build(obj.reshape(-1, 3), nodes, src, dst, te, nw_max=16)
        cap = HostPlan.build(obj.reshape(-1, 3), nodes, src, dst, te, edge_cap=30, nw_max=16)
        geo.add(cap.geometry)
        assert cap.n_wtiles == plain.n_wtiles == 16 and cap.n_eblocks == 32 >= plain.n_eblocks
        wp, wc = plain.arrays[3], cap.arrays[3]
        assert np.array_equal(wp[:, [2, 3]], wc[:, [2, 3]])           # same towers per wave-tile
        for t in range(16):
            a, n = wp[t, 0], wp[t, 1]
            b, m = wc[t, 0], wc[t, 1]
            assert m == 2 and n <= m
            for arr in (4, 5):
                got = cap.arrays[arr][32 * b: 32 * (b + m)]
                want = plain.arrays[arr][32 * a: 32 * (a + n)]
                assert np.array_equal(got[:len(want)], want) and np.all(got[len(want):] == -1)
            assert np.array_equal(cap.arrays[6][b: b + n], plain.arrays[6][a: a + n])
    assert len(geo) == 1
    with pytest.raises(ValueError):
        HostPlan.build(obj.reshape(-1, 3), nodes, src, dst, te, edge_cap=1)


def test_adam_lr_table_is_keras_adam_lr_t():
    """spwgnn_adam_lr_table (host, the table replayed steps read lr_t from) = Keras-2.x Adam's
    lr_t = lr·sqrt(1−β2^t)/(1−β1^t) (Networks.py:101), rounded to fp32 once."""
    out = np.zeros(5000, np.float32)
    assert _lib.lib().spwgnn_adam_lr_table(5e-4, 0.9, 0.999, len(out), out.ctypes.data) == 0
    t = np.arange(1, len(out), dtype=np.float64)
    want = (np.float32(5e-4).astype(np.float64) * np.sqrt(1 - np.float32(0.999).astype(np.float64) ** t)
            / (1 - np.float32(0.9).astype(np.float64) ** t)).astype(np.float32)
    assert out[0] == 0.0
    assert np.array_equal(out[1:], want)
    assert _lib.lib().spwgnn_adam_lr_table(5e-4, 0.9, 0.999, 1, out.ctypes.data) != 0


def test_small_batches_take_one_tower_per_wave_tile():
    """default_nw_max: below SMALL_BATCH_TOWERS towers of ≤ 16 boxes one tower per wave-tile (more
    waves for a batch that cannot fill the chip), from there on packed up to 16 nodes; > 16 boxes
    always one tower per tile."""
    from spwgnn_amd.batch import SMALL_BATCH_TOWERS, HostPlan, default_nw_max
    assert default_nw_max(6, 32) == 6 and default_nw_max(6, SMALL_BATCH_TOWERS) == 16
    assert default_nw_max(20, 32) == 20 and default_nw_max(20, 10 ** 6) == 20
    obj, Rs, Rr, prop, _ = D.synthetic_batch(32, 6, seed=1, fully_connected=True)
    e = np.array(O.dense_to_edges(Rs, Rr), np.int64).reshape(-1, 4)
    te = np.bincount(e[:, 0], minlength=32).astype(np.int32)
    p = HostPlan.build(obj.reshape(-1, 3), np.full(32, 6, np.int32), e[:, 0] * 6 + e[:, 2], e[:, 0] * 6 + e[:, 3], te)
    assert p.n_wtiles == 32 and p.nw_max == 6 and p.n_eblocks == 32


def test_input_validation_errors():
    """The boundary's error behaviour: a relation column that is not one-hot, a
    receiver without a sender, wrongly shaped relation matrices and towers beyond the 32-box
    limit raise instead of silently summing rows (Keras' batch_dot would)."""
    from spwgnn_amd import TowerBatch
    obj, Rs, Rr, prop, _ = D.synthetic_batch(2, 4, seed=3, fully_connected=True)
    bad = Rs.copy()
    bad[0, 1, 0] = 1.0                       # column 0 of tower 0 now has two senders
    with pytest.raises(_lib.SpwgnnError, match="one-hot"):
        TowerBatch.from_dense(obj, bad, Rr, device="cpu")
    half = Rs.copy()
    half[0, :, 3] = 0.0                      # column 3: a receiver without a sender
    with pytest.raises(_lib.SpwgnnError, match="one-hot"):
        TowerBatch.from_dense(obj, half, Rr, device="cpu")
    scaled = Rs * 2.0                        # not {0, 1}
    with pytest.raises(_lib.SpwgnnError):
        TowerBatch.from_dense(obj, scaled, Rr, device="cpu")
    with pytest.raises(ValueError):
        TowerBatch.from_dense(obj, Rs[:, :, :5], Rr[:, :, :5], device="cpu")
    big = (D.synthetic_towers(1, 33, seed=0) / 170).astype(np.float32)
    with pytest.raises(ValueError, match="33|32"):
        TowerBatch.fully_connected(big, device="cpu")
    # an all-zero column (inactive relation) is valid and dropped
    off = Rs.copy(), Rr.copy()
    off[0][0, :, 2] = 0.0
    off[1][0, :, 2] = 0.0
    b = TowerBatch.from_dense(obj, off[0], off[1], device="cpu")
    assert b.n_edges == 2 * 12 - 1


@pytest.mark.parametrize("N,thr", [(32, None), (27, None), (20, 170.0), (6, 170.0)])
def test_receiver_block_plan_invariants(N, thr):
    """spwgnn_plan_fill_recv: one 32-edge block per node holding exactly that node's in-edges (input
    order kept within a receiver), padding after them, every edge once, the csr sorted per block; the
    automatic choice takes it for dense towers of more than 16 nodes only."""
    B = 5
    raw = D.synthetic_towers(B, N, seed=N + 1)
    Rs, Rr = O.relation_matrices(raw, thr)
    dense = TowerBatch.from_dense((raw / 170).astype(np.float32), Rs, Rr, device="cpu")
    b = TowerBatch.from_edges(dense.pos.numpy()[:, :3], dense.tower_nodes, dense.src, dense.dst, dense.tower_edges,
                              device="cpu", recv_blocks=True)
    assert b.flags == _lib.BATCH_RECV_BLOCKS and b.n_eblocks == b.n_nodes
    esrc, edst, csr, wt = b.edge_src.numpy(), b.edge_dst.numpy(), b.blk_csr.numpy(), b.wtile.numpy()
    assert np.array_equal(wt[:, 1], wt[:, 3]) and wt[:, 1].sum() == b.n_nodes
    seen = []
    for fb, nb, n0, nn in wt:
        for j in range(nb):
            blk = fb + j
            s, d = esrc[blk * 32:(blk + 1) * 32], edst[blk * 32:(blk + 1) * 32]
            valid = s >= 0
            nv = int(valid.sum())
            assert np.all(valid[:nv]) and np.all(d[valid] == n0 + j)        # node n0 + j's in-edges only
            ref = [(x, y) for x, y in zip(dense.src, dense.dst) if y == n0 + j]   # input order kept
            assert list(zip(s[:nv], d[:nv])) == ref
            seen += ref
            for base, key in ((0, d), (64, s)):
                order, nodes = csr[blk, base:base + 32], csr[blk, base + 32:base + 64]
                assert sorted(order) == list(range(32)) and np.all(nodes[nv:] == 255)
                assert np.all(nodes[:nv] == key[order[:nv]] - n0)
    assert sorted(seen) == sorted(zip(dense.src, dense.dst))
    auto = TowerBatch.from_edges(dense.pos.numpy()[:, :3], dense.tower_nodes, dense.src, dense.dst, dense.tower_edges,
                                 device="cpu")
    assert (auto.flags == _lib.BATCH_RECV_BLOCKS) == (N > 16 and thr is None and N >= 27)


def _swap16(x, y):
    """v_permlane16_swap on 64-lane registers (lane axis 0): odd 16-lane rows of x <-> even rows of y."""
    x2, y2 = x.copy(), y.copy()
    for r in (0, 2):
        x2[16 * (r + 1):16 * (r + 2)] = y[16 * r:16 * (r + 1)]
        y2[16 * r:16 * (r + 1)] = x[16 * (r + 1):16 * (r + 2)]
    return x2, y2


def _swap32(x, y):
    """v_permlane32_swap: upper 32 lanes of x <-> lower 32 lanes of y."""
    x2, y2 = x.copy(), y.copy()
    x2[32:], y2[:32] = y[:32], x[32:]
    return x2, y2


@pytest.mark.parametrize("kh,nkb", [(0, 7), (0, 8), (76, 10), (56, 7)])
def test_half_tile_layout_algebra(kh, nkb):
    """The half-tile products (gemm_blocks.h ht_*, k_prep's ht slots) restated lane by
    lane in numpy: the 16x16x32 operands built by one permlane16 swap per k-block pair, multiplied
    with the image's ht slot, and converted back to the 32x32 C layout give rows 96..111 of Wᵀ·B for
    every node of the column tile (both k mappings: chain C layout and half rows)."""
    rng = np.random.default_rng(kh + nkb)
    K = 2 * kh if kh else 16 * nkb
    W = rng.standard_normal((K, 128))
    B = rng.standard_normal((K, 32))

    def kidx(kb, h, e):
        if kh:
            return (kh * h + 8 * kb + e) if 8 * kb + e < kh else None
        return 16 * kb + 8 * (e >> 2) + 4 * h + (e & 3)

    def bop(kb):   # 32x32x16 B operand of k-block kb: [lane][e]
        v = np.zeros((64, 8))
        if kb >= nkb:
            return v
        for l in range(64):
            for e in range(8):
                k = kidx(kb, l >> 5, e)
                v[l, e] = B[k, l & 31] if k is not None else 0.0
        return v

    def aop(P):    # the image's ht slot of pair P: lane (i, g) = W[k(2P + (g&1), g>>1, e)][96 + i]
        a = np.zeros((64, 8))
        for l in range(64):
            i, g = l & 15, l >> 4
            kb = 2 * P + (g & 1)
            for e in range(8):
                k = kidx(kb, g >> 1, e) if kb < nkb else None
                a[l, e] = W[k, 96 + i] if k is not None else 0.0
        return a

    q = np.zeros((2, 64, 4))   # two 16x16 accumulators: lane (c, g) reg r = row 4g + r, node 16q + c
    for P in range((nkb + 1) // 2):
        b0, b1 = _swap16(bop(2 * P), bop(2 * P + 1))
        a = aop(P)
        for qi, bq in enumerate((b0, b1)):
            for l in range(64):
                c, g = l & 15, l >> 4
                for r in range(4):
                    i = 4 * g + r
                    q[qi, l, r] += sum(a[i + 16 * gg] @ bq[c + 16 * gg] for gg in range(4))
    out = np.zeros((64, 16))
    for r in range(4):
        x, y = _swap16(q[0, :, r], q[1, :, r])
        lo, hi = _swap32(x, y)
        out[:, r], out[:, 4 + r] = lo, hi
    ref = W.T @ B                       # [128 features][32 nodes]
    for l in range(64):
        j, h = l & 31, l >> 5
        for r in range(8):
            f = 96 + (r & 3) + 8 * (r >> 2) + 4 * h
            assert abs(out[l, r] - ref[f, j]) < 1e-9, (l, r)
    # and the inverse conversion (ht_enter) restores the accumulators
    q2 = np.zeros_like(q)
    for r in range(4):
        x, y = _swap32(out[:, r], out[:, 4 + r])
        q2[0, :, r], q2[1, :, r] = _swap16(x, y)
    assert np.array_equal(q2, q)


def test_team_limit_is_a_runtime_setting():
    """spwgnn_team_max_blocks (ABI 5): the small-batch limit defaults to 512 blocks, can be moved at run
    time (0 = every batch on the wide kernels) and is restored; spwgnn_fused_path follows it (host
    planning only, no device work — the batch arrays may live in host memory for this query)."""
    from spwgnn_amd import engine as E
    assert E.team_max_blocks() == 512
    obj, Rs, Rr, prop, _ = D.synthetic_batch(4, 6, seed=1)
    batch = TowerBatch.from_dense(obj, Rs, Rr, prop, device="cpu")
    run = E.RunConfig(5, training=True, math="x6")
    assert E.fused_path(batch, run) == 3
    with E.wide_kernels():
        assert E.team_max_blocks() == 0
        assert E.fused_path(batch, run) == 0
    assert E.team_max_blocks() == 512
    assert E.team_max_blocks(7) == 512 and E.team_max_blocks(512) == 7


def test_packed_tower_order_fills_blocks():
    """spwgnn_plan_order (ABI 5): a permutation, deterministic; planned in that order a ragged batch never
    needs more 32-edge blocks than in its own order, and BASELINE config 4's ragged 4-16-box thresholded
    towers fill >= 75 % of their blocks (67 % in input order); node rows, edges and tower ids follow."""
    from spwgnn_amd.batch import HostPlan, pack_order
    pos, sizes, src, dst, te, _ = D.ragged_batch(8192, 4, 16, seed=4000)
    o = pack_order(sizes, te, 16)
    assert np.array_equal(np.sort(o), np.arange(len(sizes))) and np.array_equal(o, pack_order(sizes, te, 16))
    a = HostPlan.build(pos, sizes, src, dst, te)
    b = HostPlan.build(pos, sizes, src, dst, te, pack=True)
    assert b.n_eblocks <= a.n_eblocks and len(src) / (32 * b.n_eblocks) >= 0.75 > len(src) / (32 * a.n_eblocks)
    perm = b.node_perm
    assert np.array_equal(np.sort(perm), np.arange(len(pos)))
    assert np.array_equal(b.arrays[0][:, :3], pos[perm])          # node rows in plan order
    # every edge of the packed batch is an input edge, rebased: (perm[s], perm[d]) in the input's set
    inp = set(zip(src.tolist(), dst.tolist()))
    assert all((int(perm[s]), int(perm[d])) in inp for s, d in zip(b.src, b.dst)) and len(b.src) == len(src)
    # each node keeps its tower id (the dropout key) and its index inside the tower
    tower_of = np.repeat(np.arange(len(sizes)), sizes)
    assert np.array_equal(b.arrays[1], tower_of[perm])
    starts = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    assert np.array_equal(b.arrays[2], perm - starts[tower_of[perm]])
    # random small ragged batches: never more blocks
    rng = np.random.default_rng(3)
    for _ in range(20):
        T = int(rng.integers(1, 200))
        tn = rng.integers(1, 17, T).astype(np.int32)
        tev = np.array([rng.integers(0, n * (n - 1) + 1) for n in tn], np.int32)
        sz = _lib.PlanSizes()
        L = _lib.lib()
        L.spwgnn_plan_size(T, tn.ctypes.data, tev.ctypes.data, 16, C.byref(sz))
        n0 = sz.n_eblocks
        oo = pack_order(tn, tev, 16)
        tn2, te2 = np.ascontiguousarray(tn[oo]), np.ascontiguousarray(tev[oo])
        L.spwgnn_plan_size(T, tn2.ctypes.data, te2.ctypes.data, 16, C.byref(sz))
        assert sz.n_eblocks <= n0


def test_packed_batch_maps_rows_both_ways():
    """TowerBatch.from_edges(pack=True) on host memory: 'propagation' rows follow their nodes, and
    to_plan_order / to_input_order are inverse permutations (numpy and torch)."""
    import torch
    pos, sizes, src, dst, te, _ = D.ragged_batch(300, 4, 16, seed=8)
    n = int(sizes.sum())
    prop = np.random.default_rng(1).normal(size=(n, 100)).astype(np.float32)
    b = TowerBatch.from_edges(pos, sizes, src, dst, te, prop=prop, device="cpu", pack=True)
    assert b.node_perm is not None
    assert np.array_equal(b.prop.numpy(), prop[b.node_perm])
    assert np.array_equal(b.pos.numpy()[:, :3], pos[b.node_perm])
    x = np.arange(n, dtype=np.float32)
    assert np.array_equal(b.to_input_order(b.to_plan_order(x)), x)
    t = torch.arange(n, dtype=torch.float32)
    assert torch.equal(b.to_input_order(b.to_plan_order(t)), t)
    assert np.array_equal(b.to_plan_order(x), x[b.node_perm])
    plain = TowerBatch.from_edges(pos, sizes, src, dst, te, device="cpu")
    assert plain.node_perm is None and plain.to_plan_order(x) is x
