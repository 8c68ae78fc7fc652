"""Numpy restatement of the engine's dropout key (spwgnn_amd/csrc/device_common.h: mix32,
drop_row_key, drop_keep) — TEST INFRASTRUCTURE ONLY.

Keras draws its Dropout masks from TensorFlow's RNG (Networks.py:77-78), which cannot be
reproduced; the engine uses its own counter-based key instead, and this module rebuilds the same
multiplicative masks bit-exactly so the oracle can be run with identical dropout.
"""
from __future__ import annotations

import numpy as np

M32 = np.uint64(0xFFFFFFFF)


def mix32(x):
    x = np.asarray(x, dtype=np.uint64) & M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & M32
    x ^= x >> np.uint64(16)
    return x


def row_key(seed: int, kind: int, tower, a, b):
    lo = np.uint64(seed & 0xFFFFFFFF)
    hi = np.uint64((seed >> 32) & 0xFFFFFFFF)
    h = mix32(lo ^ mix32((hi + np.uint64(kind)) & M32))
    h = mix32(h ^ (np.asarray(tower, np.uint64) & M32))
    ab = ((np.asarray(a, np.uint64) << np.uint64(16)) | (np.asarray(b, np.uint64) & np.uint64(0xFFFF))) & M32
    return mix32(h ^ ab)


def keep(rowkey, n_features: int, rate: float):
    thresh = np.uint64(min(0xFFFFFFFF, int(np.floor(rate * 4294967296.0))))
    f = np.arange(n_features, dtype=np.uint64)
    return mix32(np.asarray(rowkey, np.uint64)[..., None] ^ f) >= thresh


def relation_mask(seed: int, rate: float, B: int, N: int):
    """(B, E, 150) multiplicative mask for c_r, slot order sender-major (main.py:72-81)."""
    m_idx, j_idx = np.nonzero(~np.eye(N, dtype=bool))
    tw = np.repeat(np.arange(B), len(m_idx))
    k = row_key(seed, 1, tw, np.tile(m_idx, B), np.tile(j_idx, B))
    scale = np.float32(1.0) / (np.float32(1.0) - np.float32(rate))
    return (keep(k, 150, rate).astype(np.float32) * scale).reshape(B, len(m_idx), 150)


def object_mask(seed: int, rate: float, B: int, N: int):
    """(B, N, 100) multiplicative mask for c_o."""
    tw = np.repeat(np.arange(B), N)
    k = row_key(seed, 2, tw, np.tile(np.arange(N), B), np.full(B * N, 0xFFFF))
    scale = np.float32(1.0) / (np.float32(1.0) - np.float32(rate))
    return (keep(k, 100, rate).astype(np.float32) * scale).reshape(B, N, 100)


def relation_mask_towers(seed: int, rate: float, tower_ids, N: int):
    """(T, E, 150) relation masks of fully connected N-box towers with the given batch tower ids
    (the engine keys a mask by the tower's id, so a sub-batch cut with `tower_ids` reproduces the
    whole batch's masks for its towers)."""
    tower_ids = np.asarray(tower_ids)
    m_idx, j_idx = np.nonzero(~np.eye(N, dtype=bool))
    tw = np.repeat(tower_ids, len(m_idx))
    k = row_key(seed, 1, tw, np.tile(m_idx, len(tower_ids)), np.tile(j_idx, len(tower_ids)))
    scale = np.float32(1.0) / (np.float32(1.0) - np.float32(rate))
    return (keep(k, 150, rate).astype(np.float32) * scale).reshape(len(tower_ids), len(m_idx), 150)


def object_mask_towers(seed: int, rate: float, tower_ids, N: int):
    """(T, N, 100) object masks for the given batch tower ids."""
    tower_ids = np.asarray(tower_ids)
    tw = np.repeat(tower_ids, N)
    k = row_key(seed, 2, tw, np.tile(np.arange(N), len(tower_ids)), np.full(len(tower_ids) * N, 0xFFFF))
    scale = np.float32(1.0) / (np.float32(1.0) - np.float32(rate))
    return (keep(k, 100, rate).astype(np.float32) * scale).reshape(len(tower_ids), N, 100)
