"""Flat parameter buffer ↔ Keras-layout tensors.

The four MLPs of the reference (rm, om, rmp, omp — src/Networks.py:46-50; Dense stacks of
src/Blocks.py:20-28 / 60-68) are stored in one flat fp32 buffer whose layout is defined by the
C library (``spwgnn_param_tensor``): kernels in Keras (in, out) row-major layout, biases (out,),
each tensor on a 64-float boundary. One flat buffer = one gradient bucket for the all-reduce and
one Adam launch.
"""
from __future__ import annotations

import math
from typing import Dict, List, Tuple

import numpy as np
import torch

from . import _lib

# Networks.py:46-50 (mirrors the C table; checked against it in tests)
MLP_SPECS = {
    "rm": (2, [150, 150, 150, 150]),
    "om": (2, [100, 100]),
    "rmp": (350, [150, 150, 100]),
    "omp": (300, [100, 101]),
}


def layout() -> List[Tuple[str, int, Tuple[int, ...]]]:
    """[(name, offset, shape)] from the C library; bias shapes are (cols,)."""
    out = []
    for name, off, rows, cols in _lib.param_tensors():
        shape = (cols,) if name.endswith("bias") else (rows, cols)
        out.append((name, off, shape))
    return out


def flat_size() -> int:
    return int(_lib.lib().spwgnn_param_count())


def real_size() -> int:
    return int(_lib.lib().spwgnn_param_real_count())


def to_flat(params: Dict[str, np.ndarray], device="cpu", dtype=torch.float32) -> torch.Tensor:
    flat = torch.zeros(flat_size(), dtype=dtype)
    for name, off, shape in layout():
        arr = torch.as_tensor(np.asarray(params[name]), dtype=dtype).reshape(-1)
        if arr.numel() != int(np.prod(shape)):
            raise ValueError(f"{name}: expected {shape}, got {tuple(np.asarray(params[name]).shape)}")
        flat[off:off + arr.numel()] = arr
    return flat.to(device)


def from_flat(flat: torch.Tensor) -> Dict[str, np.ndarray]:
    f = flat.detach().to("cpu", torch.float64).numpy()
    return {name: f[off:off + int(np.prod(shape))].reshape(shape).copy() for name, off, shape in layout()}


def glorot_uniform(seed: int = 0) -> Dict[str, np.ndarray]:
    """Keras Dense defaults (Blocks.py:23-27): glorot_uniform kernels, zero biases."""
    rng = np.random.default_rng(seed)
    out = {}
    for name, _, shape in layout():
        if name.endswith("kernel"):
            lim = math.sqrt(6.0 / (shape[0] + shape[1]))
            out[name] = rng.uniform(-lim, lim, size=shape).astype(np.float32)
        else:
            out[name] = np.zeros(shape, np.float32)
    return out
