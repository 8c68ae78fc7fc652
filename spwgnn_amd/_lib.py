"""ctypes binding of libspwgnn_hip.so (the C-ABI in include/spwgnn.h).

The product path has no fallback: if the library is missing or cannot be loaded, every entry
point raises. Device pointers are passed as plain integers (torch ``data_ptr()``).
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path
from typing import Optional

_LIB_PATH = Path(__file__).resolve().parent / "libspwgnn_hip.so"
_lib: Optional[C.CDLL] = None


class SpwgnnError(RuntimeError):
    pass


class ParamInfo(C.Structure):
    _fields_ = [("name", C.c_char_p), ("offset", C.c_int64), ("rows", C.c_int32), ("cols", C.c_int32)]


class PlanSizes(C.Structure):
    _fields_ = [("n_wtiles", C.c_int32), ("n_eblocks", C.c_int32), ("nw_max", C.c_int32)]


class BatchC(C.Structure):
    _fields_ = [
        ("n_towers", C.c_int32), ("n_nodes", C.c_int32), ("n_wtiles", C.c_int32), ("n_eblocks", C.c_int32),
        ("nw_max", C.c_int32), ("flags", C.c_int32),
        ("pos", C.c_void_p), ("prop", C.c_void_p), ("node_tower", C.c_void_p), ("node_local", C.c_void_p),
        ("wtile", C.c_void_p), ("edge_src", C.c_void_p), ("edge_dst", C.c_void_p), ("blk_csr", C.c_void_p),
    ]


class PrologueC(C.Structure):
    """spwgnn_prologue: a replayed step's batch upload and key/step advance, run by the forward's
    first launch."""
    _fields_ = [("copy_src", C.c_void_p), ("copy_dst", C.c_void_p), ("copy_bytes", C.c_int64),
                ("key", C.c_void_p), ("step", C.c_void_p), ("mode", C.c_int32), ("rank", C.c_int32),
                ("seed", C.c_uint64)]


class RunC(C.Structure):
    _fields_ = [("mp_steps", C.c_int32), ("training", C.c_int32), ("dropout", C.c_float), ("math", C.c_int32),
                ("seed", C.c_uint64), ("prof_kernel", C.c_int32), ("prof_count", C.c_int32),
                ("prof_events", C.c_void_p), ("seed_dev", C.c_void_p), ("prologue", C.c_void_p),
                ("grads_early_event", C.c_void_p)]


K_EDGE_FWD, K_NODE_FWD, K_EDGE_BWD, K_NODE_BWD, K_ENC_EDGE, K_ENC_EDGE_BWD, K_WGRAD_W2, K_DA = 1, 2, 3, 4, 5, 6, 7, 8
K_WGRAD_WS, K_ENC_NODE, K_ENC_NODE_BWD = 9, 10, 11
MATH_F32, MATH_X6, MATH_BF16 = 0, 1, 2
STEP_KEY_COUNTER, STEP_KEY_SPLITMIX = 0, 1
ABI_VERSION = 6        # SPWGNN_ABI_VERSION this binding's structs follow
BATCH_RECV_BLOCKS = 1  # spwgnn_batch.flags: a receiver-block plan (spwgnn_plan_fill_recv)
READOUT_SUM_PROB, READOUT_MEAN_PROB, READOUT_SUM_LOGIT, READOUT_MEAN_LOGIT = 0, 1, 2, 3


def _declare(lib: C.CDLL) -> None:
    i32, i64, vp, f32 = C.c_int32, C.c_int64, C.c_void_p, C.c_float
    sig = {
        "spwgnn_version": (i32, []),
        "spwgnn_struct_size": (i32, [i32]),
        "spwgnn_strerror": (C.c_char_p, [i32]),
        "spwgnn_param_tensor_count": (i32, []),
        "spwgnn_param_count": (i64, []),
        "spwgnn_param_real_count": (i64, []),
        "spwgnn_param_tensor": (i32, [i32, C.POINTER(ParamInfo)]),
        "spwgnn_dense_to_edges": (i32, [vp, vp, i32, i32, vp, vp, vp, i64, C.POINTER(i64), vp]),
        "spwgnn_plan_size": (i32, [i32, vp, vp, i32, C.POINTER(PlanSizes)]),
        "spwgnn_plan_fill": (i32, [i32, vp, vp, vp, vp, i32, C.POINTER(PlanSizes), vp, vp, vp, vp, vp]),
        "spwgnn_plan_size_cap": (i32, [i32, vp, vp, i32, C.POINTER(PlanSizes)]),
        "spwgnn_plan_order": (i32, [i32, vp, vp, i32, vp]),
        "spwgnn_plan_fill_cap": (i32, [i32, vp, vp, vp, vp, vp, i32, C.POINTER(PlanSizes), vp, vp, vp, vp, vp]),
        "spwgnn_plan_size_recv": (i32, [i32, vp, i32, C.POINTER(PlanSizes)]),
        "spwgnn_plan_fill_recv": (i32, [i32, vp, vp, vp, vp, i32, C.POINTER(PlanSizes), vp, vp, vp, vp, vp]),
        "spwgnn_workspace_bytes": (i64, [i32, i32, i32, i32]),
        "spwgnn_fused_path": (i32, [C.POINTER(BatchC), C.POINTER(RunC)]),
        "spwgnn_team_max_blocks": (i32, [i32]),
        "spwgnn_host_device_ptr": (i32, [vp, C.POINTER(vp)]),
        "spwgnn_forward": (i32, [vp, C.POINTER(BatchC), C.POINTER(RunC), vp, i64, vp, vp]),
        "spwgnn_backward": (i32, [vp, C.POINTER(BatchC), C.POINTER(RunC), vp, i64, vp, vp, vp, vp]),
        "spwgnn_bce_scratch_bytes": (i64, [i64]),
        "spwgnn_bce": (i32, [vp, vp, i64, vp, vp, vp, vp]),
        "spwgnn_bce_accumulate": (i32, [vp, vp, i64, vp, vp, vp, vp, vp, vp]),
        "spwgnn_bce_backward": (i32, [vp, vp, vp, vp, i64, vp, vp, i64, vp, vp, vp, vp, vp, vp, vp, vp]),
        "spwgnn_adam": (i32, [vp, vp, vp, vp, i64, i32, f32, f32, f32, f32, f32, f32, vp]),
        "spwgnn_adam_dev": (i32, [vp, vp, vp, vp, i64, vp, vp, i32, f32, f32, f32, f32, f32, vp]),
        "spwgnn_adam_lr_table": (i32, [f32, f32, f32, i32, vp]),
        "spwgnn_step_advance": (i32, [vp, vp, i32, C.c_uint64, i32, vp]),
        "spwgnn_sigmoid": (i32, [vp, vp, i64, vp]),
        "spwgnn_copy_in": (i32, [vp, vp, i64, vp]),
        "spwgnn_accumulate_out3": (i32, [vp, vp, vp, vp]),
        "spwgnn_tower_readout": (i32, [vp, vp, i32, i32, vp, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args


def lib() -> C.CDLL:
    """Load (once) the in-tree HIP library. Raises if it is absent: there is no fallback."""
    global _lib
    if _lib is None:
        path = Path(os.environ.get("SPWGNN_LIB", _LIB_PATH))
        if not path.exists():
            raise SpwgnnError(f"{path} not found — build it with `python -m spwgnn_amd.build` "
                              "(the HIP path has no CPU fallback)")
        lib_ = C.CDLL(str(path), mode=C.RTLD_GLOBAL)
        _declare(lib_)
        if lib_.spwgnn_version() != ABI_VERSION:
            raise SpwgnnError(f"{path} implements ABI {lib_.spwgnn_version()}, this binding expects {ABI_VERSION}: "
                              "rebuild with `python -m spwgnn_amd.build`")
        for which, st in enumerate((BatchC, RunC, PlanSizes, ParamInfo)):
            if lib_.spwgnn_struct_size(which) != C.sizeof(st):
                raise SpwgnnError(f"{path} was built with a different {st.__name__} layout "
                                  f"({lib_.spwgnn_struct_size(which)} vs {C.sizeof(st)} bytes): rebuild it")
        _lib = lib_
    return _lib


_hip = None


def hip_runtime() -> C.CDLL:
    """The HIP runtime already mapped into this process — the copy torch and libspwgnn_hip.so run on —
    opened by its mapped path (never a second runtime found by soname). For the event calls of the
    bench's timing hook."""
    global _hip
    if _hip is None:
        lib()
        with open("/proc/self/maps") as f:
            paths = {ln.split()[-1] for ln in f if "libamdhip64.so" in ln}
        if not paths:
            raise SpwgnnError("the HIP runtime is not mapped into this process")
        _hip = C.CDLL(sorted(paths)[0])
    return _hip


def host_device_ptr(ptr: int) -> int:
    """spwgnn_host_device_ptr: the device address of pinned, device-mapped host memory."""
    out = C.c_void_p()
    check(lib().spwgnn_host_device_ptr(C.c_void_p(ptr), C.byref(out)), "host_device_ptr (not device-mapped?)")
    return int(out.value)


def check(status: int, what: str = "") -> None:
    if status != 0:
        msg = lib().spwgnn_strerror(status).decode()
        raise SpwgnnError(f"{what}: {msg} (status {status})")


def param_tensors():
    L = lib()
    out = []
    info = ParamInfo()
    for i in range(L.spwgnn_param_tensor_count()):
        check(L.spwgnn_param_tensor(i, C.byref(info)), "param_tensor")
        out.append((info.name.decode(), int(info.offset), int(info.rows), int(info.cols)))
    return out
