"""Build libspwgnn_hip.so in-tree for gfx950 (hipcc, no JIT cache)."""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
INCLUDE = HERE.parent / "include"
LIB = HERE / "libspwgnn_hip.so"
OBJDIR = HERE / "csrc" / "build"
# A/B and diagnosis builds (e.g. SPWGNN_CFLAGS=-DSPWGNN_DIAG): SPWGNN_BUILD_OUT names the library to
# write instead of the in-tree one; its objects go to a directory of their own
if os.environ.get("SPWGNN_BUILD_OUT"):
    LIB = Path(os.environ["SPWGNN_BUILD_OUT"]).resolve()
    OBJDIR = HERE / "csrc" / ("build_" + LIB.stem)
SOURCES = ["host.cpp", "api.hip", "kernels_fwd.hip", "kernels_bwd.hip", "kernels_misc.hip", "kernels_team.hip"]
HEADERS = ["spwgnn_layout.h", "device_common.h", "gemm_blocks.h", "kernels.h"]
ARCH = os.environ.get("SPWGNN_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: libspwgnn_hip.so cannot be built")


def _flags(src: str):
    # -fno-slp-vectorize: packed f32 VALU (v_pk_add_f32 …) issues slower than scalar pairs beside
    # the matrix pipe (MI355X_MICROARCH.md; measured −2 % step time)
    f = ["-O3", "-std=c++17", "-fPIC", "-fno-slp-vectorize", f"-I{INCLUDE}", f"-I{CSRC}"]
    f += os.environ.get("SPWGNN_CFLAGS", "").split()
    if src.endswith(".hip"):
        f += [f"--offload-arch={ARCH}", "-x", "hip"]
    return f


def _stale(obj: Path, src: Path) -> bool:
    if not obj.exists():
        return True
    deps = [src] + [CSRC / h for h in HEADERS] + [INCLUDE / "spwgnn.h"]
    t = obj.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> Path:
    OBJDIR.mkdir(parents=True, exist_ok=True)
    LIB.parent.mkdir(parents=True, exist_ok=True)
    hipcc = _hipcc()
    jobs = []
    objs = []
    for s in SOURCES:
        src = CSRC / s
        obj = OBJDIR / (s.rsplit(".", 1)[0] + ".o")
        objs.append(obj)
        if force or _stale(obj, src):
            jobs.append([hipcc, *_flags(s), "-c", str(src), "-o", str(obj)])
    if jobs:
        with cf.ThreadPoolExecutor(max_workers=min(len(jobs), 8)) as ex:
            results = list(ex.map(lambda cmd: subprocess.run(cmd, capture_output=True, text=True), jobs))
        for cmd, r in zip(jobs, results):
            if verbose or r.returncode != 0:
                sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
            if r.returncode != 0:
                raise RuntimeError(f"hipcc failed on {cmd[-3]}")
    if force or jobs or not LIB.exists() or any(o.stat().st_mtime > LIB.stat().st_mtime for o in objs):
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(LIB)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stdout + r.stderr)
            raise RuntimeError("link of libspwgnn_hip.so failed")
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose="-v" in sys.argv))
