"""Build libqtx.so (the HIP/gfx950 kernels + C-ABI) in-tree with hipcc.

The shared library is written next to this file so it travels with the repository
snapshot to the GPU box (the JIT caches under ~/.cache do not).
"""
from __future__ import annotations

import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "csrc")
REPO = os.path.dirname(os.path.dirname(HERE))
LIB = os.path.join(HERE, "libqtx.so")
SOURCES = ["qtx_kernels.hip", "qtx_decode.hip", "qtx_gemm.hip", "qtx_wsgemm.hip", "qtx_attn.hip",
           "qtx_ffn.hip", "qtx_api.hip", "qtx_knobs.hip"]
# measured-negative kernel variants and their switches: compiled only into the diagnostic
# library (build(extra=...) -> libqtx_diag.so, with -DQTX_DIAG), never into libqtx.so
DIAG_SOURCES = ["diag/qtx_wsgemm_diag.hip"]   # csrc/diag/: outside the product sources
HEADERS = ["qtx_common.h", "qtx_kernels.h", "qtx_ws.h", "qtx_knobs.h"]

# -ffp-contract=off: every float op is a separate IEEE op (the numerics contract,
# DESIGN.md §3); HIP keeps correctly rounded fp32 '/' and sqrtf by default.
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
         "-ffp-contract=off", "-fno-fast-math", "-Wall"]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the qtx HIP extension cannot be built")


def _inputs():
    files = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    files.append(os.path.join(REPO, "include", "qtx.h"))
    files.append(os.path.abspath(__file__))
    return files


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(f) <= t for f in _inputs())


def build(force: bool = False, verbose: bool = False, extra=()) -> str:
    """Compile the library if any source is newer; returns its path.  Each source is
    compiled to a relocatable gfx950 object in parallel (-fgpu-rdc is not needed: no
    cross-file device symbols), then linked into one shared library."""
    from concurrent.futures import ThreadPoolExecutor
    out = LIB if not extra else LIB.replace(".so", "_diag.so")
    extra = list(extra) + (["-DQTX_DIAG"] if extra and "-DQTX_DIAG" not in extra else [])
    if not force and not extra and up_to_date():
        return LIB
    objdir = os.path.join(HERE, "build_obj")
    os.makedirs(objdir, exist_ok=True)
    cflags = [f for f in FLAGS if f != "-shared"] + list(extra)

    def compile_one(src):
        obj = os.path.join(objdir, os.path.splitext(os.path.basename(src))[0] + ("_x" if extra else "") + ".o")
        cmd = [hipcc(), *cflags, "-c", "-o", obj, os.path.join(CSRC, src)]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src} ({r.returncode}):\n{r.stderr[-4000:]}")
        return obj

    srcs = SOURCES + (DIAG_SOURCES if extra else [])
    with ThreadPoolExecutor(max_workers=min(len(srcs), os.cpu_count() or 1)) as ex:
        objs = list(ex.map(compile_one, srcs))
    tmp = out + ".tmp"
    cmd = [hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", tmp, *objs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc link failed ({r.returncode}):\n{r.stderr[-4000:]}")
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    print(build(force=True, verbose=True))
