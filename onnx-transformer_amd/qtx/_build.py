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
SOURCES = ["qtx_kernels.hip", "qtx_decode.hip", "qtx_gemm.hip", "qtx_attn.hip", "qtx_api.hip"]
HEADERS = ["qtx_common.h", "qtx_kernels.h"]

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


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile the library if any source is newer; returns its path."""
    if not force and up_to_date():
        return LIB
    tmp = LIB + ".tmp"
    cmd = [hipcc(), *FLAGS, "-o", tmp, *[os.path.join(CSRC, s) for s in SOURCES]]
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed ({r.returncode}):\n{r.stderr[-4000:]}")
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force=True, verbose=True))
