"""Build the product library's sources with extra compiler flags into another file, for
A/B runs (tools/lib_ab.py, QTX_LIB_PATH) — no -DQTX_DIAG, so the kernels are the product's:

    python tools/build_variant.py onnx-transformer_amd/qtx/libqtx_v.so -fno-slp-vectorize
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "onnx-transformer_amd"))
from qtx import _build  # noqa: E402


def main():
    out, extra = os.path.abspath(sys.argv[1]), sys.argv[2:]
    objdir = os.path.join(REPO, "onnx-transformer_amd", "qtx", "build_obj_variant" + os.environ.get("QTX_VARIANT_TAG", ""))
    os.makedirs(objdir, exist_ok=True)
    cflags = [f for f in _build.FLAGS if f != "-shared"] + extra

    def one(src):
        obj = os.path.join(objdir, os.path.splitext(os.path.basename(src))[0] + ".o")
        r = subprocess.run([_build.hipcc(), *cflags, "-c", "-o", obj, os.path.join(_build.CSRC, src)],
                           capture_output=True, text=True)
        if r.returncode:
            raise SystemExit(f"{src}: {r.stderr[-3000:]}")
        return obj
    with ThreadPoolExecutor(max_workers=8) as ex:
        objs = list(ex.map(one, _build.SOURCES))
    r = subprocess.run([_build.hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, *objs],
                       capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(r.stderr[-3000:])
    print(out)


if __name__ == "__main__":
    main()
