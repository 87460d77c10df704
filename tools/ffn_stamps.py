"""Per-phase in-kernel cycles of the fused FFN launch (k_ffn_fused) at cfg3 from s_memtime
stamps (thread 0 of each workgroup; a diagnostic build, never the product):
    python tools/ffn_stamps.py build          # here: libqtx_stamps.so with -DQTX_STAMPS
    python tools/ffn_stamps.py                # on the GPU box
Slots: 0 start, 1 prologue done, 2 pass 1 done, 3 pass 2 done, 4 end; 8..11 pass 2's
accumulated ring waits, FFN1 MFMA, hidden epilogue, FFN2 MFMA (wave 0)."""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, R + "/onnx-transformer_amd", R + "/tools"]
STAMP_LIB = os.path.join(R, "onnx-transformer_amd/qtx/libqtx_stamps.so")


def build():
    from qtx import _build
    cmd = [_build.hipcc(), *_build.FLAGS, "-DQTX_STAMPS", "-o", STAMP_LIB,
           *[os.path.join(_build.CSRC, s) for s in _build.SOURCES]]
    subprocess.run(cmd, check=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        build()
        return
    os.environ["QTX_LIB_PATH"] = STAMP_LIB
    import torch
    import ffn_ab
    fused, _, _ = ffn_ab.launches()
    buf = torch.zeros((4096, 16), dtype=torch.int64, device="cuda")
    C.CDLL(STAMP_LIB).qtx_debug_set_stamps_ffn(C.c_void_p(buf.data_ptr()))
    for _ in range(20):      # >= a second of back-to-back launches: the clock under load
        fused()
    torch.cuda.synchronize()
    buf.zero_()
    fused()
    torch.cuda.synchronize()
    s = buf[:256].cpu().numpy()
    d = np.diff(s[:, :5], axis=1)
    names = ["prologue", "pass 1", "pass 2", "epilogue"]
    for i, n in enumerate(names):
        print(f"{n:10s} median {np.median(d[:, i]):9.0f} cycles  (min {d[:, i].min()}, max {d[:, i].max()})")
    print(f"total      median {np.median(s[:, 4] - s[:, 0]):9.0f} cycles; start spread {s[:, 0].max() - s[:, 0].min()}")
    for i, n in zip(range(8, 12), ["ring waits", "FFN1 MFMA", "h epilogue", "FFN2 MFMA"]):
        print(f"  pass 2 {n:12s} median {np.median(s[:, i]):9.0f} cycles")


if __name__ == "__main__":
    main()
