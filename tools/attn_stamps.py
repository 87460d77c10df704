"""Phase cycles of k_attn_encq (stamp build): staging, heads, quant; head 0: scores,
softmax, PV.  QTX_LIB_PATH=onnx-transformer_amd/qtx/libqtx_stamps.so python tools/attn_stamps.py"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "onnx-transformer_amd")
from qtx import _lib  # noqa: E402

L = _lib.lib(build=False)
raw = C.CDLL(os.environ["QTX_LIB_PATH"])
buf = torch.zeros((4096, 16), dtype=torch.int64, device="cuda")
raw.qtx_debug_set_stamps_attn(C.c_void_p(buf.data_ptr()))
B, S = 256, 128
rng = np.random.default_rng(0)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
P = lambda t: C.c_void_p(t.data_ptr())
q, k, v = (T(rng.integers(-127, 128, (B, S, 512)).astype(np.int8)) for _ in range(3))
sq, sk, sv = (T(rng.uniform(0.002, 0.03, (B, S)).astype(np.float32)) for _ in range(3))
km = T(np.ones((B, S), np.uint8))
ctx8 = torch.empty((B, S, 512), dtype=torch.int8, device="cuda")
sc = torch.empty((B, S), device="cuda")
for _ in range(3):
    buf.zero_()
    L.qtx_attention_i8_quant(P(q), P(sq), P(k), P(sk), P(v), P(sv), P(km), B, S, P(ctx8), P(sc), C.c_void_p(0))
    torch.cuda.synchronize()
st = buf[:B].cpu().numpy().astype(np.float64)
d = lambda a, b: np.median(st[:, b] - st[:, a])
print("staging", d(0, 1), "heads", d(1, 2), "quant+store", d(2, 3))
print("per head iteration (wave 0, after the barrier):", [round(d(4 + h, 5 + h)) for h in range(8)],
      "last PV", d(12, 2))
pw = buf.view(-1)[4096:4096 + 4 * B * 8].cpu().numpy().reshape(B, 8, 4).astype(np.float64)
for i, name in enumerate(["barrier wait", "PV", "scores+softmax", "V convert"]):
    print(f"{name:15s} over the head loop per wave (median over WGs):", np.median(pw[:, :, i], axis=0).round())
print("total span", (st[:, 3].max() - st[:, 0].min()), "cyc; median WG", d(0, 3))
