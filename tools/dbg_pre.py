import os, sys, numpy as np
R='/root/repo'; sys.path[:0]=[R, R+'/onnx-transformer_amd', R+'/tests']
import torch
from qtx.model import QtxModel
from qtx.weights import ModelConfig, synthetic_state_dict
from qtx.decode import greedy_decode
from test_gpu_configs import _cfg2_src
m = QtxModel(synthetic_state_dict(20241223, ln_random=True), ModelConfig())
src, mk = _cfg2_src(505, 256)
os.environ["QTX_PRE_GRAPH"] = "0"
base = greedy_decode(m, src[:32], mk[:32], 72, 0)
for part in ("0", "1", "2"):
    os.environ["QTX_PRE_GRAPH"] = "1"; os.environ["QTX_PRE_PART"] = part
    m._tls.ws = None
    a = greedy_decode(m, src[:32], mk[:32], 72, 0)
    b = greedy_decode(m, src, mk, 72, 0)
    c = greedy_decode(m, src[:32], mk[:32], 72, 0)
    d = greedy_decode(m, src[:32], mk[:32], 72, 0)
    print(f"part={part}: a {np.array_equal(a, base)} c {np.array_equal(c, base)} d {np.array_equal(d, base)}", flush=True)
