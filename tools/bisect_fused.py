"""Debug aid: compare greedy decode paths (fused / unfused / debug tail) with the oracle."""
import os
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "onnx-transformer_amd")
from oracle.qtx_oracle import OracleModel  # noqa: E402
from qtx.decode import greedy_decode  # noqa: E402
from qtx.model import QtxModel  # noqa: E402
from qtx.weights import ModelConfig, synthetic_state_dict  # noqa: E402

L = int(os.environ.get("NL", "1"))
cfg = ModelConfig(n_layers=L)
sd = synthetic_state_dict(5, cfg=cfg, ln_random=True)
g = np.load("tests/golden/golden_model.npz")
src, mask = g["src"], g["src_mask"]
om = OracleModel(sd, n_layers=L)
ref = om.greedy_decode(src, mask, max_len=6)
m = QtxModel(sd, cfg)
for env in [{}, {"QTX_NO_GRAPH": "1"}, {"QTX_UNFUSED": "1"}, {"QTX_DBG_TAIL": "1", "QTX_NO_GRAPH": "1"}]:
    for k in ("QTX_NO_GRAPH", "QTX_UNFUSED", "QTX_DBG_TAIL"):
        os.environ.pop(k, None)
    os.environ.update(env)
    ys = greedy_decode(m, src, mask, 6, 0)
    print(env, "match" if np.array_equal(ys, ref) else f"MISMATCH\n{ys}\n{ref}")
