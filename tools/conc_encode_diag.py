"""Diagnose tests/test_gpu_configs.py::test_cfg3_encoder_split_two_threads: two threads
share one model handle, each encoding its own cfg3 batch 3x on its own stream; report
which outputs / sentences differ from a single-stream encode and the device status word.
usage: python tools/conc_encode_diag.py [reps]"""
import os
import sys
import threading

import numpy as np
import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "onnx-transformer_amd")]
from qtx.model import QtxModel  # noqa: E402
from qtx.weights import synthetic_state_dict  # noqa: E402

m = QtxModel(synthetic_state_dict(1))
rng = np.random.default_rng(303)
x = rng.standard_normal((256, 128, 512)).astype(np.float32)
mk = np.ones((256, 128), np.uint8)
mk[::16, 100:] = 0
ref = m.encode(torch.from_numpy(x).cuda(), torch.from_numpy(mk).cuda()).cpu().numpy()
ref2 = ref[::-1]
x2, mk2 = np.ascontiguousarray(x[::-1]), np.ascontiguousarray(mk[::-1])
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    res, errs = {}, []

    def run(tag, xx, mm):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                xd, md = torch.from_numpy(xx).cuda(), torch.from_numpy(mm).cuda()
                outs = [m.encode(xd, md) for _ in range(3)]
                s.synchronize()
                m.check()
            res[tag] = [o.cpu().numpy() for o in outs]
        except Exception as e:
            errs.append(repr(e))
    th = [threading.Thread(target=run, args=("a", x, mk)), threading.Thread(target=run, args=("b", x2, mk2))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    bad = []
    for tag, r in (("a", ref), ("b", ref2)):
        for i, o in enumerate(res.get(tag, [])):
            rows = np.nonzero((o != r).any(-1))
            if len(rows[0]):
                sents = sorted(set(rows[0].tolist()))
                bad.append((tag, i, len(rows[0]), sents[:8]))
    print(f"rep {rep}: errs={errs} bad={bad}", flush=True)
