import sys, numpy as np, torch
sys.path.insert(0, '.'); sys.path.insert(0, 'onnx-transformer_amd')
from qtx.model import QtxModel
from qtx.weights import synthetic_state_dict
g = np.load('tests/golden/golden_ops.npz')
sd = synthetic_state_dict(20241223, ln_random=True)
m = QtxModel(sd)
ids = torch.from_numpy(g['emb_ids']).cuda()
out = m.embed(ids, 'src').cpu().numpy()
np.save('gpurun_out/emb_gpu.npy', out)
print('mismatch', (out != g['emb_ref']).sum())
