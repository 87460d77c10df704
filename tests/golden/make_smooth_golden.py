"""Fixtures of the SmoothQuant fold, from the REFERENCE (build container only):

    python tests/golden/make_smooth_golden.py

* ``transformer_scales.npz``: the reference's activation maxima (scales/transformer_scales.pt,
  loaded weights_only), converted to npz — data, read by the test and usable with
  ``qtx.weights.load_act_scales``.
* ``smooth_golden.npz``: the reference's ``smooth_lm`` (get_quantized_model.py:46-148)
  applied to a make_model carrying the seeded synthetic weights; for every tensor it
  changes, the float64 sum and 257 elements at fixed strided positions.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)

from make_golden import REF, SEED, import_reference  # noqa: E402


def sample(a):
    a = np.ascontiguousarray(a, np.float32).ravel()
    return a[np.linspace(0, a.size - 1, 257).astype(np.int64)]


def main():
    import torch
    torch.set_grad_enabled(False)
    sys.path.insert(0, os.path.join(REPO, "onnx-transformer_amd"))
    from qtx.weights import synthetic_state_dict

    ref = import_reference()
    scales = torch.load(os.path.join(REF, "scales", "transformer_scales.pt"), weights_only=True)
    np.savez_compressed(os.path.join(HERE, "transformer_scales.npz"),
                        **{k: v.float().numpy() for k, v in scales.items()})
    sd = synthetic_state_dict(SEED, ln_random=True)
    m = ref.model.make_model(5337, 4444, N=6)
    m.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()})
    before = {k: v.clone() for k, v in m.state_dict().items()}
    ref.gq.smooth_lm(m, scales)
    out = {}
    for k, v in m.state_dict().items():
        if not torch.equal(v, before[k]):
            out[k + "|sum"] = np.float64(v.double().sum().item())
            out[k + "|sample"] = sample(v.numpy())
    np.savez_compressed(os.path.join(HERE, "smooth_golden.npz"), **out)
    print(len(out) // 2, "tensors changed")


if __name__ == "__main__":
    main()
