"""qtx — MI355X-native (gfx950) W8A8/W4A8 inference path for the reference's quantized
IWSLT14 transformer (gebegebegebe/onnx-transformer).

Public surface mirrors the reference's entry points:
  InferenceSession(path).run(None, feeds)      ~ onnxruntime.InferenceSession
  run_module(module, feeds, ...)               ~ onnx_optimized_inference.run_module
  greedy_decode(model, src, src_mask, max_len, start_symbol)
"""
from .weights import (BOS, DEFAULT_SEED, EOS, PAD, UNK, ModelConfig, load_checkpoint,
                      positional_table, synthetic_state_dict, tensor_order)

__all__ = ["BOS", "EOS", "PAD", "UNK", "DEFAULT_SEED", "ModelConfig", "load_checkpoint",
           "positional_table", "synthetic_state_dict", "tensor_order", "QtxModel",
           "InferenceSession", "run_module", "set_default_model", "greedy_decode",
           "make_src_mask", "lib"]


def __getattr__(name):
    # lazy: importing qtx must not require a GPU; using the compute entry points does.
    if name in ("QtxModel",):
        from .model import QtxModel
        return QtxModel
    if name in ("InferenceSession", "run_module", "set_default_model"):
        from . import session
        return getattr(session, name)
    if name in ("greedy_decode", "make_src_mask"):
        from . import decode
        return getattr(decode, name)
    if name == "lib":
        from ._lib import lib
        return lib
    raise AttributeError(name)
