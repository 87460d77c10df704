"""Empty-kernel graph chain cost inside a torch process, before/after libqtx loads."""
import ctypes as C
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "onnx-transformer_amd")
x = torch.zeros(1024, device="cuda")
P = C.CDLL("tools/libprobe.so")
P.probe_graph_us.restype = C.c_double
P.probe_graph_us.argtypes = [C.c_int, C.c_int, C.c_int]
print("after torch init  ", P.probe_graph_us(100, 20, 1))
from qtx.model import QtxModel  # noqa: E402
from qtx.weights import ModelConfig, synthetic_state_dict  # noqa: E402
m = QtxModel(synthetic_state_dict(1, ModelConfig(n_layers=1)), ModelConfig(n_layers=1))
print("after qtx model   ", P.probe_graph_us(100, 20, 1))
print("5325 nodes        ", P.probe_graph_us(5325, 3, 1))
Q = C.CDLL("onnx-transformer_amd/qtx/libqtx.so")
P.probe_graph_fn_us.restype = C.c_double
P.probe_graph_fn_us.argtypes = [C.c_void_p, C.c_int, C.c_int]
fn = C.cast(Q._ZN3qtx10launch_nopEP12ihipStream_t, C.c_void_p)
print("libqtx launch_nop ", P.probe_graph_fn_us(fn, 100, 20))
