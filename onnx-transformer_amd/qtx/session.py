"""Drop-in replacements for the reference's ONNX execution entry points.

* :class:`InferenceSession` — ``ort.InferenceSession(path).run(None, feeds) -> [ndarray]``
  as called at reference/onnx_reference_inference.py:625-626 (encoder) and :633-639
  (decoder).  The graph path only selects encoder vs decoder (the ``*.onnx`` files are not
  needed: the arithmetic is implemented natively); weights come from a :class:`QtxModel`.
* :func:`run_module` — ``run_module(module, input_values, module_filepath,
  module_weight_dict, module_graph, inject_parameters=None) -> (output_tensors,
  weight_dict)`` of onnx_optimized_inference.py:297-304 (reference variant
  reference/onnx_inference.py:110-113).  ``output_tensors`` is ``{"global_out": ndarray}``
  and the feeds plus the output are stored into ``weight_dict`` by name, as the node
  executor does (onnx_optimized_inference.py:57,300-301).

Feed names, shapes and dtypes are those of the exported graphs.
Missing or mis-shaped feeds raise ``ValueError`` (ORT raises InvalidArgument).
"""
from __future__ import annotations

import numpy as np

from .model import QtxModel, to_u8_mask

ENCODER_FEEDS = ("global_in", "global_in_1")
DECODER_FEEDS = ("global_in", "global_in_1", "global_in_2", "global_in_3")

_default_model: QtxModel | None = None


def set_default_model(model: QtxModel):
    """Model used by sessions / run_module calls that do not pass one."""
    global _default_model
    _default_model = model


def _module_kind(name: str) -> str:
    n = str(name).lower()
    if "encoder" in n:
        return "encoder"
    if "decoder" in n:
        return "decoder"
    raise ValueError(f"unknown module {name!r}: expected an encoder or decoder graph")


def _as_torch(a, device, dtype=None):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(a)) if isinstance(a, np.ndarray) else a
    if dtype is not None:
        t = t.to(dtype)
    return t.to(device).contiguous()


def _check(feeds, names):
    missing = [n for n in names if n not in feeds]
    if missing:
        raise ValueError(f"Required inputs ({missing}) are missing from input feed "
                         f"({sorted(feeds)}).")


def _shape(a):
    return tuple(a.shape)


def run_encoder(model: QtxModel, feeds: dict, fault=None, trace=None):
    """global_in f32 [B,S,512], global_in_1 bool [B,1,S] -> global_out f32 [B,S,512].
    trace: None (the fused forward) or a dict that the op-by-op traced executor
    (qtx.trace) fills with the named intermediates ("weights": the weight codes too)."""
    import torch
    _check(feeds, ENCODER_FEEDS)
    x, m = feeds["global_in"], feeds["global_in_1"]
    if len(_shape(x)) != 3 or _shape(x)[2] != model.cfg.d_model:
        raise ValueError(f"global_in: expected [B,S,{model.cfg.d_model}], got {_shape(x)}")
    B, S, _ = _shape(x)
    if int(np.prod(_shape(m))) != B * S:
        raise ValueError(f"global_in_1: expected [B,1,S]=[{B},1,{S}], got {_shape(m)}")
    xd = _as_torch(x, model.device, torch.float32)
    md = to_u8_mask(m, model.device).reshape(B, S)
    if trace is not None:
        from .trace import trace_encoder
        with torch.cuda.device(model.device):
            out, names = trace_encoder(model, xd, md, weights=bool(trace.pop("weights", False)))
        trace.update(names)
        return out
    return model.encode(xd, md, fault=fault)


def run_decoder(model: QtxModel, feeds: dict, fault=None, trace=None):
    """global_in [B,T,512], global_in_1 memory [B,S,512], global_in_2 [B,1,S],
    global_in_3 int64 [1,T,T] (or [B,T,T]) -> global_out [B,T,512]."""
    import torch
    _check(feeds, DECODER_FEEDS)
    y, mem, sm, tm = (feeds[n] for n in DECODER_FEEDS)
    if len(_shape(y)) != 3 or _shape(y)[2] != model.cfg.d_model:
        raise ValueError(f"global_in: expected [B,T,{model.cfg.d_model}], got {_shape(y)}")
    B, T, _ = _shape(y)
    if len(_shape(mem)) != 3 or _shape(mem)[0] != B or _shape(mem)[2] != model.cfg.d_model:
        raise ValueError(f"global_in_1: expected [{B},S,{model.cfg.d_model}], got {_shape(mem)}")
    S = _shape(mem)[1]
    if int(np.prod(_shape(sm))) != B * S:
        raise ValueError(f"global_in_2: expected [{B},1,{S}], got {_shape(sm)}")
    ts = _shape(tm)
    if ts[-2:] != (T, T) or int(np.prod(ts)) not in (T * T, B * T * T):
        raise ValueError(f"global_in_3: expected [1,{T},{T}], got {ts}")
    yd = _as_torch(y, model.device, torch.float32)
    md = _as_torch(mem, model.device, torch.float32)
    smd = to_u8_mask(sm, model.device).reshape(B, S)
    tmd = to_u8_mask(tm, model.device)
    tmd = tmd.reshape(T, T) if int(np.prod(ts)) == T * T else tmd.reshape(B, T, T)
    if trace is not None:
        from .trace import trace_decoder
        with torch.cuda.device(model.device):
            out, names = trace_decoder(model, yd, md, smd, tmd,
                                       weights=bool(trace.pop("weights", False)))
        trace.update(names)
        return out
    return model.decode(yd, md, smd, tmd, fault=fault)


class InferenceSession:
    """Session-shaped front end: ``InferenceSession(path).run(None, feeds)``."""

    def __init__(self, path_or_module: str, model: QtxModel | None = None, **_ignored):
        self.kind = _module_kind(path_or_module)
        self.model = model or _default_model
        if self.model is None:
            raise ValueError("no QtxModel: pass model= or call qtx.set_default_model()")

    def get_inputs(self):
        return list(ENCODER_FEEDS if self.kind == "encoder" else DECODER_FEEDS)

    def get_outputs(self):
        return ["global_out"]

    def run_torch(self, feeds: dict):
        """Same as run() but returns the device tensor (no host copy)."""
        fn = run_encoder if self.kind == "encoder" else run_decoder
        return fn(self.model, feeds)

    def run(self, output_names, input_feed: dict):
        t = self.run_torch(input_feed)
        self.model.check()
        out = t.cpu().numpy()
        if output_names not in (None, [], ["global_out"]):
            raise ValueError(f"unknown outputs {output_names}; the graph has ['global_out']")
        return [out]


def run_module(module, input_values, module_filepath=None, module_weight_dict=None,
               module_graph=None, inject_parameters=None, model: QtxModel | None = None,
               rng=None, expose_intermediates=False):
    """onnx_optimized_inference.py:297-304 contract: returns (output_tensors, weight_dict).

    expose_intermediates: True stores every quantizer's int8 codes (``Round_<n>_out0``,
    float32 as the graph's Round nodes produce them, + ``Round_<n>_scale``) and every
    QuantLinear MatMul's accumulators (``MatMul_<n>_out0``) in weight_dict under the
    exported graph's names, as the reference's node-by-node executor does
    (onnx_optimized_inference.py:57); "weights" adds the weight codes.  The module then
    runs op by op (qtx.trace; same result bit for bit) instead of fused.

    inject_parameters: the reference's dict (inject_type INPUT/WEIGHT/INPUT16/WEIGHT16/
    RANDOM/RANDOM_BITFLIP, faulty_operation_name "MatMul_<n>", targetted_module,
    faulty_bit_position; parallelized_inject_onnx_transformer.py:837-858), or a
    qtx.fault.Fault.  One fault is injected into this run; the drawn fault is stored in
    weight_dict["qtx_fault"] (the reference records its choice in the experiment log)."""
    from . import fault as F
    model = model or _default_model
    if model is None:
        raise ValueError("no QtxModel: pass model= or call qtx.set_default_model()")
    weight_dict = {} if module_weight_dict is None else module_weight_dict
    for k, v in input_values.items():
        weight_dict[k] = v
    kind = _module_kind(module)
    fn = run_encoder if kind == "encoder" else run_decoder
    flt = None
    if inject_parameters and not isinstance(inject_parameters, F.Fault):
        # INPUT / WEIGHT kinds are injected only into the module they target
        # (onnx_optimized_inference.py:74: `module in inject_parameters["targetted_module"]`);
        # RANDOM kinds match the node name alone (:59), i.e. the module being run
        kind_ = inject_parameters["inject_type"]
        targetted = str(inject_parameters.get("targetted_module", module))
        if "RANDOM" not in kind_ and str(module) not in targetted:
            inject_parameters = None
        elif "RANDOM" in kind_:
            # a name that is no MatMul of this module's graph matches no node there: the
            # reference then injects nothing (onnx_optimized_inference.py:59)
            try:
                F.matmul_target(inject_parameters["faulty_operation_name"], kind,
                                model.cfg.n_layers)
            except ValueError:
                inject_parameters = None
    if inject_parameters:
        if isinstance(inject_parameters, F.Fault):
            flt = inject_parameters
        else:
            x = input_values["global_in"]
            rows = int(np.prod(_shape(x)[:2]))
            mod, _, lin = F.matmul_target(inject_parameters["faulty_operation_name"], kind)
            if lin in ("CK", "CV"):
                rows = int(np.prod(_shape(input_values["global_in_1"])[:2]))
            golden = None
            if inject_parameters["inject_type"] == "RANDOM_BITFLIP":
                raise ValueError("RANDOM_BITFLIP needs the golden MatMul output: draw the "
                                 "fault with qtx.fault.random_fault(golden_output=...)")
            B, Sq = _shape(x)[:2]
            Sk = _shape(input_values["global_in_1"])[1] if lin in ("CQK", "CPV") else Sq
            flt = F.from_inject_parameters(dict(inject_parameters, targetted_module=kind), rows,
                                           rng, model.cfg.n_layers, golden, (B, Sq, Sk))
        weight_dict["qtx_fault"] = flt
    if expose_intermediates:
        if flt is not None:
            raise ValueError("expose_intermediates runs the golden (fault-free) module only")
        trace = {"weights": expose_intermediates == "weights"}
        out = fn(model, input_values, None, trace).cpu().numpy()
        weight_dict.update(trace)
        weight_dict["global_out"] = out
        return {"global_out": out}, weight_dict
    t = fn(model, input_values, flt)
    model.check()
    out = t.cpu().numpy()
    weight_dict["global_out"] = out
    return {"global_out": out}, weight_dict
