"""Host-side handle of the device-resident quantized model.

torch tensors are used only as device containers and for the current HIP stream; every
computation runs in libqtx.so (HIP kernels for gfx950).  If the extension cannot be
loaded, or no GPU is visible, construction raises — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import threading

import numpy as np

from . import _lib
from .weights import ModelConfig, positional_table, tensor_order


def _torch():
    import torch
    return torch


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)


def _stream(device=None):
    torch = _torch()
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _on_device(fn):
    """Run a QtxModel entry point with the model's device current: its streams, events
    and workspace then belong to that device whatever device the caller has selected."""
    import functools

    @functools.wraps(fn)
    def wrapped(self, *a, **k):
        with _torch().cuda.device(self.device):
            return fn(self, *a, **k)
    return wrapped


def require_gpu():
    torch = _torch()
    if not torch.cuda.is_available():
        raise RuntimeError("qtx needs a ROCm GPU (gfx950); no device is visible")


class QtxModel:
    """Quantized W8A8 (or W4A8) model on one GPU, built from a reference state dict."""

    def __init__(self, state_dict: dict, cfg: ModelConfig = ModelConfig(), device=None):
        torch = _torch()
        require_gpu()
        self.cfg = cfg
        self.device = torch.device(device or "cuda")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        L = _lib.lib()
        self.ccfg = _lib.QtxConfig(cfg.src_vocab, cfg.tgt_vocab, cfg.n_layers, cfg.d_model,
                                   cfg.d_ff, cfg.n_heads, cfg.max_len, cfg.weight_bits)
        keys = tensor_order(cfg)
        n = L.qtx_model_tensor_count(C.byref(self.ccfg))
        if n != len(keys):
            raise RuntimeError(f"tensor count mismatch: lib {n} vs host {len(keys)}")
        with torch.cuda.device(self.device):
            dev = [torch.from_numpy(np.ascontiguousarray(state_dict[k], np.float32)
                                    .reshape(-1)).to(self.device) for k in keys]
            pe_np = state_dict.get("src_embed.1.pe")
            pe_np = positional_table(cfg.d_model, cfg.max_len) if pe_np is None else pe_np
            pe = torch.from_numpy(np.ascontiguousarray(pe_np, np.float32).reshape(-1)).to(self.device)
            arr = (C.c_void_p * len(dev))(*[t.data_ptr() for t in dev])
            h = C.c_void_p()
            _lib.call("qtx_model_create", C.byref(self.ccfg), arr, len(dev), _ptr(pe),
                      _stream(self.device), C.byref(h))
        self.handle = h
        self._tls = threading.local()

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                _lib.lib().qtx_model_destroy(h)
            except Exception:
                pass
            self.handle = None

    @_on_device
    def check(self):
        """Synchronise the current stream and raise QtxError (status QTX_E_DEVICE) if a
        kernel of this thread's last call on the model flagged an error in the thread's
        device status word (qtx_model_check); called wherever the host synchronises anyway."""
        _lib.call("qtx_model_check", self.handle, _stream(self.device))

    @property
    def device_bytes(self) -> int:
        return int(_lib.lib().qtx_model_device_bytes(self.handle))

    # ---- workspace (grown on demand, reused; never allocated inside a hot call) --------
    # One per calling thread: the handle is shared by threads (include/qtx.h), each with
    # its own stream, so each also needs its own scratch.
    @_on_device
    def workspace(self, nbytes: int):
        torch = _torch()
        ws = getattr(self._tls, "ws", None)
        if ws is None or ws.numel() < nbytes:
            ws = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=self.device)
            self._tls.ws = ws
        return ws

    # ---- model-level entry points (device tensors in, device tensors out) -------------
    @_on_device
    def encode(self, x, src_mask_u8, fault=None):
        """x [B,S,512] f32, src_mask_u8 [B,S] uint8 -> memory [B,S,512] f32.
        fault: an optional qtx.fault.Fault (one injected fault, module "Encoder")."""
        torch = _torch()
        B, S, _ = x.shape
        out = torch.empty_like(x)
        nb = _lib.lib().qtx_encoder_workspace_size(self.handle, B, S)
        ws = self.workspace(nb)
        if fault is None:
            _lib.call("qtx_encoder_forward", self.handle, _ptr(x), _ptr(src_mask_u8), B, S,
                      _ptr(out), _ptr(ws), ws.numel(), _stream(self.device))
        else:
            _lib.call("qtx_encoder_forward_fault", self.handle, _ptr(x), _ptr(src_mask_u8), B,
                      S, _ptr(out), _ptr(ws), ws.numel(), C.byref(fault.to_c()), _stream(self.device))
        return out

    @_on_device
    def decode(self, y, memory, src_mask_u8, tgt_mask_u8, fault=None):
        """y [B,T,512], memory [B,S,512], src_mask [B,S] u8, tgt_mask [T,T] or [B,T,T] u8."""
        torch = _torch()
        B, T, _ = y.shape
        S = memory.shape[1]
        out = torch.empty_like(y)
        nb = _lib.lib().qtx_decoder_workspace_size(self.handle, B, T, S)
        ws = self.workspace(nb)
        batched = 1 if tgt_mask_u8.dim() == 3 and tgt_mask_u8.shape[0] == B and B > 1 else 0
        if fault is None:
            _lib.call("qtx_decoder_forward", self.handle, _ptr(y), _ptr(memory),
                      _ptr(src_mask_u8), _ptr(tgt_mask_u8), batched, B, T, S, _ptr(out),
                      _ptr(ws), ws.numel(), _stream(self.device))
        else:
            _lib.call("qtx_decoder_forward_fault", self.handle, _ptr(y), _ptr(memory),
                      _ptr(src_mask_u8), _ptr(tgt_mask_u8), batched, B, T, S, _ptr(out),
                      _ptr(ws), ws.numel(), C.byref(fault.to_c()), _stream(self.device))
        return out

    @_on_device
    def greedy(self, src, src_mask_u8, max_len: int = 72, start: int = 0, out=None, fault=None):
        """src int64 [B,S], src_mask [B,S] u8 -> ids int64 [B,max_len] (device).
        fault: an optional encoder qtx.fault.Fault."""
        torch = _torch()
        B, S = src.shape
        ids = out if out is not None else torch.empty((B, max_len), dtype=torch.int64,
                                                      device=self.device)
        nb = _lib.lib().qtx_greedy_workspace_size(self.handle, B, S, max_len)
        ws = self.workspace(nb)
        if fault is None:
            _lib.call("qtx_greedy_decode", self.handle, _ptr(src), _ptr(src_mask_u8), B, S,
                      max_len, int(start), _ptr(ids), _ptr(ws), ws.numel(), _stream(self.device))
        else:
            _lib.call("qtx_greedy_decode_fault", self.handle, _ptr(src), _ptr(src_mask_u8), B,
                      S, max_len, int(start), _ptr(ids), _ptr(ws), ws.numel(),
                      C.byref(fault.to_c()), _stream(self.device))
        return ids

    @_on_device
    def embed(self, ids, which: str = "src", pos0: int = 0):
        torch = _torch()
        B, T = ids.shape
        out = torch.empty((B, T, self.cfg.d_model), dtype=torch.float32, device=self.device)
        _lib.call("qtx_embed", self.handle, 0 if which == "src" else 1, _ptr(ids), B, T, pos0,
                  _ptr(out), _stream(self.device))
        return out

    @_on_device
    def generator(self, x, want_logp: bool = True, return_logits: bool = False):
        """x [M,512] -> (logp [M,V] or None, ids int64 [M]) (+ raw logits [M,V])."""
        torch = _torch()
        M = x.shape[0]
        V = self.cfg.tgt_vocab
        logp = torch.empty((M, V), dtype=torch.float32, device=self.device) if want_logp else None
        ids = torch.empty((M,), dtype=torch.int64, device=self.device)
        ws = torch.empty((M * V,), dtype=torch.float32, device=self.device)
        _lib.call("qtx_generator", self.handle, _ptr(x), M, _ptr(logp), _ptr(ids), _ptr(ws),
                  ws.numel() * 4, _stream(self.device))
        if return_logits:
            return logp, ids, ws.view(M, V)
        return logp, ids


def to_u8_mask(mask, device):
    """Any bool/int mask tensor or array -> contiguous uint8 device tensor (nonzero = keep)."""
    torch = _torch()
    if isinstance(mask, np.ndarray):
        mask = torch.from_numpy(np.ascontiguousarray(mask))
    return (mask != 0).to(torch.uint8).to(device).contiguous()
