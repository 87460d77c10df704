"""The one-pass FFN1 (k_gemm_wsx, qtx_linear_rows kp = 3) exchanges row maxima between the
workgroups of a row group inside the launch, with bounded waits.  A wait that times out
must never pass silently (quant_linear.py:30-43 needs the whole row's maximum): the kernel
sets a device status word, qtx_model_check / the next model call report QTX_E_DEVICE.

Also: two concurrent launches on separate streams with separate exchange scratch (the
per-thread workspace case) are bit-exact and never raise the flag."""
import ctypes as C

import numpy as np
import pytest

from oracle import qtx_oracle as O

pytestmark = pytest.mark.gpu
f32 = np.float32
M = 32768          # cfg3's B*S: 1024 row blocks, every workgroup runs several


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def ffn1(torch):
    """Operands of one cfg3-sized FFN1 launch (WS weights, KP activations) and the
    two-pass result (kp = 2: row-max pass + quant pass, oracle-checked in test_gpu_ops)."""
    from qtx._lib import lib
    rng = np.random.default_rng(11)
    qx, sx = O.quant_rows(rng.standard_normal((M, 512)).astype(f32))
    qw, sw = O.quant_weight((rng.standard_normal((2048, 512)) * 0.05).astype(f32), 8)
    b = rng.standard_normal(2048).astype(f32)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    kp = np.ascontiguousarray(qx.reshape(-1, 2, 8, 64).transpose(0, 2, 1, 3)).reshape(-1, 512)
    wk = torch.empty((2048, 512), dtype=torch.int8, device="cuda")
    assert lib().qtx_pack_w_ws(C.c_void_p(T(qw).data_ptr()), 2048, 512,
                               C.c_void_p(wk.data_ptr()), C.c_void_p(0)) == 0
    base = dict(A=T(kp), sa=T(sx), W=wk, sw=T(sw), bias=T(b), M=M, N=2048, K=512, epi=3)
    pm = torch.empty((4, M), dtype=torch.float32, device="cuda")
    run(torch, dict(base, epi=2, kp=2, pmax_out=pm))
    h8 = torch.zeros((M, 2048), dtype=torch.int8, device="cuda")
    sh = torch.empty(M, dtype=torch.float32, device="cuda")
    run(torch, dict(base, kp=2, pmax_in=pm, pmax_n=4, out8=h8, ldo8=2048, os=sh))
    torch.cuda.synchronize()
    return base, h8.cpu().numpy(), sh.cpu().numpy()


def run(torch, kw, stream=None):
    from qtx._lib import RowGemm, lib
    a = RowGemm()
    for k, v in kw.items():
        setattr(a, k, v.data_ptr() if hasattr(v, "data_ptr") else v)
    st = C.c_void_p(stream.cuda_stream if stream is not None else 0)
    rc = lib().qtx_linear_rows(C.byref(a), st)
    assert rc == 0, lib().qtx_last_error()


def buffers(torch):
    return (torch.zeros((M, 2048), dtype=torch.int8, device="cuda"),
            torch.empty(M, dtype=torch.float32, device="cuda"),
            torch.empty(((32 * M + 2048) // 4,), dtype=torch.float32, device="cuda"))


def one_pass(torch, base, stream=None, status=None, bufs=None):
    h8, sh, gx = bufs if bufs is not None else buffers(torch)
    kw = dict(base, kp=3, pmax_out=gx, out8=h8, ldo8=2048, os=sh)
    if status is not None:
        kw["status"] = status
    run(torch, kw, stream)
    return h8, sh, gx


def scratch_flag(gx):
    """The status word of a launch without its own: the u32 after the ticket counter."""
    import torch
    nb = (M + 31) // 32
    return int(gx.view(torch.int32)[2 * 4 * 32 * nb + 1].item())


def test_concurrent_launches_bit_exact(torch, ffn1):
    """Two kp = 3 launches at once on two streams, each with its own scratch: both equal
    the two-pass result bit for bit, and neither raises the timeout flag."""
    base, h_ref, s_ref = ffn1
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    bufs = [buffers(torch) for _ in range(6)]
    torch.cuda.synchronize()            # the buffers' fills (current stream) are done
    outs = [one_pass(torch, base, (s1, s2)[i % 2], bufs=b) for i, b in enumerate(bufs)]
    torch.cuda.synchronize()
    for h8, sh, gx in outs:
        np.testing.assert_array_equal(h8.cpu().numpy(), h_ref)
        np.testing.assert_array_equal(sh.cpu().numpy(), s_ref)
        assert scratch_flag(gx) == 0


def test_timeout_flag_surfaces(torch, ffn1, monkeypatch):
    """With the spin bound forced to one poll (QTX_WSX_SPIN_LIMIT=0) some wait finds a
    partner's granule not yet published: the launch sets the status word instead of
    passing a partial maximum off silently.  With the default bound it stays clear."""
    base, h_ref, _ = ffn1
    st = torch.zeros(4, dtype=torch.int32, device="cuda")
    h8, _, _ = one_pass(torch, base, status=st)
    torch.cuda.synchronize()
    assert int(st[0].item()) == 0
    np.testing.assert_array_equal(h8.cpu().numpy(), h_ref)
    monkeypatch.setenv("QTX_WSX_SPIN_LIMIT", "0")
    flagged = 0
    for _ in range(4):
        st.zero_()
        one_pass(torch, base, status=st)
        torch.cuda.synchronize()
        flagged += int(st[0].item()) & 1
    assert flagged > 0, "no exchange wait timed out at a one-poll bound"


def test_model_reports_device_error(torch, gpu_model, monkeypatch):
    """Through the model: an encoder run whose FFN1 exchange timed out makes
    qtx_model_check (QtxModel.check) raise QTX_E_DEVICE = 5 once; the word is then clear."""
    from qtx._lib import QtxError
    x = torch.randn((256, 128, 512), device="cuda")
    mk = torch.ones((256, 128), dtype=torch.uint8, device="cuda")
    gpu_model.encode(x, mk)
    gpu_model.check()                                  # default bound: clean
    monkeypatch.setenv("QTX_WSX_SPIN_LIMIT", "0")
    raised = False
    for _ in range(4):
        gpu_model.encode(x, mk)
        try:
            gpu_model.check()
        except QtxError as e:
            assert e.code == 5 and "timed out" in str(e)
            raised = True
            break
    assert raised
    monkeypatch.delenv("QTX_WSX_SPIN_LIMIT")
    gpu_model.check()                                  # reported once, then cleared
    gpu_model.encode(x, mk)
    gpu_model.check()
