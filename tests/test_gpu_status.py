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


def test_timeout_flag_surfaces(torch, ffn1, knob_env):
    """A wait that finds a partner's maxima missing must not pass a partial maximum off
    silently: with the test hook that withholds slice 2's maxima (QTX_WSX_DROP_SLICE) and a
    64-poll bound, every partner wait times out and the launch sets the status word — in one
    run, deterministically.  With the default bound and no hook it stays clear."""
    base, h_ref, _ = ffn1
    st = torch.zeros(4, dtype=torch.int32, device="cuda")
    h8, _, _ = one_pass(torch, base, status=st)
    torch.cuda.synchronize()
    assert int(st[0].item()) == 0
    np.testing.assert_array_equal(h8.cpu().numpy(), h_ref)
    knob_env("QTX_WSX_SPIN_LIMIT", 64)
    knob_env("QTX_WSX_DROP_SLICE", 2)
    st.zero_()
    one_pass(torch, base, status=st)
    torch.cuda.synchronize()
    assert int(st[0].item()) & 1, "the withheld partner maxima did not time out"


def _cfg3(torch):
    return (torch.randn((256, 128, 512), device="cuda"),
            torch.ones((256, 128), dtype=torch.uint8, device="cuda"))


def test_model_reports_device_error(torch, gpu_model, knob_env):
    """Through the model: an encoder run whose FFN1 exchange timed out makes
    qtx_model_check (QtxModel.check) raise QTX_E_DEVICE = 5 once; the word is then clear,
    and a clean run stays clean."""
    from qtx._lib import QtxError
    knob_env("QTX_NO_FFN_FUSED", 1)                    # FFN1 on the one-pass exchange
    x, mk = _cfg3(torch)
    gpu_model.encode(x, mk)
    gpu_model.check()                                  # default bound: clean
    knob_env("QTX_WSX_SPIN_LIMIT", 64)
    knob_env("QTX_WSX_DROP_SLICE", 1)
    gpu_model.encode(x, mk)
    with pytest.raises(QtxError) as e:
        gpu_model.check()
    assert e.value.code == 5 and "timed out" in str(e.value)
    gpu_model.check()                                  # reported once, then cleared
    knob_env("QTX_WSX_DROP_SLICE", -1)
    gpu_model.encode(x, mk)
    gpu_model.check()


def test_status_word_is_per_call(torch, gpu_model, knob_env):
    """the status word belongs to the calling thread, not to the model as a whole.
    Thread A's cfg3 encode times out in its FFN1 exchange (hook on) while thread B encodes a
    small batch concurrently (M = 288: the two-pass FFN1, no exchange) and checks on its own
    stream: B's check is clean and cannot clear A's error; A's check raises."""
    import threading
    from qtx._lib import QtxError
    knob_env("QTX_NO_FFN_FUSED", 1)                    # FFN1 on the one-pass exchange
    knob_env("QTX_WSX_SPIN_LIMIT", 64)
    knob_env("QTX_WSX_DROP_SLICE", 3)
    xa, ma = _cfg3(torch)
    xb = torch.randn((4, 72, 512), device="cuda")
    mb = torch.ones((4, 72), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    res = {}
    go = threading.Barrier(2)

    def run(name, x, m):
        try:
            with torch.cuda.stream(torch.cuda.Stream()):
                go.wait()
                for _ in range(3 if name == "b" else 1):
                    gpu_model.encode(x, m)
                    gpu_model.check()
            res[name] = "clean"
        except QtxError as e:
            res[name] = e.code
        except Exception as e:             # noqa: BLE001 - reported below
            res[name] = repr(e)
    ts = [threading.Thread(target=run, args=("a", xa, ma)), threading.Thread(target=run, args=("b", xb, mb))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert res == {"a": 5, "b": "clean"}, res


def test_workspace_reuse_reports_no_false_error(torch, gpu_model):
    """Round 4: the status word first lived in the call's workspace; the next call on the
    same workspace (the decoder-fault greedy loop: an encode, then decoder calls) wrote its
    scratch over it and a check read that as an error.  The word now lives in the model's
    memory, per thread: an encode followed by a decoder call on the thread's one (reused)
    workspace, filled with nonzero bytes first, checks clean after each call."""
    x = torch.randn((2, 16, 512), device="cuda")
    m = torch.ones((2, 16), dtype=torch.uint8, device="cuda")
    nb = max(int(gpu_model.workspace(0).numel()), 1 << 20)
    gpu_model.workspace(nb).fill_(0xFF)
    mem = gpu_model.encode(x, m)
    gpu_model.check()
    y = torch.randn((2, 5, 512), device="cuda")
    tm = torch.tril(torch.ones((5, 5), dtype=torch.uint8, device="cuda"))
    gpu_model.workspace(nb).fill_(0xFF)
    gpu_model.decode(y, mem, m, tm)
    gpu_model.check()
    gpu_model.encode(x, m)
    gpu_model.check()


def test_decoder_call_keeps_encode_error(torch, gpu_model, knob_env):
    """a decoder call after an encode whose FFN1 exchange timed out must
    not erase that error before the check (the greedy_decode_fault loop: encode, then decoder
    calls, then one check).  B = 32, S = 72 (M = 2304): the encode runs the one-pass FFN1."""
    from qtx._lib import QtxError
    knob_env("QTX_WSX_SPIN_LIMIT", 64)
    knob_env("QTX_WSX_DROP_SLICE", 1)
    x = torch.randn((32, 72, 512), device="cuda")
    m = torch.ones((32, 72), dtype=torch.uint8, device="cuda")
    mem = gpu_model.encode(x, m)
    knob_env("QTX_WSX_DROP_SLICE", -1)
    y = torch.randn((32, 5, 512), device="cuda")
    tm = torch.tril(torch.ones((5, 5), dtype=torch.uint8, device="cuda"))
    gpu_model.decode(y, mem, m, tm)
    gpu_model.decode(y, mem, m, tm)
    with pytest.raises(QtxError) as e:
        gpu_model.check()
    assert e.value.code == 5
    gpu_model.check()                                  # reported once, then cleared


def test_status_slots_exhaustion_is_loud(torch, state_dict, knob_env):
    """VERDICT r04 hygiene: status words are never shared.  With the cap lowered to 4
    (QTX_STATUS_SLOTS), 4 live threads hold a word each and a 5th thread's encode fails with
    QTX_E_UNSUPPORTED; once those threads exit their words return to the model, and 12
    short-lived threads in turn all run clean."""
    import threading
    from qtx._lib import QtxError
    from qtx.model import QtxModel
    knob_env("QTX_STATUS_SLOTS", 4)
    model = QtxModel(state_dict)                       # fresh slots
    x = torch.randn((2, 8, 512), device="cuda")
    m = torch.ones((2, 8), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    hold, res = threading.Event(), {}

    def worker(name, wait):
        try:
            model.encode(x, m)
            model.check()
            res[name] = "ok"
        except QtxError as e:
            res[name] = e.code
        if wait:
            hold.wait(timeout=60)
    live = [threading.Thread(target=worker, args=(f"h{i}", True)) for i in range(4)]
    for t in live:
        t.start()
    import time
    t0 = time.time()
    while len(res) < 4 and time.time() - t0 < 60:
        time.sleep(0.01)
    extra = threading.Thread(target=worker, args=("extra", False))
    extra.start()
    extra.join(timeout=60)
    hold.set()
    for t in live:
        t.join(timeout=60)
    assert res == {**{f"h{i}": "ok" for i in range(4)}, "extra": 4}, res
    res.clear()
    for i in range(12):
        t = threading.Thread(target=worker, args=(f"s{i}", False))
        t.start()
        t.join(timeout=60)
    assert res == {f"s{i}": "ok" for i in range(12)}, res


def test_reclaimed_slot_drops_stale_error(torch, state_dict, knob_env):
    """a thread that exits with its encode still in flight and a device error
    unreported (its FFN1 exchange times out after it is gone) returns its status word to
    the model; the next thread to claim that word (the cap lowered to 1, so it must be the
    same word) starts clean — the claim drains the device before zeroing the word — and its
    own clean encode checks clean."""
    import threading
    from qtx.model import QtxModel
    knob_env("QTX_STATUS_SLOTS", 1)
    knob_env("QTX_NO_FFN_FUSED", 1)                    # FFN1 on the one-pass exchange
    model = QtxModel(state_dict)
    x, mk = _cfg3(torch)
    torch.cuda.synchronize()
    knob_env("QTX_WSX_SPIN_LIMIT", 64)
    knob_env("QTX_WSX_DROP_SLICE", 2)
    res = {}

    def leaver():
        with torch.cuda.stream(torch.cuda.Stream()):
            model.encode(x, mk)                        # times out on the device; no check
        res["a"] = "left"
    a = threading.Thread(target=leaver)
    a.start()
    a.join(timeout=60)
    knob_env("QTX_WSX_DROP_SLICE", -1)

    def claimer():
        try:
            with torch.cuda.stream(torch.cuda.Stream()):
                model.encode(x, mk)
                model.check()
            res["b"] = "clean"
        except Exception as e:             # noqa: BLE001 - reported below
            res["b"] = repr(e)
    b = threading.Thread(target=claimer)
    b.start()
    b.join(timeout=60)
    assert res == {"a": "left", "b": "clean"}, res
