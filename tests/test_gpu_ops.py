"""Per-op parity of the HIP kernels (through the C-ABI) against the CPU oracle.

Contract: bit-exact.  Integer tensors (quantized activations, int32-accumulator results,
argmax ids) and the float outputs of the canonical evaluation order are compared with
assert_array_equal; the only tolerance is the log-softmax value (platform log, 1 ulp).
"""
import ctypes as C

import numpy as np
import pytest

from oracle import qtx_oracle as O

pytestmark = pytest.mark.gpu
f32 = np.float32


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def P(t):
    return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)


_KEEP = []   # device tensors must outlive the C call that receives their raw pointers


@pytest.fixture(autouse=True)
def _release():
    yield
    _KEEP.clear()


def dev(torch, a):
    t = torch.from_numpy(np.ascontiguousarray(a)).cuda()
    _KEEP.append(t)
    return t


def call(name, *args):
    from qtx import _lib
    _lib.call(name, *args)


S0 = C.c_void_p(0)


@pytest.mark.parametrize("D", [512, 2048])
def test_row_quant(torch, D):
    rng = np.random.default_rng(D)
    x = (rng.standard_normal((37, D)) * rng.uniform(1e-3, 10, (37, 1))).astype(f32)
    x[0] = 0
    x[1, :4] = [127.0, 0.5, 1.5, -2.5]
    x[1, 4:] = 0
    xd = dev(torch, x)
    q = torch.empty((37, D), dtype=torch.int8, device="cuda")
    s = torch.empty((37,), dtype=torch.float32, device="cuda")
    call("qtx_row_quant", P(xd), 37, D, 127.0, P(q), P(s), S0)
    qo, so = O.quant_rows(x)
    np.testing.assert_array_equal(q.cpu().numpy(), qo)
    np.testing.assert_array_equal(s.cpu().numpy(), so)
    call("qtx_row_quant", P(xd), 37, D, 7.0, P(q), P(s), S0)     # int4 weight quantizer
    qo, so = O.quant_rows(x, 4)
    np.testing.assert_array_equal(q.cpu().numpy(), qo)


@pytest.mark.parametrize("scale", [1.0, 1e15, 1e-25])
def test_layernorm_quant(torch, golden_ops, oracle_model, scale):
    """scale 1e15 / 1e-25 push the shared-divisor division outside its guarded range, so
    the kernels' true-division fallback is exercised too."""
    x = (golden_ops["ln_x"] * np.float32(scale)).astype(f32)
    a, b = oracle_model.enc[0]["ln"][0]
    y = torch.empty(x.shape, dtype=torch.float32, device="cuda")
    q = torch.empty(x.shape, dtype=torch.int8, device="cuda")
    s = torch.empty(x.shape[:1], dtype=torch.float32, device="cuda")
    call("qtx_layernorm_quant", P(dev(torch, x)), P(dev(torch, a)), P(dev(torch, b)),
         x.shape[0], 512, P(y), P(q), P(s), S0)
    yo = O.layer_norm(x, a, b)
    np.testing.assert_array_equal(y.cpu().numpy(), yo)
    qo, so = O.quant_rows(yo)
    np.testing.assert_array_equal(q.cpu().numpy(), qo)
    np.testing.assert_array_equal(s.cpu().numpy(), so)


@pytest.mark.parametrize("M,N,K,flags,bits", [
    (16, 512, 512, 0, 8), (72, 1536, 512, 0, 8), (300, 512, 512, 2, 8),
    (130, 2048, 512, 1, 8), (257, 512, 2048, 2, 8), (33, 512, 2048, 0, 4),
    (512, 2048, 512, 1, 4), (1000, 1536, 512, 0, 8), (520, 272, 512, 1, 8),
    (256, 2048, 2048, 3, 8), (300, 512, 640, 2, 8)])
def test_linear_i8(torch, M, N, K, flags, bits):
    rng = np.random.default_rng(M * N + K)
    x = rng.standard_normal((M, K)).astype(f32)
    w = (rng.standard_normal((N, K)) * 0.05).astype(f32)
    b = rng.standard_normal(N).astype(f32)
    res = rng.standard_normal((M, N)).astype(f32)
    qx, sx = O.quant_rows(x)
    qw, sw = O.quant_weight(w, bits)
    wd = dev(torch, qw)
    if bits == 4:
        packed = torch.empty((N, K // 2), dtype=torch.uint8, device="cuda")
        call("qtx_pack_int4", P(wd), N, K, P(packed), S0)
        wd = packed
    out = dev(torch, res.copy()) if flags & 2 else torch.empty((M, N), dtype=torch.float32, device="cuda")
    call("qtx_linear_i8", P(dev(torch, qx)), P(dev(torch, sx)), P(wd), P(dev(torch, sw)),
         P(dev(torch, b)), M, N, K, bits, flags, P(out) if flags & 2 else S0, P(out), S0)
    y = O.linear_epilogue(O.int_gemm(qx, qw), sx, sw, b, relu=bool(flags & 1))
    if flags & 2:
        y = res + y
    np.testing.assert_array_equal(out.cpu().numpy(), y)


@pytest.mark.parametrize("M", [128, 512])
def test_linear_asymmetric_identity(torch, M):
    """A = I-like, asymmetric W: catches row/col swaps of the MFMA C layout (both the
    128x128 and the 256x256 GEMM)."""
    N = K = M
    qx = np.zeros((M, K), np.int8)
    qx[np.arange(M), np.arange(K)] = 1
    qw = (np.arange(N * K).reshape(N, K) % 251 - 125).astype(np.int8)
    one = np.ones(M, f32)
    out = torch.empty((M, N), dtype=torch.float32, device="cuda")
    call("qtx_linear_i8", P(dev(torch, qx)), P(dev(torch, one)), P(dev(torch, qw)),
         P(dev(torch, np.ones(N, f32))), P(dev(torch, np.zeros(N, f32))), M, N, K, 8, 0, S0,
         P(out), S0)
    np.testing.assert_array_equal(out.cpu().numpy(), qw.T.astype(f32))


@pytest.mark.parametrize("B,Sq,Sk,masked", [(2, 20, 20, True), (3, 1, 37, False),
                                            (2, 128, 128, True), (1, 7, 300, True),
                                            (3, 128, 128, "key"), (2, 72, 72, "key"),
                                            (2, 65, 100, "key"), (2, 16, 64, "key"),
                                            (1, 130, 5, "key")])
@pytest.mark.parametrize("dec", [0, 1])
def test_attention(torch, B, Sq, Sk, masked, dec):
    """qtx_attention_i8 == oracle attention, in the encoder's PV order (dec 0) and the
    decoder's (dec 1: four partial chains; k_attn_mfma<true>, and k_attention past 128 keys)."""
    rng = np.random.default_rng(Sq * 7 + Sk)
    H = 8
    q = rng.integers(-127, 128, (B, Sq, 512)).astype(np.int8)
    k = rng.integers(-127, 128, (B, Sk, 512)).astype(np.int8)
    v = rng.integers(-127, 128, (B, Sk, 512)).astype(np.int8)
    sq, sk, sv = (rng.uniform(0.002, 0.03, (B, n)).astype(f32) for n in (Sq, Sk, Sk))
    mask = np.ones((B, Sq, Sk), np.uint8)
    m_bs, m_is, mdev = Sq * Sk, Sk, mask
    if masked == "key":               # encoder form: one key mask per sentence (m_is = 0)
        km = np.ones((B, Sk), np.uint8)
        km[0, Sk - Sk // 3:] = 0
        km[-1, 1::7] = 0
        mask[:] = km[:, None, :]
        m_bs, m_is, mdev = Sk, 0, km
    elif masked:
        mask[-1, :, Sk // 2:] = 0
        mask[0] = np.tril(np.ones((Sq, Sk), np.uint8), k=Sk - Sq)
    ctx = torch.empty((B, Sq, 512), dtype=torch.float32, device="cuda")
    call("qtx_attention_i8", P(dev(torch, q)), P(dev(torch, sq)), P(dev(torch, k)),
         P(dev(torch, sk)), P(dev(torch, v)), P(dev(torch, sv)), P(dev(torch, mdev)),
         m_bs, m_is, B, H, Sq, Sk, P(ctx), dec, S0)
    co, _ = O.attention(q, sq, k, sk, v, sv, mask, H, dec=bool(dec))
    np.testing.assert_array_equal(ctx.cpu().numpy(), co)


@pytest.mark.parametrize("B,S,keymask", [(3, 128, True), (2, 72, True), (2, 5, False),
                                          (1, 1, False), (4, 100, True), (2, 128, False)])
def test_attention_quant(torch, B, S, keymask):
    """Encoder attention with the per-token-quantized context (k_attn_encq) == oracle
    attention followed by the O-projection input quantizer, bit for bit."""
    rng = np.random.default_rng(S * 11 + B)
    q, k, v = (rng.integers(-127, 128, (B, S, 512)).astype(np.int8) for _ in range(3))
    sq, sk, sv = (rng.uniform(0.002, 0.03, (B, S)).astype(f32) for _ in range(3))
    km = np.ones((B, S), np.uint8)
    if keymask:
        km[0, S - S // 3:] = 0
        km[-1, 1::7] = 0
    ctx8 = torch.empty((B, S, 512), dtype=torch.int8, device="cuda")
    sctx = torch.empty((B, S), dtype=torch.float32, device="cuda")
    call("qtx_attention_i8_quant", P(dev(torch, q)), P(dev(torch, sq)), P(dev(torch, k)),
         P(dev(torch, sk)), P(dev(torch, v)), P(dev(torch, sv)),
         P(dev(torch, km)) if keymask else S0, B, S, P(ctx8), P(sctx), S0)
    co, _ = O.attention(q, sq, k, sk, v, sv, km[:, None, :], 8)
    qc, sc = O.quant_rows(co)
    np.testing.assert_array_equal(sctx.cpu().numpy(), sc)
    np.testing.assert_array_equal(ctx8.cpu().numpy(), qc)


def test_embed(torch, gpu_model, golden_ops, oracle_model):
    # The PE table is computed at load time by torch's CPU sin/cos (as the reference
    # does), whose last ulp depends on the host CPU; compare with the oracle on the same
    # table (bit-exact) and with the golden vectors to the PE's platform tolerance.
    ids = golden_ops["emb_ids"]
    out = gpu_model.embed(dev(torch, ids), "src")
    np.testing.assert_array_equal(out.cpu().numpy(),
                                  oracle_model.embed(ids, oracle_model.src_lut))
    assert np.abs(out.cpu().numpy() - golden_ops["emb_ref"]).max() < 1e-6
    out = gpu_model.embed(dev(torch, ids[:, :5] % 4444), "tgt", pos0=9)
    np.testing.assert_array_equal(out.cpu().numpy(),
                                  oracle_model.embed(ids[:, :5] % 4444, oracle_model.tgt_lut, pos0=9))


@pytest.mark.parametrize("M", [37, 32, 5, 100, 256])
def test_generator(torch, gpu_model, golden_ops, oracle_model, M):
    """Logits bit-exact (fp32-MFMA chain == the oracle's sequential fma chain), argmax
    exact, log-probs within the platform log's ulp; M > 32 runs several 16-row blocks per
    workgroup under one load of the weight strips (ragged last group at M = 37 and 100)."""
    gx = golden_ops["gen_x"]
    x = (np.concatenate([gx] * (M // len(gx) + 1))[:M]
         * np.linspace(0.1, 3, M, dtype=f32)[:, None]).astype(f32)
    logp, ids, logits = gpu_model.generator(dev(torch, x), return_logits=True)
    np.testing.assert_array_equal(logits.cpu().numpy(), oracle_model.logits(x))
    lo, io = oracle_model.generator(x)
    np.testing.assert_array_equal(ids.cpu().numpy(), io)
    assert np.abs(logp.cpu().numpy() - lo).max() <= 2e-6


def test_generator_nonfinite_rows(torch, gpu_model, golden_ops, oracle_model):
    """qtx_generator on rows whose logits are non-finite (a NaN input; inputs so large the
    logits overflow to +-inf): torch's rule, logp all NaN and id 0, as the oracle says."""
    x = np.concatenate([golden_ops["gen_x"]] * 4)[:6].astype(f32)
    x[0, 3] = np.nan
    x[1] *= f32(1e37)
    x[2, :] = f32(3e38)
    logp, ids, logits = gpu_model.generator(dev(torch, x), return_logits=True)
    lo, io = oracle_model.generator(x)
    np.testing.assert_array_equal(ids.cpu().numpy(), io)
    np.testing.assert_array_equal(np.isnan(logp.cpu().numpy()), np.isnan(lo))
    assert io[0] == 0 and np.isnan(lo[0]).all()
    assert not np.isfinite(logits.cpu().numpy()[1:3]).all()    # the overflow rows do overflow


def _rows_call(torch, **kw):
    from qtx._lib import RowGemm, lib
    import ctypes as C
    a = RowGemm()
    for k, v in kw.items():
        setattr(a, k, v.data_ptr() if hasattr(v, "data_ptr") else v)
    rc = lib().qtx_linear_rows(C.byref(a), S0)
    assert rc == 0, lib().qtx_last_error()


@pytest.mark.parametrize("M", [300, 128, 7])
def test_linear_rows_quant_qkv(torch, M):
    """epi 0: Q/K/V GEMM with the per-token output quantization of each 512-wide tile."""
    rng = np.random.default_rng(M + 1)
    qx, sx = O.quant_rows(rng.standard_normal((M, 512)).astype(f32))
    qw, sw = O.quant_weight((rng.standard_normal((1536, 512)) * 0.05).astype(f32), 8)
    b = rng.standard_normal(1536).astype(f32)
    out8 = torch.empty((3, M, 512), dtype=torch.int8, device="cuda")
    os_ = torch.empty((3, M), dtype=torch.float32, device="cuda")
    _rows_call(torch, A=dev(torch, qx), sa=dev(torch, sx), W=dev(torch, qw), sw=dev(torch, sw),
               bias=dev(torch, b), M=M, N=1536, K=512, epi=0, out8=out8, ldo8=512,
               o8_ts=M * 512, os=os_, os_ts=M)
    y = O.linear_epilogue(O.int_gemm(qx, qw), sx, sw, b)
    for t in range(3):
        q, s = O.quant_rows(y[:, 512 * t:512 * (t + 1)])
        np.testing.assert_array_equal(out8[t].cpu().numpy(), q)
        np.testing.assert_array_equal(os_[t].cpu().numpy(), s)


@pytest.mark.parametrize("M,K,quant", [(300, 2048, True), (130, 512, False), (5, 512, True)])
def test_linear_rows_residual_layernorm(torch, oracle_model, M, K, quant):
    """epi 1: x = res + y, then the next sublayer's LayerNorm (+ per-token quant)."""
    rng = np.random.default_rng(M + K)
    qx, sx = O.quant_rows(rng.standard_normal((M, K)).astype(f32))
    qw, sw = O.quant_weight((rng.standard_normal((512, K)) * 0.05).astype(f32), 8)
    b = rng.standard_normal(512).astype(f32)
    res = (rng.standard_normal((M, 512)) * 2).astype(f32)
    la, lb = oracle_model.dec[1]["ln"][0]
    xd = dev(torch, res.copy())
    kw = dict(A=dev(torch, qx), sa=dev(torch, sx), W=dev(torch, qw), sw=dev(torch, sw),
              bias=dev(torch, b), M=M, N=512, K=K, epi=1, res=xd, xout=xd,
              ln_a=dev(torch, la), ln_b=dev(torch, lb))
    if quant:
        lnq = torch.empty((M, 512), dtype=torch.int8, device="cuda")
        lns = torch.empty(M, dtype=torch.float32, device="cuda")
        kw.update(lnq=lnq, lns=lns)
    else:
        lnout = torch.empty((M, 512), dtype=torch.float32, device="cuda")
        kw.update(lnout=lnout)
    _rows_call(torch, **kw)
    x = res + O.linear_epilogue(O.int_gemm(qx, qw), sx, sw, b)
    np.testing.assert_array_equal(xd.cpu().numpy(), x)
    ln = O.layer_norm(x, la, lb)
    if quant:
        q, s = O.quant_rows(ln)
        np.testing.assert_array_equal(lnq.cpu().numpy(), q)
        np.testing.assert_array_equal(lns.cpu().numpy(), s)
    else:
        np.testing.assert_array_equal(lnout.cpu().numpy(), ln)


@pytest.mark.parametrize("M", [260, 33])
def test_linear_rows_ffn1_two_pass(torch, M):
    """epi 2 + 3: relu(FFN1) tile maxima, then recompute + per-token quant over d_ff."""
    rng = np.random.default_rng(M + 7)
    qx, sx = O.quant_rows(rng.standard_normal((M, 512)).astype(f32))
    qw, sw = O.quant_weight((rng.standard_normal((2048, 512)) * 0.05).astype(f32), 8)
    b = rng.standard_normal(2048).astype(f32)
    pm = torch.empty((4, M), dtype=torch.float32, device="cuda")
    base = dict(A=dev(torch, qx), sa=dev(torch, sx), W=dev(torch, qw), sw=dev(torch, sw),
                bias=dev(torch, b), M=M, N=2048, K=512)
    _rows_call(torch, epi=2, pmax_out=pm, **base)
    h = O.linear_epilogue(O.int_gemm(qx, qw), sx, sw, b, relu=True)
    np.testing.assert_array_equal(pm.cpu().numpy(), h.reshape(M, 4, 512).max(-1).T)
    h8 = torch.empty((M, 2048), dtype=torch.int8, device="cuda")
    sh = torch.empty(M, dtype=torch.float32, device="cuda")
    _rows_call(torch, epi=3, pmax_in=pm, pmax_n=4, out8=h8, ldo8=2048, os=sh, **base)
    q, s = O.quant_rows(h)
    np.testing.assert_array_equal(h8.cpu().numpy(), q)
    np.testing.assert_array_equal(sh.cpu().numpy(), s)


def _to_kp(a):
    """[M, K] int8 -> the KP layout (qtx_common.h kp_off): row pair p, 64-byte K chunk c =
    one 128-byte line (p * K/64 + c), rows 2p | 2p+1 at +0 | +64; odd M padded by a row."""
    M, K = a.shape
    if M & 1:
        a = np.concatenate([a, np.zeros((1, K), a.dtype)])
    return np.ascontiguousarray(a.reshape(-1, 2, K // 64, 64).transpose(0, 2, 1, 3)).reshape(-1, K)


def _from_kp(a, M):
    K = a.shape[1]
    return a.reshape(-1, K // 64, 2, 64).transpose(0, 2, 1, 3).reshape(-1, K)[:M]


def _kp_w_order(N):
    """Row order of qtx_pack_w_kp: packed row rho of 512-column tile t holds W row
    t*512 + (rho & ~127) + 8 (rho & 15) + ((rho >> 4) & 7)."""
    rho = np.arange(512)
    r = (rho & ~127) + 8 * (rho & 15) + ((rho >> 4) & 7)
    return (np.arange(N // 512)[:, None] * 512 + r[None, :]).reshape(-1)


@pytest.mark.parametrize("N,K", [(1536, 512), (512, 2048)])
def test_pack_w_kp(torch, N, K):
    rng = np.random.default_rng(N + K)
    w = rng.integers(-127, 128, (N, K)).astype(np.int8)
    out = torch.empty((N, K), dtype=torch.int8, device="cuda")
    from qtx._lib import lib
    assert lib().qtx_pack_w_kp(P(dev(torch, w)), N, K, P(out), S0) == 0
    np.testing.assert_array_equal(out.cpu().numpy(), _to_kp(w[_kp_w_order(N)]))


@pytest.mark.parametrize("M", [300, 7, 256])
def test_linear_rows_kp(torch, oracle_model, M):
    """kp = 1 (the encoder's layout): every epilogue bit-exact against the oracle, int8
    outputs of epi 1 / 3 in the KP layout, epi 0's Q/K/V row-major."""
    from qtx._lib import lib
    rng = np.random.default_rng(M + 99)

    def weights(N, K):
        qw, sw = O.quant_weight((rng.standard_normal((N, K)) * 0.05).astype(f32), 8)
        wk = torch.empty((N, K), dtype=torch.int8, device="cuda")
        assert lib().qtx_pack_w_kp(P(dev(torch, qw)), N, K, P(wk), S0) == 0
        return qw, sw, wk, rng.standard_normal(N).astype(f32)

    qx, sx = O.quant_rows(rng.standard_normal((M, 512)).astype(f32))
    ax = dev(torch, _to_kp(qx))
    # epi 0
    qw, sw, wk, b = weights(1536, 512)
    out8 = torch.empty((3, M, 512), dtype=torch.int8, device="cuda")
    os_ = torch.empty((3, M), dtype=torch.float32, device="cuda")
    _rows_call(torch, A=ax, sa=dev(torch, sx), W=wk, sw=dev(torch, sw), bias=dev(torch, b),
               M=M, N=1536, K=512, epi=0, out8=out8, ldo8=512, o8_ts=M * 512, os=os_,
               os_ts=M, kp=1)
    y = O.linear_epilogue(O.int_gemm(qx, qw), sx, sw, b)
    for t in range(3):
        q, s = O.quant_rows(y[:, 512 * t:512 * (t + 1)])
        np.testing.assert_array_equal(out8[t].cpu().numpy(), q)
        np.testing.assert_array_equal(os_[t].cpu().numpy(), s)
    # epi 2 + 3 (FFN1), hidden written KP
    qw, sw, wk, b = weights(2048, 512)
    pm = torch.empty((4, M), dtype=torch.float32, device="cuda")
    base = dict(A=ax, sa=dev(torch, sx), W=wk, sw=dev(torch, sw), bias=dev(torch, b),
                M=M, N=2048, K=512, kp=1)
    _rows_call(torch, epi=2, pmax_out=pm, **base)
    h = O.linear_epilogue(O.int_gemm(qx, qw), sx, sw, b, relu=True)
    np.testing.assert_array_equal(pm.cpu().numpy(), h.reshape(M, 4, 512).max(-1).T)
    h8 = torch.zeros((M + (M & 1), 2048), dtype=torch.int8, device="cuda")
    sh = torch.empty(M, dtype=torch.float32, device="cuda")
    _rows_call(torch, epi=3, pmax_in=pm, pmax_n=4, out8=h8, ldo8=2048, os=sh, **base)
    qh, s = O.quant_rows(h)
    np.testing.assert_array_equal(_from_kp(h8.cpu().numpy(), M), qh)
    np.testing.assert_array_equal(sh.cpu().numpy(), s)
    # epi 1 (FFN2: K = 2048 from the KP hidden), next LayerNorm quantized KP
    qw, sw, wk, b = weights(512, 2048)
    res = (rng.standard_normal((M, 512)) * 2).astype(f32)
    la, lb = oracle_model.dec[1]["ln"][0]
    xd = dev(torch, res.copy())
    lnq = torch.zeros((M + (M & 1), 512), dtype=torch.int8, device="cuda")
    lns = torch.empty(M, dtype=torch.float32, device="cuda")
    _rows_call(torch, A=h8, sa=sh, W=wk, sw=dev(torch, sw), bias=dev(torch, b), M=M, N=512,
               K=2048, epi=1, res=xd, xout=xd, ln_a=dev(torch, la), ln_b=dev(torch, lb),
               lnq=lnq, lns=lns, kp=1)
    x = res + O.linear_epilogue(O.int_gemm(qh, qw), s, sw, b)
    np.testing.assert_array_equal(xd.cpu().numpy(), x)
    q, s2 = O.quant_rows(O.layer_norm(x, la, lb))
    np.testing.assert_array_equal(_from_kp(lnq.cpu().numpy(), M), q)
    np.testing.assert_array_equal(lns.cpu().numpy(), s2)


@pytest.mark.parametrize("M", [300, 7, 20011, 4096, 8160, 32768, 64])
def test_linear_rows_ws_qkv_scales(torch, M):
    """Q/K/V (epi 0, kp = 2) on the weight-stationary kernel (k_gemm_wsq: one barrier per
    block, quantization interleaved between the MFMAs) with row scales from 1e-35 to 1e25:
    outputs from subnormal-tiny (the 1e-5 clamp decides) to ~1e28 (the shared-reciprocal
    division at every magnitude), bit-exact; M covers 1..13 blocks per workgroup and ragged
    last blocks.  (The measured-negative variants k_gemm_wsp-for-QKV / wss / wsz / wsa are
    in the diagnostic build only, qtx_wsgemm_diag.hip.)"""
    from qtx._lib import lib
    rng = np.random.default_rng(M + 17)
    qx, sx = O.quant_rows(rng.standard_normal((M, 512)).astype(f32))
    sx = (sx * np.float32(10.0) ** rng.integers(-33, 26, M)).astype(f32)
    qw, sw = O.quant_weight((rng.standard_normal((1536, 512)) * 0.05).astype(f32), 8)
    b = (rng.standard_normal(1536) * 1e-3).astype(f32)
    wk = torch.empty((1536, 512), dtype=torch.int8, device="cuda")
    assert lib().qtx_pack_w_ws(P(dev(torch, qw)), 1536, 512, P(wk), S0) == 0
    out8 = torch.empty((3, M, 512), dtype=torch.int8, device="cuda")
    os_ = torch.empty((3, M), dtype=torch.float32, device="cuda")
    _rows_call(torch, A=dev(torch, _to_kp(qx)), sa=dev(torch, sx), W=wk, sw=dev(torch, sw),
               bias=dev(torch, b), M=M, N=1536, K=512, epi=0, out8=out8, ldo8=512,
               o8_ts=M * 512, os=os_, os_ts=M, kp=2)
    y = O.linear_epilogue(O.int_gemm(qx, qw), sx, sw, b)
    for t in range(3):
        q, s = O.quant_rows(y[:, 512 * t:512 * (t + 1)])
        np.testing.assert_array_equal(out8[t].cpu().numpy(), q)
        np.testing.assert_array_equal(os_[t].cpu().numpy(), s)


@pytest.mark.parametrize("M,neg", [(300, False), (7, False), (20011, False), (4096, False), (64, False),
                                   (32768, False), (300, True), (4096, True)])
def test_linear_rows_ws_ffn1_onepass_scales(torch, M, neg):
    """FFN1 in one pass (kp = 3: ReLU + per-token quantization over all 2048 columns, the
    4 column slices' row maxima exchanged inside the launch) on k_gemm_wsy (quantization
    between the MFMAs), with row scales from 1e-35 to 1e25; bit-exact, and the exchange
    never timed out (status word 0).  neg: a negative bias and every third row of x zero, so
    those rows are all below zero before the ReLU (row maximum 0, scale 1e-5 / 127, and
    pre-ReLU quotients down to -1e10 that the code conversion must clamp to 0).  (kp = 4 / 5,
    the 32x32x32-MFMA variants: diagnostic build, tests/diag_variants.py.)"""
    kp = 3
    from qtx._lib import lib
    wsy = 1
    rng = np.random.default_rng(M + 31 * wsy + 7 * neg)
    qx, sx = O.quant_rows(rng.standard_normal((M, 512)).astype(f32))
    sx = (sx * np.float32(10.0) ** rng.integers(-33, 26, M)).astype(f32)
    qw, sw = O.quant_weight((rng.standard_normal((2048, 512)) * 0.05).astype(f32), 8)
    b = (rng.standard_normal(2048) * 1e-3).astype(f32)
    if neg:
        b = (-np.abs(b) * 1e3 - 1e-3).astype(f32)
        qx[::3] = 0
    wk = torch.empty((2048, 512), dtype=torch.int8, device="cuda")
    assert lib().qtx_pack_w_ws(P(dev(torch, qw)), 2048, 512, P(wk), S0) == 0
    h8 = torch.zeros((M + (M & 1), 2048), dtype=torch.int8, device="cuda")
    sh = torch.full((M,), -1.0, dtype=torch.float32, device="cuda")
    nb = (M + 31) // 32
    gx = torch.empty(((32 * M + 2048) // 4,), dtype=torch.float32, device="cuda")
    _rows_call(torch, A=dev(torch, _to_kp(qx)), sa=dev(torch, sx), W=wk, sw=dev(torch, sw),
               bias=dev(torch, b), M=M, N=2048, K=512, kp=kp, epi=3, pmax_out=gx, out8=h8,
               ldo8=2048, os=sh)
    h = O.linear_epilogue(O.int_gemm(qx, qw), sx, sw, b, relu=True)
    qh, s = O.quant_rows(h)
    if neg:
        assert (s[::3] == np.float32(1e-5) / np.float32(127)).all() and not qh[::3].any()
    np.testing.assert_array_equal(_from_kp(h8.cpu().numpy(), M), qh)
    np.testing.assert_array_equal(sh.cpu().numpy(), s)
    status = gx.view(torch.int32)[2 * (4 * 32 * nb) + 1].item()
    assert status == 0


@pytest.mark.parametrize("M,ks,lnq", [(7, 4, True), (300, 4, True), (2304, 4, True),
                                      (300, 2, True), (300, 8, True), (129, 4, False),
                                      (8192, 4, True)])
def test_linear_rows_res_ln_splitk(torch, oracle_model, M, ks, lnq):
    """FFN2 (epi 1, kp = 1, K = 2048) with K split over ks workgroups per row tile (int32
    partials, then the row-wise residual + LayerNorm + quant epilogue): bit-exact against the
    oracle, for the quantized KP output and the fp32 LayerNorm output (the encoder's last
    layer), ragged M included."""
    from qtx._lib import lib
    rng = np.random.default_rng(M + 7 * ks)
    qh, sh = O.quant_rows(np.maximum(rng.standard_normal((M, 2048)), 0).astype(f32))
    qw, sw = O.quant_weight((rng.standard_normal((512, 2048)) * 0.05).astype(f32), 8)
    wk = torch.empty((512, 2048), dtype=torch.int8, device="cuda")
    assert lib().qtx_pack_w_kp(P(dev(torch, qw)), 512, 2048, P(wk), S0) == 0
    b = rng.standard_normal(512).astype(f32)
    res = (rng.standard_normal((M, 512)) * 2).astype(f32)
    la, lb = oracle_model.dec[1]["ln"][0]
    xd = dev(torch, res.copy())
    part = torch.empty((ks * M * 512,), dtype=torch.int32, device="cuda")
    out = dict(lnq=torch.zeros((M + (M & 1), 512), dtype=torch.int8, device="cuda"),
               lns=torch.empty(M, dtype=torch.float32, device="cuda")) if lnq else \
        dict(lnout=torch.empty((M, 512), dtype=torch.float32, device="cuda"))
    _rows_call(torch, A=dev(torch, _to_kp(qh)), sa=dev(torch, sh), W=wk, sw=dev(torch, sw),
               bias=dev(torch, b), M=M, N=512, K=2048, epi=1, res=xd, xout=xd,
               ln_a=dev(torch, la), ln_b=dev(torch, lb), kp=1, part=part, ksplit=ks, **out)
    x = res + O.linear_epilogue(O.int_gemm(qh, qw), sh, sw, b)
    np.testing.assert_array_equal(xd.cpu().numpy(), x)
    ln = O.layer_norm(x, la, lb)
    if lnq:
        q, s2 = O.quant_rows(ln)
        np.testing.assert_array_equal(_from_kp(out["lnq"].cpu().numpy(), M), q)
        np.testing.assert_array_equal(out["lns"].cpu().numpy(), s2)
    else:
        np.testing.assert_array_equal(out["lnout"].cpu().numpy(), ln)


def test_linear_rows_splitk_bad_k_is_invalid(torch):
    """A split-K shape the launcher cannot tile (K / 64 not a multiple of 4 * ksplit) is an
    argument error (QTX_E_INVALID = 1 at the C-ABI), not a HIP error."""
    from qtx._lib import RowGemm, lib
    import ctypes as C
    M = 64
    z8 = torch.zeros((M, 512), dtype=torch.int8, device="cuda")
    f = torch.zeros(M * 512, dtype=torch.float32, device="cuda")
    a = RowGemm()
    kw = dict(A=z8, sa=f, W=z8, sw=f, bias=f, M=M, N=512, K=512, epi=1, res=f, xout=f,
              ln_a=f, ln_b=f, lnq=z8, lns=f, kp=1, part=f, ksplit=4)
    for k, v in kw.items():
        setattr(a, k, v.data_ptr() if hasattr(v, "data_ptr") else v)
    assert lib().qtx_linear_rows(C.byref(a), S0) == 1
    assert b"ksplit" in lib().qtx_last_error()


def _ws_pack_ref(w):
    """The WS order of qtx_pack_w_ws (include/qtx.h), restated in numpy: 1 KB block
    ((t*8 + w)*8 + s)*4 + j, lane l: W[512t + 64w + 16((l & 15) >> 2) + 4j + (l & 3)]
    [64s + 16(l >> 4) .. +16]."""
    N, K = w.shape
    t, wv, s, j, l = np.meshgrid(np.arange(N // 512), np.arange(8), np.arange(8), np.arange(4),
                                 np.arange(64), indexing="ij")
    n = 512 * t + 64 * wv + 16 * ((l & 15) >> 2) + 4 * j + (l & 3)
    k0 = 64 * s + 16 * (l >> 4)
    rows = w[n.reshape(-1)]                                  # [chunks, K]
    idx = k0.reshape(-1)[:, None] + np.arange(16)[None, :]
    return np.take_along_axis(rows, idx, axis=1).reshape(N, K)


def test_pack_w_ws(torch):
    rng = np.random.default_rng(5)
    w = rng.integers(-127, 128, (1024, 512)).astype(np.int8)
    out = torch.empty((1024, 512), dtype=torch.int8, device="cuda")
    from qtx._lib import lib
    assert lib().qtx_pack_w_ws(P(dev(torch, w)), 1024, 512, P(out), S0) == 0
    np.testing.assert_array_equal(out.cpu().numpy(), _ws_pack_ref(w))
    assert lib().qtx_pack_w_ws(P(dev(torch, w)), 1024, 256, P(out), S0) != 0   # K != 512


@pytest.mark.parametrize("M,nopipe", [(300, 0), (7, 0), (64, 0), (20011, 0),
                                     pytest.param(20011, 1, marks=pytest.mark.diag),
                                     pytest.param(300, 1, marks=pytest.mark.diag)])
def test_linear_rows_ws(torch, oracle_model, knob_env, M, nopipe):
    """kp = 2 (weight-stationary, K = 512): every epilogue bit-exact against the oracle —
    Q/K/V per-token quant (row-major out), FFN1 row maxima + hidden quant (KP out), O-proj
    residual + LayerNorm + quant (KP out) and its fp32 variant; M = 20011 runs several row
    blocks per workgroup and a ragged last block.  nopipe: the unpipelined 64-row kernel
    (QTX_WS_NOPIPE; RE_RES_LN always runs on it)."""
    from qtx._lib import lib
    if nopipe:
        knob_env("QTX_WS_NOPIPE", 1)
    rng = np.random.default_rng(M + 7)

    def weights(N):
        qw, sw = O.quant_weight((rng.standard_normal((N, 512)) * 0.05).astype(f32), 8)
        wk = torch.empty((N, 512), dtype=torch.int8, device="cuda")
        assert lib().qtx_pack_w_ws(P(dev(torch, qw)), N, 512, P(wk), S0) == 0
        return qw, sw, wk, rng.standard_normal(N).astype(f32)

    qx, sx = O.quant_rows(rng.standard_normal((M, 512)).astype(f32))
    ax = dev(torch, _to_kp(qx))
    # epi 0 (QKV)
    qw, sw, wk, b = weights(1536)
    out8 = torch.empty((3, M, 512), dtype=torch.int8, device="cuda")
    os_ = torch.empty((3, M), dtype=torch.float32, device="cuda")
    _rows_call(torch, A=ax, sa=dev(torch, sx), W=wk, sw=dev(torch, sw), bias=dev(torch, b),
               M=M, N=1536, K=512, epi=0, out8=out8, ldo8=512, o8_ts=M * 512, os=os_,
               os_ts=M, kp=2)
    y = O.linear_epilogue(O.int_gemm(qx, qw), sx, sw, b)
    for t in range(3):
        q, s = O.quant_rows(y[:, 512 * t:512 * (t + 1)])
        np.testing.assert_array_equal(out8[t].cpu().numpy(), q)
        np.testing.assert_array_equal(os_[t].cpu().numpy(), s)
    # epi 2 + 3 (FFN1), hidden written KP
    qw, sw, wk, b = weights(2048)
    pm = torch.empty((4, M), dtype=torch.float32, device="cuda")
    base = dict(A=ax, sa=dev(torch, sx), W=wk, sw=dev(torch, sw), bias=dev(torch, b),
                M=M, N=2048, K=512, kp=2)
    _rows_call(torch, epi=2, pmax_out=pm, **base)
    h = O.linear_epilogue(O.int_gemm(qx, qw), sx, sw, b, relu=True)
    np.testing.assert_array_equal(pm.cpu().numpy(), h.reshape(M, 4, 512).max(-1).T)
    h8 = torch.zeros((M + (M & 1), 2048), dtype=torch.int8, device="cuda")
    sh = torch.empty(M, dtype=torch.float32, device="cuda")
    _rows_call(torch, epi=3, pmax_in=pm, pmax_n=4, out8=h8, ldo8=2048, os=sh, **base)
    qh, s = O.quant_rows(h)
    np.testing.assert_array_equal(_from_kp(h8.cpu().numpy(), M), qh)
    np.testing.assert_array_equal(sh.cpu().numpy(), s)
    # kp = 3: the same hidden in ONE pass (row maxima exchanged between the column slices'
    # workgroups inside the launch; pmax_in unused, pmax_out = exchange scratch)
    h8b = torch.zeros_like(h8)
    shb = torch.full((M,), -1.0, dtype=torch.float32, device="cuda")
    gx = torch.empty(((32 * M + 2048) // 4,), dtype=torch.float32, device="cuda")
    _rows_call(torch, **{**base, "kp": 3}, epi=3, pmax_out=gx, out8=h8b, ldo8=2048, os=shb)
    np.testing.assert_array_equal(_from_kp(h8b.cpu().numpy(), M), qh)
    np.testing.assert_array_equal(shb.cpu().numpy(), s)
    # epi 1 (O-proj), next LayerNorm quantized KP, then the fp32 LayerNorm output variant
    qw, sw, wk, b = weights(512)
    res = (rng.standard_normal((M, 512)) * 2).astype(f32)
    la, lb = oracle_model.dec[1]["ln"][0]
    xd = dev(torch, res.copy())
    lnq = torch.zeros((M + (M & 1), 512), dtype=torch.int8, device="cuda")
    lns = torch.empty(M, dtype=torch.float32, device="cuda")
    obase = dict(A=ax, sa=dev(torch, sx), W=wk, sw=dev(torch, sw), bias=dev(torch, b), M=M,
                 N=512, K=512, epi=1, ln_a=dev(torch, la), ln_b=dev(torch, lb), kp=2)
    _rows_call(torch, res=xd, xout=xd, lnq=lnq, lns=lns, **obase)
    x = res + O.linear_epilogue(O.int_gemm(qx, qw), sx, sw, b)
    np.testing.assert_array_equal(xd.cpu().numpy(), x)
    ln = O.layer_norm(x, la, lb)
    q, s2 = O.quant_rows(ln)
    np.testing.assert_array_equal(_from_kp(lnq.cpu().numpy(), M), q)
    np.testing.assert_array_equal(lns.cpu().numpy(), s2)
    xd2 = dev(torch, res.copy())
    lnout = torch.empty((M, 512), dtype=torch.float32, device="cuda")
    _rows_call(torch, res=xd2, xout=xd2, lnout=lnout, **obase)
    np.testing.assert_array_equal(xd2.cpu().numpy(), x)
    np.testing.assert_array_equal(lnout.cpu().numpy(), ln)
