"""Per-kernel parity of the fused decode-step kernels (skinny GEMM prologue/epilogue modes,
one-query attention with KV-cache append) against the oracle — bit-exact."""
import ctypes as C

import numpy as np
import pytest

from oracle import qtx_oracle as O

pytestmark = pytest.mark.gpu
f32 = np.float32
S0 = C.c_void_p(0)
_KEEP = []


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(autouse=True)
def _release():
    yield
    _KEEP.clear()


def dev(torch, a):
    t = torch.from_numpy(np.ascontiguousarray(a)).cuda()
    _KEEP.append(t)
    return t


def P(t):
    return C.c_void_p(t.data_ptr()) if t is not None else S0


def call(name, *args):
    from qtx import _lib
    _lib.call(name, *args)


def weights(rng, N, K, bits):
    qw, sw = O.quant_weight((rng.standard_normal((N, K)) * 0.05).astype(f32), bits)
    b = rng.standard_normal(N).astype(f32)
    return qw, sw, b


def wdev(torch, qw, bits):
    wd = dev(torch, qw)
    if bits == 4:
        N, K = qw.shape
        packed = torch.empty((N, K // 2), dtype=torch.uint8, device="cuda")
        call("qtx_pack_int4", P(wd), N, K, P(packed), S0)
        _KEEP.append(packed)
        return packed
    return wd


def tile_max(y):
    """Per 16-column tile row absmax, [N/16, M] (EPI_ROWMAX output layout)."""
    M, N = y.shape
    return np.abs(y).reshape(M, N // 16, 16).max(-1).T


def head_max(ctx):
    """[8, B] per-head absmax of context rows [B, 512]."""
    return np.abs(ctx).reshape(-1, 8, 64).max(-1).T


@pytest.mark.parametrize("M", [1, 2, 16, 32, 45, 100, 256])
@pytest.mark.parametrize("N,K,flags,bits", [(512, 512, 2, 8), (1536, 512, 0, 8),
                                             (2048, 512, 5, 8), (512, 2048, 2, 4),
                                             (512, 2048, 2, 8)])
def test_skinny_i8(torch, M, N, K, flags, bits):
    rng = np.random.default_rng(M + N + K + flags)
    qx, sx = O.quant_rows(rng.standard_normal((M, K)).astype(f32))
    qw, sw, b = weights(rng, N, K, bits)
    res = rng.standard_normal((M, N)).astype(f32)
    out = dev(torch, res.copy())
    pm = torch.zeros((N // 16, M), dtype=torch.float32, device="cuda")
    call("qtx_skinny_linear", 0, P(dev(torch, qx)), P(dev(torch, sx)), S0, 0, S0, S0, S0, 0,
         P(wdev(torch, qw, bits)), P(dev(torch, sw)), P(dev(torch, b)), M, N, K, bits, flags,
         P(out), P(out), P(pm), S0)
    y = O.linear_epilogue(O.int_gemm(qx, qw), sx, sw, b, relu=bool(flags & 1))
    if flags & 2:
        y = res + y
    np.testing.assert_array_equal(out.cpu().numpy(), y)
    if flags & 4:
        np.testing.assert_array_equal(pm.cpu().numpy(), tile_max(y))


@pytest.mark.parametrize("M", [2, 5, 32, 98, 256])
def test_skinny_layernorm_prologue(torch, M, oracle_model):
    rng = np.random.default_rng(M)
    x = (rng.standard_normal((M, 512)) * 3).astype(f32)
    a, bb = oracle_model.dec[0]["ln"][2]
    qw, sw, b = weights(rng, 2048, 512, 8)
    out = torch.empty((M, 2048), dtype=torch.float32, device="cuda")
    pm = torch.zeros((2048 // 16, M), dtype=torch.float32, device="cuda")
    call("qtx_skinny_linear", 1, S0, S0, P(dev(torch, x)), 512, P(dev(torch, a)),
         P(dev(torch, bb)), S0, 0, P(dev(torch, qw)), P(dev(torch, sw)), P(dev(torch, b)), M,
         2048, 512, 8, 1 | 4, S0, P(out), P(pm), S0)
    qx, sx = O.quant_rows(O.layer_norm(x, a, bb))
    y = O.linear_epilogue(O.int_gemm(qx, qw), sx, sw, b, relu=True)
    np.testing.assert_array_equal(out.cpu().numpy(), y)
    np.testing.assert_array_equal(pm.cpu().numpy(), tile_max(y))


@pytest.mark.parametrize("M", [1, 3, 5, 32, 40, 100, 200, 256])
@pytest.mark.parametrize("K,nparts", [(2048, 128), (2048, 32), (512, 8), (512, 1)])
def test_skinny_partial_max_prologue(torch, M, K, nparts):
    """amode 2: fp32 rows quantized per token from partial row maxima (FFN2 from FFN1's
    per-tile maxima — 128 of 16 columns or 32 of 64 (k_skinny_wide); the output projection
    from the attention's per-head maxima).  K = 2048 with 8-bit weights and the residual
    runs the 8-wave k_skinny8_ffn2 up to M = 32 (M not a multiple of its 4-row blocks: 1, 3,
    5), the 4-wave k_skinny above (40) with 8- / 16-row blocks from M = 96 / 192 (100, 200,
    256), where the K = 512 projection runs N-split (k_skinny_wide, 8-row blocks)."""
    rng = np.random.default_rng(M + K + nparts)
    h = np.maximum(rng.standard_normal((M, K)), 0).astype(f32)
    h[0] = 0                                         # an all-zero row: clamp 1e-5
    parts = np.abs(h).reshape(M, nparts, K // nparts).max(-1).T.copy()   # [nparts, M]
    qw, sw, b = weights(rng, 512, K, 8)
    res = rng.standard_normal((M, 512)).astype(f32)
    out = dev(torch, res.copy())
    call("qtx_skinny_linear", 2, S0, S0, P(dev(torch, h)), K, S0, S0, P(dev(torch, parts)),
         nparts, P(dev(torch, qw)), P(dev(torch, sw)), P(dev(torch, b)), M, 512, K, 8, 2,
         P(out), P(out), S0, S0)
    qx, sx = O.quant_rows(h)
    np.testing.assert_array_equal(out.cpu().numpy(),
                                  res + O.linear_epilogue(O.int_gemm(qx, qw), sx, sw, b))


@pytest.mark.parametrize("M", [1, 3, 5, 32, 40, 100, 256])
@pytest.mark.parametrize("K", [512, 2048])
def test_skinny_own_max_prologue(torch, M, K):
    """amode 3: fp32 rows [M, K] quantized per token from their own row absmax (the fused
    decode's O / Oc projections and FFN2: rows the GEMM loads anyway; K = 2048 up to M = 32
    runs k_skinny8_ffn2, whose two half-row waves meet their maxima in LDS), the same
    results as amode 2 over complete partial maxima."""
    rng = np.random.default_rng(M + K + 3)
    h = rng.standard_normal((M, K)).astype(f32)
    if K == 2048:
        h = np.maximum(h, 0)                         # a ReLU hidden
    h[0] = 0                                         # an all-zero row: clamp 1e-5
    qw, sw, b = weights(rng, 512, K, 8)
    res = rng.standard_normal((M, 512)).astype(f32)
    out = dev(torch, res.copy())
    call("qtx_skinny_linear", 3, S0, S0, P(dev(torch, h)), K, S0, S0, S0, 0,
         P(dev(torch, qw)), P(dev(torch, sw)), P(dev(torch, b)), M, 512, K, 8, 2,
         P(out), P(out), S0, S0)
    qx, sx = O.quant_rows(h)
    np.testing.assert_array_equal(out.cpu().numpy(),
                                  res + O.linear_epilogue(O.int_gemm(qx, qw), sx, sw, b))


def vgroup4(v):
    """[B, n, 512] int8 values -> qtx_decode_attention's 4-key group layout
    [B, ceil(n/4), 512, 4] (include/qtx.h)."""
    B, n, D = v.shape
    g4 = (n + 3) // 4
    vp = np.zeros((B, 4 * g4, D), np.int8)
    vp[:, :n] = v
    return np.ascontiguousarray(vp.reshape(B, g4, 4, D).transpose(0, 1, 3, 2))


def vungroup4(vg, n):
    B, g4, D, _ = vg.shape
    return vg.transpose(0, 1, 3, 2).reshape(B, 4 * g4, D)[:, :n]


@pytest.mark.parametrize("B,step,kv_bs", [(2, 0, 8), (3, 5, 8), (32, 40, 72), (1, 127, 128),
                                          (4, 70, 72), (2, 15, 17), (2, 16, 17)])
def test_decode_self_attention(torch, B, step, kv_bs):
    rng = np.random.default_rng(B * 1000 + step)
    y = rng.standard_normal((B, 1536)).astype(f32)
    kc = rng.integers(-127, 128, (B, kv_bs, 512)).astype(np.int8)
    vc = rng.integers(-127, 128, (B, kv_bs, 512)).astype(np.int8)
    skc = rng.uniform(0.002, 0.03, (B, kv_bs)).astype(f32)
    svc = rng.uniform(0.002, 0.03, (B, kv_bs)).astype(f32)
    kcd, vcd, skd, svd = dev(torch, kc), dev(torch, vgroup4(vc)), dev(torch, skc), dev(torch, svc)
    stepd = dev(torch, np.array([step], np.int32))
    ctxd = torch.empty((B, 512), dtype=torch.float32, device="cuda")
    pm = torch.empty((8, B), dtype=torch.float32, device="cuda")
    for _ in range(2):      # the second call re-appends the same row: idempotent
        call("qtx_decode_attention", 1, P(dev(torch, y)), 1536, P(kcd), P(vcd), P(skd),
             P(svd), kv_bs, P(stepd), 0, S0, B, P(ctxd), P(pm), S0)
    qq, sq = O.quant_rows(y[:, :512])
    qk, sk = O.quant_rows(y[:, 512:1024])
    qv, sv = O.quant_rows(y[:, 1024:])
    kc[:, step], vc[:, step], skc[:, step], svc[:, step] = qk, qv, sk, sv
    np.testing.assert_array_equal(kcd.cpu().numpy(), kc)       # cache append
    np.testing.assert_array_equal(vungroup4(vcd.cpu().numpy(), kv_bs), vc)
    np.testing.assert_array_equal(skd.cpu().numpy(), skc)
    n = step + 1
    ctx, _ = O.attention(qq[:, None], sq[:, None], kc[:, :n], skc[:, :n], vc[:, :n],
                         svc[:, :n], np.ones((B, 1, n), np.uint8), dec=True)
    np.testing.assert_array_equal(ctxd.cpu().numpy(), ctx[:, 0])
    np.testing.assert_array_equal(pm.cpu().numpy(), head_max(ctx[:, 0]))


@pytest.mark.parametrize("B,S,holes", [(2, 16, 0), (32, 72, 0), (5, 128, 0), (3, 1, 0), (2, 17, 0),
                                       (8, 72, 1)])
def test_decode_cross_attention(torch, B, S, holes):
    """Suffix masks (padding), and with holes: masked keys inside the sentence and a fully
    masked row (the key loops stop after the last unmasked key, exactly)."""
    rng = np.random.default_rng(B + S)
    y = rng.standard_normal((B, 512)).astype(f32)
    kc = rng.integers(-127, 128, (B, S, 512)).astype(np.int8)
    vc = rng.integers(-127, 128, (B, S, 512)).astype(np.int8)
    skc = rng.uniform(0.002, 0.03, (B, S)).astype(f32)
    svc = rng.uniform(0.002, 0.03, (B, S)).astype(f32)
    mask = np.ones((B, S), np.uint8)
    for b in range(B):
        mask[b, rng.integers(1, S + 1):] = 0
    if holes:
        mask[:, 3:9:2] = 0
        mask[1, :] = 0
        mask[2, 70] = 1
    ctxd = torch.empty((B, 512), dtype=torch.float32, device="cuda")
    pm = torch.empty((8, B), dtype=torch.float32, device="cuda")
    call("qtx_decode_attention", 0, P(dev(torch, y)), 512, P(dev(torch, kc)), P(dev(torch, vgroup4(vc))),
         P(dev(torch, skc)), P(dev(torch, svc)), S, S0, S, P(dev(torch, mask)), B, P(ctxd),
         P(pm), S0)
    qq, sq = O.quant_rows(y)
    ctx, _ = O.attention(qq[:, None], sq[:, None], kc, skc, vc, svc, mask[:, None], dec=True)
    np.testing.assert_array_equal(ctxd.cpu().numpy(), ctx[:, 0])
    np.testing.assert_array_equal(pm.cpu().numpy(), head_max(ctx[:, 0]))


def oracle_first_argmax(logits):
    """OracleModel.generator's token rule on given logits: first argmax of
    (x - max) - lse with the canonical lane-split denominator; 0 for a non-finite row."""
    return O.log_softmax_argmax(logits)[1]


@pytest.mark.parametrize("case", ["random", "exact_ties", "near_ties", "collapse", "nan_rows"])
def test_decode_argmax_embed(torch, gpu_model, oracle_model, case):
    """The decode tail: fast path (one logit within 4e-6 of the max) and the exact
    log-softmax path (ties, near-ties, values that round onto the max's log-prob,
    non-finite rows) give the oracle's first-argmax token and its embedding."""
    rng = np.random.default_rng(hash(case) % 1000)
    M, V = 32, 4444
    lg = (rng.standard_normal((M, V)) * 2).astype(f32)
    if case == "exact_ties":
        for r in range(M):
            j = rng.integers(0, V, 3)
            lg[r, j] = lg[r].max() + 1.0
    elif case == "near_ties":
        for r in range(M):
            j = rng.integers(0, V, 2)
            mx = lg[r].max() + 0.5
            lg[r, j[0]] = mx
            lg[r, j[1]] = np.nextafter(mx, f32(-np.inf)) if r % 2 else mx - f32(3e-6)
    elif case == "collapse":          # many values within a few ulps: lse-rounding decides
        for r in range(M):
            mx = f32(rng.uniform(1, 6))
            j = rng.choice(V, 6, replace=False)
            lg[r, j] = mx - f32(1e-7) * rng.integers(0, 12, 6).astype(f32)
    elif case == "nan_rows":          # torch's rule: NaN / +inf / all -inf rows -> id 0
        lg[0, :] = np.nan
        lg[1, 5] = np.nan
        lg[2, 17] = np.inf
        lg[3, :] = -np.inf
        lg[4, 9] = -np.inf            # a zero probability among finite values: a normal row
        lg[5, V - 1] = np.nan
    ids = torch.zeros((M, 72), dtype=torch.int64, device="cuda")
    step = torch.tensor([7, 0], dtype=torch.int32, device="cuda")
    xn = torch.empty((M, 512), dtype=torch.float32, device="cuda")
    call("qtx_decode_argmax_embed", gpu_model.handle, P(dev(torch, lg)), M, P(ids), 72, P(step),
         P(xn), S0)
    got = ids[:, 8].cpu().numpy()
    want = oracle_first_argmax(lg)
    if case == "nan_rows":
        assert (want[[0, 1, 2, 3, 5]] == 0).all()
    np.testing.assert_array_equal(got, want)
    assert step.cpu().tolist() == [8, 0]
    ids_all = ids[:, 8].cpu().numpy()
    emb = oracle_model.embed(ids_all[:, None], oracle_model.tgt_lut, pos0=8)[:, 0]
    np.testing.assert_array_equal(xn.cpu().numpy(), emb)
