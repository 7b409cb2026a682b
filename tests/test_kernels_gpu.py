"""Numerics of every gfx950 kernel against the fp32 PyTorch reference of the
same op (the CPU path of distributed_tf_serving_amd.ops)."""
import copy

import pytest
import torch

from distributed_tf_serving_amd import ops
from distributed_tf_serving_amd.config import ModelConfig
from distributed_tf_serving_amd.models import build_model

pytestmark = pytest.mark.gpu


def _close(a, b, rtol, atol, what=""):
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (err > tol).sum().item()
    assert bad == 0, f"{what}: {bad}/{a.numel()} mismatches, max err {err.max().item():.4g}"


def test_pack_ids(cuda):
    ids = torch.randint(-(1 << 40), 1 << 40, (33, 43), dtype=torch.int64)
    out = ops.pack_ids(ids.to(cuda), modulo=1000003)
    assert out.dtype == torch.int32
    assert torch.equal(out.cpu(), ops.pack_ids(ids, modulo=1000003))
    mf = torch.randint(1, 1000, (43,), dtype=torch.int64)
    of = torch.cumsum(mf, 0) - mf
    out = ops.pack_ids(ids.to(cuda), modulo_f=mf.to(cuda), offset_f=of.to(cuda))
    assert torch.equal(out.cpu(), ops.pack_ids(ids, modulo_f=mf, offset_f=of))


@pytest.mark.parametrize("D", [8, 16, 32, 64, 128])
@pytest.mark.parametrize("F", [1, 43, 70])
def test_embed_fm(cuda, D, F):
    V, B = 5000, 37
    g = torch.Generator().manual_seed(D * 100 + F)
    table = (torch.rand(V, D, generator=g) - 0.5).to(torch.bfloat16)
    lin = torch.rand(V, generator=g) - 0.5
    ids = torch.randint(-10**9, 10**9, (B, F), generator=g)
    wts = torch.rand(B, F, generator=g) * 2
    for ids_dt in (torch.int64, torch.int32):
        x, fm = ops.embed(table.to(cuda), ids.to(ids_dt).to(cuda), wts.to(cuda), lin=lin.to(cuda), modulo=V,
                          bias=0.25, want_x=True, want_fm=True, fm2=True)
        xr, fmr = ops.embed(table, ids.to(ids_dt), wts, lin=lin, modulo=V, bias=0.25, want_x=True, want_fm=True,
                            fm2=True)
        _close(x, xr, 1e-2, 1e-3, "x")
        _close(fm, fmr, 2e-3, 2e-3 * F, "fm")
    # no weights, no lin, only first-order off
    x, fm = ops.embed(table.to(cuda), ids.to(cuda), None, modulo=V, want_x=True, want_fm=True, fm2=False)
    xr, fmr = ops.embed(table, ids, None, modulo=V, want_x=True, want_fm=True, fm2=False)
    _close(x, xr, 1e-2, 1e-3, "x nowts")
    _close(fm, fmr, 1e-5, 1e-5, "bias only")


def test_embed_per_field_tables(cuda):
    T, rows, D, B = 30, 1000, 64, 19
    table = (torch.rand(T * rows, D) - 0.5).to(torch.bfloat16)
    mf = torch.full((T,), rows, dtype=torch.int64)
    of = torch.arange(T, dtype=torch.int64) * rows
    ids = torch.randint(0, 10**7, (B, T))
    x, _ = ops.embed(table.to(cuda), ids.to(cuda), None, modulo_f=mf.to(cuda), offset_f=of.to(cuda))
    xr, _ = ops.embed(table, ids, None, modulo_f=mf, offset_f=of)
    _close(x, xr, 0, 0, "per-field")


def test_embed_row_shards(cuda):
    # row-wise sharded tables: rows outside [lo, lo+n) must contribute zeros
    T, rows, D, B = 6, 1000, 64, 33
    lo = torch.tensor([0, 250, 500, 750, 100, 999], dtype=torch.int64)
    n = torch.tensor([250, 250, 250, 250, 0, 1], dtype=torch.int64)
    of = torch.cumsum(torch.cat([torch.zeros(1, dtype=torch.int64), n[:-1]]), 0)
    table = (torch.rand(int(n.sum()) + 1, D) - 0.5).to(torch.bfloat16)
    mf = torch.full((T,), rows, dtype=torch.int64)
    ids = torch.randint(0, 10**7, (B, T))
    wts = torch.rand(B, T)
    args = dict(modulo_f=mf, offset_f=of, shard_lo_f=lo, shard_n_f=n)
    x, _ = ops.embed(table.to(cuda), ids.to(cuda), wts.to(cuda), **{k: v.to(cuda) for k, v in args.items()})
    xr, _ = ops.embed(table, ids, wts, **args)
    _close(x, xr, 0, 0, "row shards")
    assert (xr.view(B, T, D)[:, 4] == 0).all()  # empty shard
    own = (torch.remainder(ids, rows) - lo >= 0) & (torch.remainder(ids, rows) - lo < n)
    assert ((xr.view(B, T, D).abs().sum(-1) > 0) <= own).all()


def test_sharded_dlrm_single_rank_gpu(cuda):
    from distributed_tf_serving_amd.config import ModelConfig
    from distributed_tf_serving_amd.parallel.dist import DistContext
    from distributed_tf_serving_amd.parallel.embedding_sharding import ShardedDLRM

    cfg = ModelConfig(family="dlrm", table_rows=5000, mlp_dims=(256, 128))
    ref = build_model(cfg, cuda)
    m = ShardedDLRM(cfg, DistContext(device=cuda), device=cuda)
    ids = torch.randint(0, 1 << 40, (300, 43), device=cuda)
    wts = torch.rand(300, 43, device=cuda)
    _close(m(ids, wts), ref(ids, wts), 0, 1e-6, "sharded dlrm (1 rank)")


@pytest.mark.parametrize("mean", [False, True])
def test_embedding_bag(cuda, mean):
    R, D, nb = 3000, 64, 41
    table = (torch.rand(R, D) - 0.5).to(torch.bfloat16)
    lens = torch.randint(0, 9, (nb,))
    offsets = torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(lens, 0)])
    idx = torch.randint(0, 10**6, (int(offsets[-1]),))
    psw = None if mean else torch.rand(idx.numel())
    out = ops.embedding_bag(table.to(cuda), idx.to(cuda), offsets.to(cuda),
                            None if psw is None else psw.to(cuda), modulo=R, mean=mean)
    ref = ops.embedding_bag(table, idx, offsets, psw, modulo=R, mean=mean)
    _close(out, ref, 1e-4, 1e-4, "bag")


GEMM_SHAPES = [(1, 1024, 2752), (37, 256, 512), (100, 64, 16), (512, 1024, 2752), (513, 512, 1024),
               (2048, 1024, 2752), (4096, 256, 512), (8192, 512, 1024), (300, 2752, 2752)]


@pytest.mark.parametrize("M,N,K", GEMM_SHAPES)
@pytest.mark.parametrize("act", ["none", "relu", "sigmoid"])
def test_gemm_bf16(cuda, M, N, K, act):
    g = torch.Generator().manual_seed(M + N + K)
    x = (torch.randn(M, K, generator=g)).to(torch.bfloat16)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, generator=g) * 0.1
    y = ops.linear(x.to(cuda), W.to(cuda), b.to(cuda), act, out_f32=True)
    ref = ops.linear(x, W, b, act, out_f32=True)
    _close(y, ref, 2e-3, 2e-3, f"gemm {M}x{N}x{K} {act}")
    yb = ops.linear(x.to(cuda), W.to(cuda), b.to(cuda), act)
    assert yb.dtype == torch.bfloat16
    _close(yb, ref, 1e-2, 1e-2, "gemm bf16 out")


@pytest.mark.parametrize("variant", [4, 8, 10, 14, 17, 18])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (300, 200, 128), (8192, 1024, 2752), (1000, 2752, 2752),
                                   (16384, 512, 1024), (513, 1024, 192)])
def test_gemm_variants_bf16(cuda, variant, M, N, K):
    g = torch.Generator().manual_seed(M + 7 * N + K + variant)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, generator=g) * 0.1
    h = ops.hip()
    for _ in range(3):  # repeat: a pipeline race shows up as run-to-run differences
        y = h.gemm(x.to(cuda), W.to(cuda), b.to(cuda), 1, None, None, True, None, None, None, variant)
        _close(y, ops.linear(x, W, b, "relu", out_f32=True), 2e-3, 2e-3, f"v{variant} {M}x{N}x{K}")


@pytest.mark.parametrize("variant", [17, 18])
@pytest.mark.parametrize("M,N,K", [(8192, 1024, 2752), (1000, 2752, 2752), (513, 1024, 192), (700, 1020, 256)])
@pytest.mark.parametrize("epi", [0, 1, 2])
def test_gemm_8phase_bf16_out_epilogues(cuda, variant, M, N, K, epi):
    """bf16 output of the 8-phase tile (the LDS-staged epilogue when N % 8 ==
    0, the register epilogue otherwise: N = 1020) for none / ReLU / sigmoid,
    ragged M and N, vs the fp32 CPU reference."""
    g = torch.Generator().manual_seed(M + 3 * N + K + epi)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, generator=g) * 0.1
    y = ops.hip().gemm(x.to(cuda), W.to(cuda), b.to(cuda), epi, None, None, False, None, None, None, variant)
    ref = ops.linear(x, W, b, {0: "none", 1: "relu", 2: "sigmoid"}[epi], out_f32=True)
    assert y.dtype == torch.bfloat16 and y.shape == (M, N)
    _close(y, ref, 1e-2, 1e-2, f"8-phase bf16 out v{variant} {M}x{N}x{K} epi {epi}")


@pytest.mark.parametrize("variant", [17, 18])
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (8192, 2752, 2752), (700, 1024, 2816)])
def test_gemm_8phase_fp8(cuda, M, N, K, variant):
    g = torch.Generator().manual_seed(M + N)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16)
    xq, sx = ops.quant_rows_fp8(x.to(cuda), ops.FP8_K_PAD)
    wq, sw = ops.quant_rows_fp8(W.to(cuda), ops.FP8_K_PAD)
    b = torch.randn(N, generator=g) * 0.1
    y = ops.hip().gemm(xq, wq, b.to(cuda), 1, None, None, True, sx, sw, None, variant)
    ref = ops.linear_fp8(xq.cpu(), sx.cpu(), wq.cpu(), sw.cpu(), b, "relu", out_f32=True)
    _close(y, ref, 2e-3, 2e-3, f"fp8 8-phase v{variant}")


def test_gemm_layout_asymmetric(cuda):
    # A = I (padded), W asymmetric: C must equal W^T exactly (catches row/col swaps)
    M = N = 64
    K = 64
    A = torch.eye(M, K).to(torch.bfloat16)
    W = torch.arange(N * K, dtype=torch.float32).view(N, K).remainder(97).to(torch.bfloat16)
    C = ops.linear(A.to(cuda), W.to(cuda), None, out_f32=True).cpu()
    assert torch.equal(C, W.float().t())


@pytest.mark.parametrize("M,N,K", [(64, 64, 128), (37, 256, 512), (512, 1024, 2752), (2048, 512, 1024)])
def test_gemm_fp8(cuda, M, N, K):
    g = torch.Generator().manual_seed(7 + M)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    W = torch.randn(N, K, generator=g).to(torch.bfloat16) / K ** 0.5
    xq, sx = ops.quant_rows_fp8(x)
    wq, sw = ops.quant_rows_fp8(W.to(torch.bfloat16))
    b = torch.randn(N, generator=g) * 0.1
    y = ops.linear_fp8(xq.to(cuda), sx.to(cuda), wq.to(cuda), sw.to(cuda), b.to(cuda), "relu", out_f32=True)
    ref = ops.linear_fp8(xq, sx, wq, sw, b, "relu", out_f32=True)
    _close(y, ref, 2e-3, 2e-3, "fp8 gemm")


@pytest.mark.parametrize("M,N,K", [(64, 64, 128), (300, 512, 2752), (8192, 1024, 2752), (1000, 2752, 2752)])
def test_gemm_fp8_k_padded(cuda, M, N, K):
    # the model path: K padded to 128 (zero columns), full 128-deep MX-fp8 tiles
    g = torch.Generator().manual_seed(11 + M)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    W = torch.randn(N, K, generator=g).to(torch.bfloat16) / K ** 0.5
    xq, sx = ops.quant_rows_fp8(x.to(cuda), ops.FP8_K_PAD)
    wq, sw = ops.quant_rows_fp8(W.to(cuda), ops.FP8_K_PAD)
    assert xq.shape[1] % 128 == 0 and (xq[:, K:].view(torch.uint8) == 0).all()
    b = torch.randn(N, generator=g) * 0.1
    y = ops.linear_fp8(xq, sx, wq, sw, b.to(cuda), "relu", out_f32=True)
    ref = ops.linear_fp8(xq.cpu(), sx.cpu(), wq.cpu(), sw.cpu(), b, "relu", out_f32=True)
    _close(y, ref, 2e-3, 2e-3, "fp8 gemm (K padded)")


def test_quant_rows_fp8(cuda):
    x = (torch.randn(77, 2752) * 3).to(torch.bfloat16)
    q, s = ops.quant_rows_fp8(x.to(cuda))
    qr, sr = ops.quant_rows_fp8(x)
    _close(s, sr, 1e-6, 0, "scale")
    deq = q.cpu().float() * s.cpu()[:, None]
    deqr = qr.float() * sr[:, None]
    # at most one e4m3 ulp apart (multiply-by-reciprocal vs divide): 3 mantissa
    # bits = 1/8 relative at the bottom of a binade
    _close(deq, deqr, 0.126, 1e-6, "fp8 values")
    exact = (deq == deqr).float().mean().item()
    assert exact > 0.99, f"only {exact:.4f} of fp8 values bit-identical"


@pytest.mark.parametrize("M,N,K", [(100, 256, 512), (1000, 2752, 2816), (8192, 2752, 2816)])
def test_gemm_mx_block_scaled_input(cuda, M, N, K):
    # activations in OCP MX-fp8 (per-32 E8M0 block scales fed to the MFMA)
    g = torch.Generator().manual_seed(3 + M)
    x = torch.randn(M, K, generator=g) * torch.exp2(torch.randint(-6, 6, (1, K // 32), generator=g).float()
                                                     ).repeat_interleave(32, dim=1)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16)
    q, s = ops.quant_mx_fp8(x, 128)
    wq, sw = ops.quant_rows_fp8(W.to(cuda), ops.FP8_K_PAD)
    b = torch.randn(N, generator=g) * 0.1
    y = ops.linear_fp8(q.to(cuda), None, wq, sw, b.to(cuda), "relu", out_f32=True, sx_blk=s.to(cuda))
    ref = ops.linear_fp8(q, None, wq.cpu(), sw.cpu(), b, "relu", out_f32=True, sx_blk=s)
    _close(y, ref, 2e-3, 2e-3, f"MX-fp8 input {M}x{N}x{K}")


@pytest.mark.parametrize("M", [100, 8192])
def test_cross_mx_epilogue(cuda, M):
    # the cross epilogue writes bf16 y AND y as the next layer's MX-fp8 operand
    N, K = 2752, 2816
    g = torch.Generator().manual_seed(M)
    x0 = torch.randn(M, N, generator=g).to(torch.bfloat16)
    xl = torch.randn(M, N, generator=g).to(torch.bfloat16)
    W = (torch.randn(N, N, generator=g) / N ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, generator=g) * 0.1
    xq, sx = ops.quant_rows_fp8(xl.to(cuda), ops.FP8_K_PAD)
    wq, sw = ops.quant_rows_fp8(W.to(cuda), ops.FP8_K_PAD)
    # poison the output buffers' previous contents: padding must be written
    torch.cuda.empty_cache()
    junk = torch.full((M, K), 0x7F, dtype=torch.uint8, device=cuda)
    del junk
    y, q, sq = ops.linear_fp8(xq, sx, wq, sw, b.to(cuda), x0=x0.to(cuda), xl=xl.to(cuda), emit_mx=K)
    yr, qr, sqr = ops.linear_fp8(xq.cpu(), sx.cpu(), wq.cpu(), sw.cpu(), b, x0=x0, xl=xl, emit_mx=K)
    _close(y, yr, 2e-2, 2e-2, "cross y")
    assert q.shape == (M, K) and sq.shape == (M, K // 32)
    assert (q[:, N:].view(torch.uint8) == 0).all(), "K padding of the MX output not zero"
    assert (sq[:, N // 32:] == 127).all()
    # the scale is the block's own exponent (same fp32 values up to accumulation order)
    same = (sq.cpu() == sqr).float().mean().item()
    assert same > 0.99, f"only {same:.4f} of block scales match"
    # dequantised values: within one e4m3 step of the fp32 result, per block
    deq = ops.dequant_mx_fp8(q.cpu(), sq.cpu())[:, :N]
    yf = yr.float()
    blk_amax = yf.abs().view(M, N // 32, 32).amax(dim=2).repeat_interleave(32, dim=1)
    assert ((deq - yf).abs() <= blk_amax / 16 + 2e-2 * yf.abs() + 1e-3).all()


@pytest.mark.parametrize("M,N", [(1, 8), (37, 264), (1000, 2752), (4099, 2752)])
def test_cross_combine(cuda, M, N):
    """Split cross layer combine pass: z = x0*y + xl, its e4m3 quantisation and
    the head dot, against the CPU reference of the same op."""
    g = torch.Generator().manual_seed(M + N)
    y, x0, xl = (torch.randn(M, N, generator=g).to(torch.bfloat16) for _ in range(3))
    hw = torch.randn(N, generator=g) * 0.05
    z, q, s, d = ops.cross_combine(y.to(cuda), x0.to(cuda), xl.to(cuda), True, ops.FP8_K_PAD, hw.to(cuda))
    zr, qr, sr, dr = ops.cross_combine(y, x0, xl, True, ops.FP8_K_PAD, hw)
    torch.cuda.synchronize()
    assert torch.equal(z.cpu(), zr)
    _close(s, sr, 1e-6, 0, "scale")
    assert q.shape == qr.shape
    # x * (1/s) on the GPU vs x / s on the CPU: at most 1 e4m3 ulp apart (<= 1/8 relative)
    _close(q.float(), qr.float(), 0.126, 1e-3, "q")
    _close(d, dr, 1e-4, 1e-3, "dot")
    # head-only form writes nothing else
    z2, q2, s2, d2 = ops.cross_combine(y.to(cuda), x0.to(cuda), xl.to(cuda), False, 0, hw.to(cuda))
    assert z2 is None and q2 is None and s2 is None
    _close(d2, dr, 1e-4, 1e-3, "dot only")


@pytest.mark.parametrize("B,F,D", [(1, 43, 64), (4099, 43, 64), (300, 13, 32), (77, 64, 16)])
def test_embed_fp8_matches_quant_rows(cuda, B, F, D):
    """The gather's own e4m3 copy of x == quant_rows_fp8(x) (same rounding,
    same K padding) and x itself is unchanged."""
    g = torch.Generator().manual_seed(B + F + D)
    table = torch.randn(5000, D, generator=g).to(torch.bfloat16).to(cuda)
    ids = torch.randint(0, 1 << 40, (B, F), generator=g).to(cuda)
    wts = torch.rand(B, F, generator=g).to(cuda)
    x, q, sc = ops.embed_fp8(table, ids, wts, 5000, ops.FP8_K_PAD)
    xr, _ = ops.embed(table, ids, wts, modulo=5000, want_x=True)
    qr, sr = ops.quant_rows_fp8(xr, ops.FP8_K_PAD)
    torch.cuda.synchronize()
    assert torch.equal(x, xr)
    assert torch.equal(sc, sr)
    assert q.shape == qr.shape and torch.equal(q.view(torch.uint8), qr.view(torch.uint8))


def test_dcn_v2_split_cross_matches_fused(cuda, monkeypatch):
    """DCN-v2 fp8: split cross layers (plain GEMM + combine/quant/head pass) vs
    the fused cross epilogue + quant_rows + head, same weights."""
    from distributed_tf_serving_amd.config import ModelConfig
    from distributed_tf_serving_amd.models import build_model

    cfg = ModelConfig(family="dcn_v2", vocab_size=20000, embed_dim=64, num_fields=43, mlp_dims=(1024, 512, 256),
                      num_cross_layers=3, gemm_dtype="fp8")
    m = build_model(cfg, cuda)
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(0, 1 << 30, (4096, 43), generator=g).to(cuda)
    wts = torch.rand(4096, 43, generator=g).to(cuda)
    a = m(ids, wts)  # split cross layers
    # the fused cross epilogue, layer by layer, on the same weights
    x0, _ = ops.embed(m.emb, ids, wts, modulo=cfg.vocab_size, want_x=True)
    xl = x0
    for i in range(cfg.num_cross_layers):
        xl = m._cross_layer(i, x0, xl)
    cross = ops.head(xl, m.head_wc, 0.0, sigmoid=False)
    b = m.mlp.forward_head(x0, m.head_wd, m.head_b, extra=cross)
    torch.cuda.synchronize()
    assert (a - b).abs().max().item() < 0.02


@pytest.mark.parametrize("M,N,same", [(700, 2752, False), (256, 264, True), (1030, 512, False)])
def test_cross_gemm_fp8_staged_epilogue(cuda, M, N, same):
    """One-launch DCN-v2 cross layer (8-phase fp8 GEMM + LDS-staged cross
    epilogue) == plain fp8 GEMM + cross_combine (z bit for bit, per-tile partial
    logits summing to the combine's dot), and close to the fp32 CPU reference;
    ragged M / N tiles, x_l = x0 (first layer)."""
    g = torch.Generator().manual_seed(M + N)
    K = -(-N // 128) * 128
    x0 = (torch.randn(M, N, generator=g) * 0.5).to(torch.bfloat16)
    xl = x0 if same else (torch.randn(M, N, generator=g) * 0.5).to(torch.bfloat16)
    W = torch.randn(N, N, generator=g) / N ** 0.5
    Wq, sw = ops.quant_rows_fp8(W.to(torch.bfloat16), 128)
    b = torch.randn(N, generator=g) * 0.1
    q, sx = ops.quant_rows_fp8(xl, 128)
    hw = torch.randn(N, generator=g) * 0.05
    dq, dsx, dW, dsw, db, dx0, dhw = (t.to(cuda) for t in (q, sx, Wq, sw, b, x0, hw))
    dxl = dx0 if same else xl.to(cuda)
    assert q.shape[1] == K and Wq.shape == (N, K)
    z, d = ops.cross_gemm_fp8(dq, dsx, dW, dsw, db, dx0, dxl, want_z=True, head_w=dhw)
    y = ops.linear_fp8(dq, dsx, dW, dsw, db)
    zr, _, _, dr = ops.cross_combine(y, dx0, dxl, True, 0, dhw)
    z2, d2 = ops.cross_gemm_fp8(dq, dsx, dW, dsw, db, dx0, dxl, want_z=False, head_w=dhw)
    z3, d3 = ops.cross_gemm_fp8(dq, dsx, dW, dsw, db, dx0, dxl, want_z=True)
    torch.cuda.synchronize()
    assert d.shape == (-(-N // 256), M) and z2 is None and d3 is None
    assert torch.equal(z.cpu(), zr.cpu()) and torch.equal(z3.cpu(), zr.cpu())
    _close(d.sum(0), dr, 1e-4, 1e-4, "partial logits")
    assert torch.equal(d2.cpu(), d.cpu())
    zc, dc = ops.cross_gemm_fp8(q, sx, Wq, sw, b, x0, xl, want_z=True, head_w=hw)
    _close(z, zc, 2e-2, 2e-2, "z vs CPU")
    _close(d, dc, 2e-2, 2e-2, "dot vs CPU")


def test_dcn_v2_fused_cross_matches_split(cuda, monkeypatch):
    """A full-chip DCN-v2 fp8 step (6144 rows: 264 cross tiles) through the
    one-launch cross layers vs the split GEMM + combine path, same weights."""
    from distributed_tf_serving_amd.config import ModelConfig
    from distributed_tf_serving_amd.models import build_model

    cfg = ModelConfig(family="dcn_v2", vocab_size=20000, embed_dim=64, num_fields=43, mlp_dims=(1024, 512, 256),
                      num_cross_layers=3, gemm_dtype="fp8")
    m = build_model(cfg, cuda)
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(0, 1 << 30, (6144, 43), generator=g).to(cuda)
    wts = torch.rand(6144, 43, generator=g).to(cuda)
    assert ops.cross_gemm_fits(6144, 2752)
    a = m(ids, wts)
    monkeypatch.setattr(ops, "cross_gemm_fits", lambda M, N: False)
    b = m(ids, wts)
    torch.cuda.synchronize()
    assert (a - b).abs().max().item() < 1e-3


def test_cross_v2_epilogue(cuda):
    M, d = 130, 256
    x0 = torch.randn(M, d).to(torch.bfloat16)
    xl = torch.randn(M, d).to(torch.bfloat16)
    W = (torch.randn(d, d) / d ** 0.5).to(torch.bfloat16)
    b = torch.randn(d) * 0.1
    y = ops.cross_v2(x0.to(cuda), xl.to(cuda), W.to(cuda), b.to(cuda))
    ref = ops.cross_v2(x0, xl, W, b)
    _close(y, ref, 2e-2, 2e-2, "cross_v2")


@pytest.mark.parametrize("d", [64, 2752, 4096])
def test_cross_v1(cuda, d):
    B, L = 45, 3
    x0 = (torch.randn(B, d) * 0.1).to(torch.bfloat16)
    w = torch.randn(L, d) / d ** 0.5
    b = torch.randn(L, d) * 0.01
    hw = torch.randn(d) / d ** 0.5
    x, dot = ops.cross_v1(x0.to(cuda), w.to(cuda), b.to(cuda), want_x=True, head_w=hw.to(cuda))
    xr, dr = ops.cross_v1(x0, w, b, want_x=True, head_w=hw)
    _close(x, xr, 1e-2, 1e-3, "cross_v1 x")
    _close(dot, dr, 1e-3, 1e-3, "cross_v1 dot")


@pytest.mark.parametrize("T", [1, 26, 30, 31])
def test_dot_interaction(cuda, T):
    B = 23
    dense = torch.randn(B, 64).to(torch.bfloat16)
    emb = torch.randn(B, T, 64).to(torch.bfloat16)
    z = ops.dot_interaction(dense.to(cuda), emb.to(cuda))
    zr = ops.dot_interaction(dense, emb)
    assert z.shape == zr.shape
    _close(z, zr, 1e-2, 5e-2, "dot")


@pytest.mark.parametrize("T,ids64", [(1, True), (26, False), (30, True), (31, False)])
def test_dot_interaction_gather(cuda, T, ids64):
    """K1 fused into K5: the interaction reads its rows from the tables (row
    view of the ids, per-table modulo + offset, negative ids) == gather +
    dot_interaction on the GPU (bit for bit) and the fp32 CPU reference."""
    g = torch.Generator().manual_seed(T)
    B, rows = 517, 1000
    dense = torch.randn(B, 64, generator=g).to(torch.bfloat16)
    table = torch.randn(T * rows, 64, generator=g).to(torch.bfloat16)
    full = torch.randint(-(1 << 40), 1 << 40, (B, T + 13), generator=g)
    ids = (full if ids64 else full.to(torch.int32))[:, 13:]  # a row view, like DLRM.sparse_ids
    mod = torch.full((T,), rows, dtype=torch.int64)
    off = torch.arange(T, dtype=torch.int64) * rows
    dc, tc, ic, mc, oc = (t.to(cuda) for t in (dense, table, full if ids64 else full.to(torch.int32), mod, off))
    z = ops.dot_interaction_gather(dc, tc, ic[:, 13:], mc, oc)
    emb, _ = ops.embed(tc, ic[:, 13:], None, modulo_f=mc, offset_f=oc, want_x=True)
    z2 = ops.dot_interaction(dc, emb.view(B, T, 64))
    zr = ops.dot_interaction_gather(dense, table, ids, mod, off)
    torch.cuda.synchronize()
    assert z.shape == zr.shape == (B, ops.interaction_cols(T, 64))
    assert torch.equal(z.cpu(), z2.cpu())
    _close(z, zr, 1e-2, 5e-2, "dot gather")


@pytest.mark.parametrize("M,nd", [(1, 13), (517, 13), (4096, 64), (33, 1)])
def test_bottom_mlp3(cuda, M, nd):
    """Fused DLRM bottom MLP (pad + 3 relu layers in one kernel, a row view of
    feat_wts) vs the same layers one GEMM at a time on the GPU and the fp32
    CPU reference."""
    g = torch.Generator().manual_seed(M + nd)
    full = torch.rand(M, nd + 30, generator=g) * 2 - 1
    dims, k, layers = ops.BOTTOM_MLP3_DIMS, 64, []
    for n in dims:
        layers.append(((torch.randn(n, k, generator=g) / k ** 0.5).to(torch.bfloat16), torch.randn(n, generator=g) * 0.1))
        k = n
    dl = [(w.to(cuda), b.to(cuda)) for w, b in layers]
    y = ops.bottom_mlp3(full.to(cuda)[:, :nd + 5], nd, dl)
    x = torch.zeros(M, 64, dtype=torch.bfloat16, device=cuda)
    x[:, :nd] = full[:, :nd].to(torch.bfloat16).to(cuda)
    for w, b in dl:
        x = ops.linear(x, w, b, "relu")
    yr = ops.bottom_mlp3(full[:, :nd + 5], nd, layers)
    torch.cuda.synchronize()
    assert y.shape == (M, 64) and y.dtype == torch.bfloat16
    _close(y, x, 1e-2, 1e-2, "vs layer by layer")
    _close(y, yr, 2e-2, 2e-2, "vs CPU")


def test_head(cuda):
    x = torch.randn(101, 256).to(torch.bfloat16)
    w = torch.randn(256) * 0.05
    e = torch.randn(101)
    y = ops.head(x.to(cuda), w.to(cuda), 0.3, e.to(cuda), True)
    _close(y, ops.head(x, w, 0.3, e, True), 1e-5, 1e-5, "head")


@pytest.mark.parametrize("M,N,K", [(1, 256, 512), (37, 256, 512), (4096, 256, 512), (8192, 256, 512),
                                   (5000, 256, 1024), (300, 128, 256), (77, 64, 128), (129, 40, 64),
                                   # ragged rows / columns at the served batch sizes
                                   (16421, 256, 512), (9000, 200, 256), (8200, 136, 128), (8192, 256, 1024)])
@pytest.mark.parametrize("act", ["relu", "none"])
def test_linear_head_fused(cuda, M, N, K, act):
    g = torch.Generator().manual_seed(M * 3 + N + K)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    W = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, generator=g) * 0.1
    hw = torch.randn(N, generator=g) * 0.05
    e = torch.randn(M, generator=g)
    for extra, sig in ((e, True), (None, False)):
        y = ops.linear_head(x.to(cuda), W.to(cuda), b.to(cuda), act, hw.to(cuda), 0.2,
                            None if extra is None else extra.to(cuda), sig)
        ref = ops.linear_head(x, W, b, act, hw, 0.2, extra, sig)
        _close(y, ref, 1e-4, 1e-3, f"linear_head {M}x{N}x{K} {act}")


def test_linear_head_into_pinned_host(cuda):
    M, N, K = 2048, 256, 512
    x = torch.randn(M, K).to(torch.bfloat16)
    W = (torch.randn(N, K) / K ** 0.5).to(torch.bfloat16)
    b, hw = torch.randn(N) * 0.1, torch.randn(N) * 0.05
    out = torch.zeros(M, dtype=torch.float32).pin_memory()
    ops.linear_head(x.to(cuda), W.to(cuda), b.to(cuda), "relu", hw.to(cuda), 0.0, None, True, out=out)
    torch.cuda.synchronize()
    _close(out, ops.linear_head(x, W, b, "relu", hw, 0.0, None, True), 1e-4, 1e-3, "linear_head pinned")


def _mlp_tail_ref(x, W2, b2, act2, W3, b3, act3, hw, hb, extra, sig):
    """fp32 reference of the fused tail: h2 rounded to bf16 like the kernel (the unfused path's rounding)."""
    h2 = x.float() @ W2.float().t() + b2
    if act2 == "relu":
        h2 = torch.relu(h2)
    return ops.linear_head(h2.to(torch.bfloat16), W3, b3, act3, hw, hb, extra, sig)


@pytest.mark.parametrize("M", [8192, 8200, 16384, 16421])
@pytest.mark.parametrize("act3", ["relu", "none"])
def test_mlp_tail_fused(cuda, M, act3):
    g = torch.Generator().manual_seed(M + (act3 == "relu"))
    x = torch.randn(M, 1024, generator=g).to(torch.bfloat16)
    W2 = (torch.randn(512, 1024, generator=g) / 32).to(torch.bfloat16)
    W3 = (torch.randn(256, 512, generator=g) / 512 ** 0.5).to(torch.bfloat16)
    b2, b3 = torch.randn(512, generator=g) * 0.1, torch.randn(256, generator=g) * 0.1
    hw = torch.randn(256, generator=g) * 0.05
    parts = torch.randn(2, M + 100, generator=g)  # the gather-GEMM's [2, Mp] partial logits
    W2p, W3p = ops.pack_bfrag(W2.to(cuda)), ops.pack_bfrag(W3.to(cuda))
    for extra, sig in ((parts, True), (None, False)):
        y = ops.mlp_tail(x.to(cuda), W2p, b2.to(cuda), "relu", W3p, b3.to(cuda), act3, hw.to(cuda), 0.2,
                         None if extra is None else extra.to(cuda), sig)
        ref = _mlp_tail_ref(x, W2, b2, "relu", W3, b3, act3, hw, 0.2, extra, sig)
        # h2 is bf16: a ReLU/rounding boundary flip moves a logit by ~1e-3
        _close(y, ref, 2e-3, 2e-3, f"mlp_tail {M} {act3}")


def test_mlp_tail_into_pinned_host_and_model_path(cuda):
    M = 16384
    cfg = ModelConfig(family="deepfm", vocab_size=20000)
    m = build_model(cfg, cuda)
    l2, l3 = m.mlp.layers[1], m.mlp.layers[2]
    x = (torch.randn(M, 1024) * 0.5).to(torch.bfloat16).to(cuda)
    extra = torch.randn(2, M).to(cuda)
    out = torch.zeros(M, dtype=torch.float32).pin_memory()

    def two_kernels():  # GEMM2 + the fused last layer / head: what the tail replaces
        return ops.linear_head(l2(x), l3.weight, l3.bias, l3.act, m.head_w, 0.1, extra=extra)

    y = m.mlp.forward_head(x, m.head_w, 0.1, extra=extra, out=out, start=1)
    torch.cuda.synchronize()
    assert y.data_ptr() == out.data_ptr()
    _close(out, two_kernels(), 2e-3, 2e-3, "mlp_tail model path vs GEMM2 + fused head")
    # a weight update re-packs (load_state_dict bumps the version)
    with torch.no_grad():
        l2.weight.mul_(0.5)
    y2 = m.mlp.forward_head(x, m.head_w, 0.1, extra=extra, start=1)
    _close(y2, two_kernels(), 2e-3, 2e-3, "mlp_tail after a weight update")


@pytest.mark.parametrize("n", [1, 7, 1500, 4096, 8192])
@pytest.mark.parametrize("desc", [False, True])
def test_sort(cuda, n, desc):
    s = torch.rand(n)
    s[: n // 3] = s[n // 3: 2 * (n // 3)]  # ties
    v, p = ops.sort_scores(s.to(cuda), descending=desc)
    vr, pr = torch.sort(s, descending=desc, stable=True)
    assert torch.equal(v.cpu(), vr)
    assert torch.equal(s[p.cpu()], vr)
    v, p = ops.sort_scores(s.to(cuda), descending=True, k=min(10, n))
    assert torch.equal(v.cpu(), torch.sort(s, descending=True).values[: min(10, n)])


@pytest.mark.parametrize("family", ["wdl", "deepfm", "dcn", "dcn_v2", "dlrm"])
def test_models_gpu_vs_cpu(cuda, family):
    cfg = ModelConfig(family=family, vocab_size=20000, table_rows=1000, embed_dim=64 if family == "dlrm" else 32,
                      mlp_dims=(256, 128), bottom_mlp=(64, 64), num_cross_layers=2)
    m = build_model(cfg, "cpu")
    mg = copy.deepcopy(m).to(cuda)
    ids = torch.randint(0, 10**9, (300, 43))
    wts = torch.rand(300, 43)
    y = mg(ids.to(cuda), wts.to(cuda))
    yr = m(ids, wts)
    _close(y, yr, 2e-2, 5e-3, family)


def test_dcn_v2_fp8_close_to_bf16(cuda):
    base = ModelConfig(family="dcn_v2", vocab_size=20000, embed_dim=32, mlp_dims=(256, 128), num_cross_layers=2)
    m16 = build_model(base, "cpu").to(cuda)
    f8 = copy.deepcopy(base)
    f8.gemm_dtype = "fp8"
    m8 = build_model(f8, "cpu").to(cuda)
    ids = torch.randint(0, 10**9, (256, 43), device=cuda)
    wts = torch.rand(256, 43, device=cuda)
    a, b = m16(ids, wts), m8(ids, wts)
    assert (a - b).abs().max().item() < 0.05


def test_unpack_arena_gpu_matches_cpu(cuda):
    from distributed_tf_serving_amd.client.synth import SyntheticRequests
    from distributed_tf_serving_amd.serving.arena import ArenaLayout
    from distributed_tf_serving_amd.serving.packing import PackedLayout

    A, L = ArenaLayout(43, 2048), PackedLayout(43)
    ar = A.alloc()
    s = SyntheticRequests(dist="zipf", id_space=1 << 50, seed=5)
    reqs = [s.message(n, raw=r).SerializeToString() for n, r in ((1, True), (300, True), (17, False), (512, True))]
    ab = A.build(ar, A.place(ar, reqs))
    assert ab.total_rows == 830 and not any(ab.errors) and ab.n_gpu_varint == 1
    dev = ar.to(cuda)  # before the CPU reference fills the host copy's decoded-id region
    ref = A.unpack_cpu(ar, L.alloc(1024))
    got = L.alloc(1024, device=cuda)
    got.fill_(-1)
    A.decode_varints(dev)  # packed varint ids of the 17-row request, on the GPU
    ops.hip().unpack_arena(dev, got, 43)
    assert torch.equal(got.cpu(), ref)  # rows past total_rows are zeroed too


def test_unpack_arena_narrow_matches_cpu(cuda):
    """Narrow fan-out rows: [int32 id mod m | fp32 weight] from raw, varint
    and host-narrowed arena rows vs the wide CPU unpack + narrowing."""
    from distributed_tf_serving_amd.client.synth import SyntheticRequests
    from distributed_tf_serving_amd.serving.arena import ArenaLayout
    from distributed_tf_serving_amd.serving.packing import PackedLayout

    m = 999_983
    A, W, N = ArenaLayout(43, 2048), PackedLayout(43), PackedLayout(43, m)
    assert N.row_bytes == 344 and W.row_bytes == 520
    ar = A.alloc()
    s = SyntheticRequests(dist="zipf", id_space=1 << 50, seed=6)
    reqs = [s.message(n, raw=r).SerializeToString() for n, r in ((3, True), (250, False), (64, True))]
    ab = A.build(ar, A.place(ar, reqs))
    assert not any(ab.errors)
    dev = ar.to(cuda)
    wide = A.unpack_cpu(ar, W.alloc(512))
    ref = N.pack(W.ids(wide), W.wts(wide))
    got = N.alloc(512, device=cuda)
    got.fill_(-1)
    A.decode_varints(dev)
    ops.hip().unpack_arena(dev, got, 43, m)
    torch.cuda.synchronize()
    assert torch.equal(got.cpu(), ref)


@pytest.mark.parametrize("family", ["deepfm", "wdl", "dcn", "dcn_v2", "dlrm"])
def test_forward_arena_matches_packed(cuda, family):
    # K0 fused into K1: the gather reads ids / weights from the raw request bytes
    # (DLRM: the fused bottom MLP reads the dense features, the fused
    # interaction the sparse ids)
    from distributed_tf_serving_amd.client.synth import SyntheticRequests
    from distributed_tf_serving_amd.serving.arena import ArenaLayout
    from distributed_tf_serving_amd.serving.packing import PackedLayout

    cfg = ModelConfig(family=family, vocab_size=20_000)
    if family == "dlrm":
        cfg.table_rows = 5000
    m = build_model(cfg, cuda)
    assert m.supports_arena
    A, L = ArenaLayout(43, 2048), PackedLayout(43)
    ar = A.alloc()
    s = SyntheticRequests(dist="zipf", id_space=1 << 50, seed=9)
    reqs = [s.message(n, raw=r).SerializeToString() for n, r in ((3, True), (250, True), (17, False), (200, True))]
    ab = A.build(ar, A.place(ar, reqs))
    dev = ar.to(cuda)
    A.decode_varints(dev)
    B = 512  # > total_rows: padding rows must score like zero-weight rows
    packed = A.unpack_cpu(ar, L.alloc(B))
    want = m(L.ids(packed).to(cuda), L.wts(packed).to(cuda)).cpu()
    got = m.forward_arena(dev, B).cpu()
    _close(got[:ab.total_rows], want[:ab.total_rows], 0, 1e-6, f"{family} arena vs packed")
    _close(got, want, 0, 1e-6, f"{family} arena padding rows")
    out = torch.zeros(B, dtype=torch.float32).pin_memory()
    m.forward_arena(dev, B, out=out)
    torch.cuda.synchronize()
    _close(out, want, 0, 1e-6, f"{family} arena into pinned host")


def test_arena_varint_gpu_decode(cuda):
    # packed varint ids (reference client encoding) decoded by the GPU kernel:
    # multi-chunk runs, varints straddling 4 KiB chunk and lane boundaries,
    # 10-byte negative ids, 1-byte small ids
    from distributed_tf_serving_amd.ops import native
    from distributed_tf_serving_amd.serving.arena import ArenaLayout
    from distributed_tf_serving_amd.serving.packing import PackedLayout

    F = 43
    g = torch.Generator().manual_seed(3)
    A, L = ArenaLayout(F, 4096), PackedLayout(F)
    ar = A.alloc()
    reqs, want = [], []
    for n, kind in ((700, "mixed"), (1, "small"), (900, "neg"), (333, "mixed")):
        if kind == "small":
            ids = torch.randint(1, 100, (n, F), generator=g)
        elif kind == "neg":
            ids = torch.randint(-(1 << 62), 1 << 62, (n, F), generator=g)
        else:
            ids = torch.randint(0, 1 << 40, (n, F), generator=g) >> torch.randint(0, 40, (n, F), generator=g)
        wts = torch.rand(n, F, generator=g)
        reqs.append(native().encode_predict_request("DCN", "serving_default", None,
                                                    [("feat_ids", ids), ("feat_wts", wts)], False))
        want.append((ids, wts))
    ab = A.build(ar, A.place(ar, reqs))
    assert not any(ab.errors) and ab.n_gpu_varint == 4 and ab.n_decoded == 0
    dev = ar.to(cuda)
    A.decode_varints(dev)
    B = ab.total_rows
    got = L.alloc(B, device=cuda)
    ops.hip().unpack_arena(dev, got, F)
    got = got.cpu()
    ids_all = torch.cat([w[0] for w in want])
    wts_all = torch.cat([w[1] for w in want])
    assert torch.equal(L.ids(got), ids_all)
    assert torch.equal(L.wts(got), wts_all)
    assert torch.equal(A.unpack_cpu(ar, L.alloc(B)), got)


def test_deepfm_full_mlp_gpu_vs_cpu(cuda):
    # the serving MLP 2752 -> 1024 -> 512 -> 256: 8-phase GEMM, narrow GEMM, fused last layer + head
    cfg = ModelConfig(family="deepfm", vocab_size=20000)
    m = build_model(cfg, "cpu")
    mg = copy.deepcopy(m).to(cuda)
    ids = torch.randint(0, 10**9, (300, 43))
    wts = torch.rand(300, 43)
    _close(mg(ids.to(cuda), wts.to(cuda)), m(ids, wts), 2e-2, 5e-3, "deepfm full MLP")


@pytest.mark.parametrize("waves", [4, 8, 64])
def test_embed_pipelined_rows_per_wave(cuda, waves):
    # the pipelined gather with many rows per wave (next row's ids prefetched),
    # extreme ids for the multiply-high modulo, and the arena-fed variant
    from distributed_tf_serving_amd.client.synth import SyntheticRequests
    from distributed_tf_serving_amd.serving.arena import ArenaLayout
    from distributed_tf_serving_amd.serving.packing import PackedLayout

    V, D, F, B = 99991, 64, 43, 1000
    g = torch.Generator().manual_seed(waves)
    table = (torch.rand(V, D, generator=g) - 0.5).to(torch.bfloat16)
    lin = torch.rand(V, generator=g) - 0.5
    ids = torch.randint(-(1 << 62), 1 << 62, (B, F), generator=g)
    ids[0, :4] = torch.tensor([-(1 << 63), (1 << 63) - 1, -1, 0])
    wts = torch.rand(B, F, generator=g)
    h = ops.hip()
    try:
        h.set_embed_wave_cap(waves)
        x, fm = ops.embed(table.to(cuda), ids.to(cuda), wts.to(cuda), lin=lin.to(cuda), modulo=V, bias=0.1,
                          want_x=True, want_fm=True, fm2=True)
        xr, fmr = ops.embed(table, ids, wts, lin=lin, modulo=V, bias=0.1, want_x=True, want_fm=True, fm2=True)
        _close(x, xr, 1e-2, 1e-3, "pipelined x")
        _close(fm, fmr, 2e-3, 2e-3 * F, "pipelined fm")
        A, L = ArenaLayout(F, 2048), PackedLayout(F)
        ar = A.alloc()
        s = SyntheticRequests(dist="zipf", id_space=1 << 50, seed=waves)
        reqs = [s.message(n, raw=r).SerializeToString() for n, r in ((3, True), (250, True), (17, False), (200, True))]
        ab = A.build(ar, A.place(ar, reqs))
        dev = ar.to(cuda)
        A.decode_varints(dev)
        packed = A.unpack_cpu(ar, L.alloc(512))
        want = ops.embed(table.to(cuda), L.ids(packed).to(cuda), L.wts(packed).to(cuda), lin=lin.to(cuda), modulo=V,
                         want_x=True, want_fm=True, fm2=True)
        got = ops.embed(table.to(cuda), ops.ArenaRows(dev, 512, F), None, lin=lin.to(cuda), modulo=V,
                        want_x=True, want_fm=True, fm2=True)
        assert ab.total_rows == 470
        _close(got[0], want[0], 0, 0, "arena x")
        _close(got[1], want[1], 0, 1e-6, "arena fm")
    finally:
        h.set_embed_wave_cap(4096)


@pytest.mark.parametrize("D,F,L", [(64, 43, 3), (16, 43, 1), (64, 10, 7), (32, 64, 2)])
def test_embed_cross_matches_layerwise_reference(cuda, D, F, L):
    """K3 in K1: the gather computes DCN v1's whole cross network from its L + 1
    dot products (alpha / c recurrence) - vs the layer-by-layer fp32 reference."""
    g = torch.Generator().manual_seed(D + F + L)
    V, B = 3000, 300
    d = F * D
    table = (torch.rand(V, D, generator=g) - 0.5).to(torch.bfloat16)
    ids = torch.randint(0, 1 << 40, (B, F), generator=g)
    wts = torch.rand(B, F, generator=g) * 2
    w = (torch.rand(L, d, generator=g) - 0.5) / d ** 0.5
    b = (torch.rand(L, d, generator=g) - 0.5) * 0.1
    hw = (torch.rand(d, generator=g) - 0.5) / d ** 0.5
    x, logit = ops.embed_cross(table.to(cuda), ids.to(cuda), wts.to(cuda), V, w.to(cuda), b.to(cuda), hw.to(cuda))
    xr, lr = ops.embed_cross(table, ids, wts, V, w, b, hw)
    _close(x, xr, 0, 0, "x")
    _close(logit, lr, 1e-4, 1e-4, "cross logit")


def _gather_gemm_case(B, F=43, V=50_000, N=1024, seed=5, ids32=False):
    g = torch.Generator().manual_seed(seed)
    table = ((torch.rand(V, 64, generator=g) - 0.5) * 0.2).to(torch.bfloat16)
    lin = (torch.rand(V, generator=g) - 0.5) * 0.1
    W = ((torch.rand(N, F * 64, generator=g) - 0.5) * 0.05).to(torch.bfloat16)
    b = (torch.rand(N, generator=g) - 0.5) * 0.1
    ids = torch.randint(-(1 << 40), 1 << 40, (B, F), generator=g)
    if ids32:
        ids = ids.remainder(1 << 31).to(torch.int32)
    wts = torch.rand(B, F, generator=g)
    return table, lin, W, b, ids, wts


def _gather_gemm_ref(table, lin, W, b, ids, wts, V, bias, fm2):
    rows = torch.remainder(ids.long(), V)
    e = table[rows].float() * wts[..., None]  # [B, F, 64]
    h = torch.relu(e.reshape(ids.shape[0], -1) @ W.float().t() + b)
    fm = bias + (lin[rows] * wts).sum(1)
    if fm2:
        fm = fm + 0.5 * (e.sum(1).pow(2) - e.pow(2).sum(1)).sum(1)
    return h, fm


@pytest.mark.parametrize("B,ids32", [(1, False), (300, True), (4099, False), (16384, False)])
@pytest.mark.parametrize("fm2", [True, False])
def test_embed_gemm_matches_fp32_reference(cuda, B, ids32, fm2):
    """K1 fused into K4 (gather-GEMM + resolve kernel): the first layer's
    output and the FM partial logits vs the fp32 torch math, and vs the unfused
    GPU path (gather kernel writing x, then the GEMM), which rounds x the same
    way and runs the same MFMA sequence per output."""
    V, bias = 50_000, 0.25
    table, lin, W, b, ids, wts = _gather_gemm_case(B, V=V, ids32=ids32)
    d = [t.to(cuda) for t in (table, lin, W, b, ids, wts)]
    h, parts = ops.embed_gemm(d[0], d[4], d[5], d[1], V, bias, d[2], d[3], "relu", fm2=fm2)
    assert h.shape == (B, 1024) and parts.shape[0] == (2 if fm2 else 1) and parts.shape[1] >= B
    h_ref, fm_ref = _gather_gemm_ref(table, lin, W, b, ids, wts, V, bias, fm2)
    _close(h, h_ref, 2e-2, 2e-3, "gather-GEMM h vs fp32")
    _close(parts[:, :B].sum(0), fm_ref, 1e-4, 1e-4, "FM partials vs fp32")
    xg, fmg = ops.embed(d[0], d[4], d[5], lin=d[1], modulo=V, bias=bias, want_x=True, want_fm=True, fm2=fm2)
    _close(h, ops.linear(xg, d[2], d[3], "relu"), 1e-2, 1e-4, "gather-GEMM vs gather + GEMM")
    _close(parts[:, :B].sum(0), fmg, 1e-5, 1e-5, "FM partials vs the gather kernel's FM")


@pytest.mark.parametrize("B,F,N,fm2", [(1, 43, 1024, True), (300, 1, 512, False), (4099, 3, 1024, True),
                                       (16384, 43, 1024, True), (16384, 43, 1024, False), (2048, 26, 2048, True),
                                       (1000, 7, 1536, False)])
def test_gather_gemm_one_wave_form(cuda, B, F, N, fm2):
    """The one-wave-per-SIMD gather-GEMM (gather_gemm.hip: packed W straight
    into registers, 6-slot A ring, scale pass one tile ahead) vs the fp32
    reference and vs the 8-phase kernel, over field counts below / above its
    prefetch depths and 1-4 column tiles (FM rows owned by tiles 0-1)."""
    V, bias = 30_000, -0.5
    table, lin, W, b, ids, wts = _gather_gemm_case(B, F=F, V=V, N=N, seed=B + F)
    d = [t.to(cuda) for t in (table, lin, W, b, ids, wts)]
    Wp = ops.pack_frag32(d[2])
    h, parts = ops.embed_gemm(d[0], d[4], d[5], d[1], V, bias, d[2], d[3], "relu", fm2=fm2, packed_w=lambda: Wp)
    h_ref, fm_ref = _gather_gemm_ref(table, lin, W, b, ids, wts, V, bias, fm2)
    _close(h, h_ref, 2e-2, 2e-3, "one-wave gather-GEMM h vs fp32")
    _close(parts[:, :B].sum(0), fm_ref, 1e-4, 1e-4, "one-wave FM partials vs fp32")
    h8, p8 = ops.embed_gemm(d[0], d[4], d[5], d[1], V, bias, d[2], d[3], "relu", fm2=fm2)
    _close(h, h8, 1e-2, 1e-4, "one-wave vs 8-phase gather-GEMM")
    _close(parts[:, :B].sum(0), p8[:, :B].sum(0), 1e-5, 1e-5, "one-wave vs 8-phase FM partials")


class _Layer:
    """The attributes ops.gather_mlp reads off a models.layers.Dense."""

    def __init__(self, W, b, act):
        self.weight, self.bias, self.act, self.fp8 = W, b, act, False
        self.in_dim = self.k = W.shape[1]

    def packed(self, layout):
        assert layout == "32"
        return ops.pack_frag32(self.weight)


@pytest.mark.parametrize("B,F,fm,act3", [(8192, 43, True, "relu"), (16421, 43, True, "none"),
                                          (16384, 43, False, "relu"), (9000, 7, True, "relu"),
                                          (8192, 1, False, "none"), (8300, 64, True, "relu")])
def test_gather_mlp_tower_vs_fp32(cuda, B, F, fm, act3):
    """The whole DeepFM / Wide&Deep tower in one launch (gather_mlp.hip: 64 rows
    x all 1024 h1 columns per workgroup, h1 / h2 in LDS) vs the fp32 torch math
    (h1 and h2 rounded to bf16 like every GPU path), over field counts below /
    above the rings' depths and row counts that are not a multiple of 64; and
    vs the two-kernel form it replaces (one-wave gather-GEMM + MLP tail)."""
    V, bias = 30_000, -0.25
    table, lin, W1, b1, ids, wts = _gather_gemm_case(B, F=F, V=V, N=1024, seed=B + F)
    g = torch.Generator().manual_seed(B * 7 + F)
    W2 = (torch.randn(512, 1024, generator=g) / 32).to(torch.bfloat16)
    W3 = (torch.randn(256, 512, generator=g) / 512 ** 0.5).to(torch.bfloat16)
    b2, b3 = torch.randn(512, generator=g) * 0.1, torch.randn(256, generator=g) * 0.1
    hw = torch.randn(256, generator=g) * 0.05
    d = [t.to(cuda) for t in (table, lin, W1, b1, ids, wts, W2, b2, W3, b3, hw)]
    layers = [_Layer(d[2], d[3], "relu"), _Layer(d[6], d[7], "relu"), _Layer(d[8], d[9], act3)]
    assert ops.gather_mlp_ok(d[0], layers, B)
    y = ops.gather_mlp(d[0], d[4], d[5], d[1], V, bias, layers, d[10], 0.2, fm=fm)
    h1, first = _gather_gemm_ref(table, lin, W1, b1, ids, wts, V, bias, fm)
    ref = _mlp_tail_ref(h1.to(torch.bfloat16), W2, b2, "relu", W3, b3, act3, hw, 0.2, first, True)
    # h1 / h2 are bf16: a ReLU / rounding boundary flip moves a logit by ~1e-3
    _close(y, ref, 2e-3, 2e-3, f"gather_mlp {B} x {F} fm={fm} vs fp32")
    h, parts = ops.embed_gemm(d[0], d[4], d[5], d[1], V, bias, d[2], d[3], "relu", fm2=fm,
                              packed_w=lambda: ops.pack_frag32(d[2]))
    y2 = ops.mlp_tail(h, ops.pack_bfrag(d[6]), d[7], "relu", ops.pack_bfrag(d[8]), d[9], act3, d[10], 0.2, parts, True)
    _close(y, y2, 2e-3, 2e-3, "gather_mlp vs gather-GEMM + MLP tail")
    # scores into pinned host memory; int32 row ids (the fan-out's exchanged rows)
    out = torch.zeros(B, dtype=torch.float32).pin_memory()
    y3 = ops.gather_mlp(d[0], d[4], d[5], d[1], V, bias, layers, d[10], 0.2, fm=fm, out=out)
    torch.cuda.synchronize()
    assert y3.data_ptr() == out.data_ptr()
    _close(out, y, 0, 0, "pinned out vs device out")
    y4 = ops.gather_mlp(d[0], torch.remainder(d[4], V).to(torch.int32), d[5], d[1], V, bias, layers, d[10], 0.2, fm=fm)
    _close(y4, y, 0, 0, "int32 rows vs int64 ids")


def test_gather_mlp_arena_rows(cuda):
    """The one-launch tower resolving its rows straight from request bytes in
    a device arena (raw and packed-varint requests, padding rows past the
    arena's rows) scores like the same rows unpacked."""
    from distributed_tf_serving_amd.client.synth import SyntheticRequests
    from distributed_tf_serving_amd.serving.arena import ArenaLayout
    from distributed_tf_serving_amd.serving.packing import PackedLayout

    V = 30_000
    table, lin, W1, b1, _, _ = _gather_gemm_case(1, V=V)
    m = build_model(ModelConfig(family="deepfm", vocab_size=V), cuda)
    with torch.no_grad():
        m.emb.copy_(table.to(cuda))
        m.lin.copy_(lin.to(cuda))
    A, L = ArenaLayout(43, 16384), PackedLayout(43)
    ar = A.alloc()
    s = SyntheticRequests(dist="zipf", id_space=1 << 50, seed=13)
    sizes = [(3, True), (1500, False), (700, True), (90, False)] * 3 + [(4000, True), (5000, False)]
    reqs = [s.message(n, raw=r).SerializeToString() for n, r in sizes]
    ab = A.build(ar, A.place(ar, reqs))
    assert not any(ab.errors)
    dev = ar.to(cuda)
    A.decode_varints(dev)
    B = 16384  # > total_rows (15879): padding rows; the served bucket the tower runs at
    packed = A.unpack_cpu(ar, L.alloc(B))
    ids, wts = L.ids(packed), L.wts(packed)
    ya = m.forward_arena(dev, B)
    assert m._gather_mlp(ids.to(cuda), wts.to(cuda), fm2=True)
    yp = m(ids.to(cuda), wts.to(cuda))
    _close(ya, yp, 0, 0, "arena vs unpacked rows")


def test_gather_mlp_model_path_and_weight_update(cuda):
    """DeepFM / Wide&Deep at a GPU-filling batch take the one-launch tower; the
    scores equal the two-kernel form's, and an in-place weight update reaches
    the packed copy the kernel (and any captured graph) reads."""
    for family in ("deepfm", "wdl"):
        m = build_model(ModelConfig(family=family, vocab_size=20000), cuda)
        ids = torch.randint(0, 1 << 40, (16384, 43)).to(cuda)
        wts = torch.rand(16384, 43).to(cuda)
        assert m._gather_mlp(ids, wts, fm2=family == "deepfm")
        y = m(ids, wts)
        try:
            type(m).use_gather_mlp = False
            want = m(ids, wts)
        finally:
            type(m).use_gather_mlp = True
        _close(y, want, 2e-3, 2e-3, f"{family}: gather_mlp vs two kernels")
        l2 = m.mlp.layers[1]
        packed = l2.packed("32")
        with torch.no_grad():
            l2.weight.mul_(0.5)
        y2 = m(ids, wts)
        assert l2.packed("32").data_ptr() == packed.data_ptr()  # re-packed in place
        try:
            type(m).use_gather_mlp = False
            want2 = m(ids, wts)
        finally:
            type(m).use_gather_mlp = True
        _close(y2, want2, 2e-3, 2e-3, f"{family}: after a weight update")


def test_embed_gemm_narrow_exchange_rows(cuda):
    """The candidate fan-out hands the forward its exchanged rows as strided
    views of [int32 row x F | fp32 weight x F] (serving/packing.py narrow
    layout): the gather-GEMM reads them in place, same result as contiguous
    copies. (Rejected as non-contiguous until round 5: the 16384-row fan-out
    step could not be built.)"""
    from distributed_tf_serving_amd.serving.packing import PackedLayout

    V, B = 40_000, 16384
    table, lin, W, b, ids, wts = _gather_gemm_case(B, V=V)
    L = PackedLayout(43, narrow_modulo=V)
    buf = L.pack(ids, wts).to(cuda)
    iv, wv = L.ids(buf), L.wts(buf)
    assert not iv.is_contiguous() and iv.stride(1) == 1
    d = [t.to(cuda) for t in (table, lin, W, b)]
    h, parts = ops.embed_gemm(d[0], iv, wv, d[1], V, 0.1, d[2], d[3], "relu")
    hc, pc = ops.embed_gemm(d[0], iv.contiguous(), wv.contiguous(), d[1], V, 0.1, d[2], d[3], "relu")
    _close(h, hc, 0, 0, "strided vs contiguous rows")
    _close(parts[:, :B], pc[:, :B], 0, 0, "strided vs contiguous FM partials")


def test_embed_gemm_arena_rows(cuda):
    """The gather-GEMM reading raw and packed-varint request bytes from a
    device arena scores like the same rows unpacked (padding rows: zeros)."""
    from distributed_tf_serving_amd.client.synth import SyntheticRequests
    from distributed_tf_serving_amd.serving.arena import ArenaLayout
    from distributed_tf_serving_amd.serving.packing import PackedLayout

    V = 30_000
    table, lin, W, b, _, _ = _gather_gemm_case(1, V=V)
    d = [t.to(cuda) for t in (table, lin, W, b)]
    A, L = ArenaLayout(43, 4096), PackedLayout(43)
    ar = A.alloc()
    s = SyntheticRequests(dist="zipf", id_space=1 << 50, seed=12)
    reqs = [s.message(n, raw=r).SerializeToString() for n, r in ((3, True), (1500, False), (700, True), (90, False))]
    ab = A.build(ar, A.place(ar, reqs))
    assert not any(ab.errors)
    dev = ar.to(cuda)
    A.decode_varints(dev)
    B = 2600  # > total_rows (2293): padding rows
    packed = A.unpack_cpu(ar, L.alloc(B))
    ids, wts = L.ids(packed), L.wts(packed)
    h, parts = ops.embed_gemm(d[0], ops.ArenaRows(dev, B, 43), None, d[1], V, 0.0, d[2], d[3], "relu")
    h_ref, fm_ref = _gather_gemm_ref(table, lin, W, b, ids, wts, V, 0.0, True)
    _close(h, h_ref, 2e-2, 2e-3, "arena gather-GEMM h vs fp32")
    _close(parts[:, :B].sum(0), fm_ref, 1e-4, 1e-4, "arena FM partials vs fp32")
    hp, pp = ops.embed_gemm(d[0], ids.to(cuda), wts.to(cuda), d[1], V, 0.0, d[2], d[3], "relu")
    _close(h, hp, 0, 0, "arena vs unpacked rows")
    _close(parts[:, :B], pp[:, :B], 0, 0, "arena vs unpacked FM partials")


@pytest.mark.parametrize("B,L", [(1, 3), (4099, 3), (16384, 3), (300, 2), (300, 1)])
def test_embed_gemm_cross_matches_layerwise_reference(cuda, B, L):
    """The gather-GEMM with the DCN v1 cross network on the scale pass: the
    cross logit vs the fp32 layer-by-layer math; h as without it."""
    V, F, d = 50_000, 43, 43 * 64
    table, lin, W, b, ids, wts = _gather_gemm_case(B, V=V)
    g = torch.Generator().manual_seed(9)
    cw = (torch.rand(max(L, 1), d, generator=g) - 0.5) * 0.02
    cb = (torch.rand(max(L, 1), d, generator=g) - 0.5) * 0.02
    hw = (torch.rand(d, generator=g) - 0.5) * 0.05
    cw, cb = cw[:L], cb[:L]
    dv = [t.to(cuda) for t in (table, W, b, ids, wts, cw, cb, hw)]
    h, parts = ops.embed_gemm(dv[0], dv[3], dv[4], None, V, 0.0, dv[1], dv[2], "relu", fm2=False,
                              cross=(dv[5], dv[6], dv[7]))
    assert parts.shape[0] == 2
    rows = torch.remainder(ids, V)
    x0 = (table[rows].float() * wts[..., None]).reshape(B, -1)
    xl = x0
    for i in range(L):
        xl = x0 * (xl @ cw[i])[:, None] + cb[i] + xl
    want = xl @ hw
    h_ref = torch.relu(x0 @ W.float().t() + b)
    _close(h, h_ref, 2e-2, 2e-3, "cross gather-GEMM h vs fp32")
    _close(parts[0, :B], torch.zeros(B), 0, 0, "part0 (no first-order term)")
    _close(parts[1, :B], want, 1e-3, 1e-4, "cross logit vs layer-by-layer fp32")


@pytest.mark.parametrize("family", ["deepfm", "wdl", "dcn"])
def test_gather_gemm_model_path_matches_unfused(cuda, family):
    """DeepFM / WDL at a served bucket size take the gather-GEMM path; scores
    match the unfused path (gather kernel + GEMM) of the same weights."""
    cfg = ModelConfig(family=family, vocab_size=100_000)
    m = build_model(cfg, cuda)
    B = max(8192, ops.GATHER_GEMM_MIN_ROWS)
    ids = torch.randint(0, 1 << 40, (B, 43), device=cuda)
    wts = torch.rand(B, 43, device=cuda)
    assert m._gather_gemm(ids, wts, fm2=family != "wdl")
    got = m(ids, wts)
    m.use_gather_gemm = False
    want = m(ids, wts)
    _close(got, want, 0, 5e-5, f"{family} gather-GEMM vs unfused")


@pytest.mark.parametrize("M,n,K,ld", [(1, 13, 64, 13), (300, 13, 64, 43), (4099, 64, 64, 70)])
def test_dense_pad(cuda, M, n, K, ld):
    x = torch.randn(M, ld + 5, device=cuda)[:, :ld]  # a row view, like packed request rows
    y = ops.hip().dense_pad(x, n, K)
    want = torch.zeros(M, K, dtype=torch.bfloat16)
    want[:, :n] = x[:, :n].cpu().to(torch.bfloat16)
    assert torch.equal(y.cpu(), want)


@pytest.mark.parametrize("hot", [1, 3])
def test_shard_route_arena_and_multi_hot(cuda, hot):
    """K1b routing on the GPU: from ids + weights and straight from a device
    request arena (raw and packed-varint requests), one-hot and multi-hot,
    vs the CPU reference; the bag kernel writes into a static out buffer."""
    from distributed_tf_serving_amd.client.synth import SyntheticRequests
    from distributed_tf_serving_amd.serving.arena import ArenaLayout
    from distributed_tf_serving_amd.serving.packing import PackedLayout

    F, W, tm = 4 + 6 * hot, 3, 2
    A, L = ArenaLayout(F, 256), PackedLayout(F)
    ar = A.alloc()
    s = SyntheticRequests(fields=F, dist="zipf", id_space=1 << 40, seed=8)
    reqs = [s.message(n, raw=r).SerializeToString() for n, r in ((30, True), (70, False), (1, True))]
    assert not any(A.build(ar, A.place(ar, reqs)).errors)
    B = 120  # > 101 rows: padding rows route id 0
    packed = A.unpack_cpu(ar, L.alloc(B))
    ids, wts = L.ids(packed), L.wts(packed)
    col = torch.tensor([4 + hot * t for t in range(W * tm)], dtype=torch.int32)
    mod = torch.tensor([997, 1000, 13, 50_000, 7, 101], dtype=torch.int64)
    off = torch.tensor([0, 997, 0, 13, 0, 7], dtype=torch.int64)
    want_w = torch.empty(W, B, tm * hot)
    want = ops.shard_route(ids, W, tm, col, mod, off, hot=hot, wts=wts, out_w=want_w)
    dev = ar.to(cuda)
    A.decode_varints(dev)
    d = [t.to(cuda) for t in (col, mod, off)]
    got_w = torch.empty(W, B, tm * hot, device=cuda)
    got = ops.shard_route(ops.ArenaRows(dev, B, F), W, tm, *d, hot=hot, out_w=got_w)
    assert torch.equal(got.cpu(), want) and torch.equal(got_w.cpu(), want_w)
    got2 = ops.shard_route(ids.to(cuda), W, tm, *d, hot=hot, wts=wts.to(cuda))
    assert torch.equal(got2.cpu(), want)
    if hot > 1:  # the owner's pooled bags into a static buffer
        table = torch.randn(50_000, 64, device=cuda).to(torch.bfloat16)
        offs = torch.arange(0, W * B * tm * hot + 1, hot, dtype=torch.int64, device=cuda)
        out = torch.empty(W * B * tm, 64, dtype=torch.bfloat16, device=cuda)
        r = ops.embedding_bag(table, got.view(-1), offs, per_sample_weights=got_w.view(-1), out_bf16=True, out=out)
        assert r.data_ptr() == out.data_ptr()
        ref = ops.embedding_bag(table.cpu(), got.cpu().view(-1), offs.cpu(), per_sample_weights=got_w.cpu().view(-1))
        _close(out.float(), ref, 2e-2, 1e-2, "bag into a static buffer")
