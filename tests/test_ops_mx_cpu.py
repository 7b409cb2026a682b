"""OCP MX-fp8 reference path (CPU): block quantisation round trip, the GEMM's
block-scaled input, and the DCN-v2 cross chain that hands MX-fp8 operands from
one layer's epilogue to the next (GPU kernels: tests/test_kernels_gpu.py)."""
import pytest
import torch

from distributed_tf_serving_amd import ops
from distributed_tf_serving_amd.config import ModelConfig
from distributed_tf_serving_amd.models import build_model


def test_quant_mx_round_trip_and_padding():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(7, 100, generator=g) * 5
    x[3, 32:64] = 0  # an all-zero block
    q, s = ops.quant_mx_fp8(x, 128)
    assert q.shape == (7, 128) and s.shape == (7, 4) and s.dtype == torch.uint8
    d = ops.dequant_mx_fp8(q, s)
    blk = torch.zeros(7, 128)
    blk[:, :100] = x
    amax = blk.abs().view(7, 4, 32).amax(2).repeat_interleave(32, dim=1)
    assert ((d - blk).abs() <= amax / 16 + 1e-6).all()
    assert (d[:, 100:] == 0).all() and s[3, 1] == 127 and (s[:, 3] >= 127 - 20).all()
    # no saturation: every block's max maps at or under the e4m3 max
    assert (q.float().abs() <= ops.FP8_MAX).all()
    assert ((blk.abs().view(7, 4, 32).amax(2) / torch.exp2(s.float() - 127)) <= ops.FP8_MAX).all()


def test_linear_fp8_block_scaled_input_equals_dequantised():
    g = torch.Generator().manual_seed(1)
    x = torch.randn(9, 256, generator=g)
    W = torch.randn(64, 256, generator=g) / 16
    q, s = ops.quant_mx_fp8(x, 128)
    wq, sw = ops.quant_rows_fp8(W, 128)
    y = ops.linear_fp8(q, None, wq, sw, None, out_f32=True, sx_blk=s)
    ref = ops.dequant_mx_fp8(q, s) @ (wq.float() * sw[:, None]).t()
    torch.testing.assert_close(y, ref)


def test_pack_bfrag_layout_and_round_trip():
    # fragment (n16, k64, kk), lane (fr, fq), value e = W[16 n16 + fr, 64 k64 + 32 kk + 8 fq + e]
    N, K = 48, 192
    W = torch.arange(N * K, dtype=torch.float32).view(N, K).to(torch.bfloat16)
    P = ops.pack_bfrag(W).view(N // 16, K // 64, 2, 64, 8)
    for n16, k64, kk, lane in ((0, 0, 0, 0), (2, 1, 1, 37), (1, 2, 0, 63), (2, 2, 1, 16)):
        fr, fq = lane & 15, lane >> 4
        want = W[16 * n16 + fr, 64 * k64 + 32 * kk + 8 * fq: 64 * k64 + 32 * kk + 8 * fq + 8]
        assert torch.equal(P[n16, k64, kk, lane], want)
    assert torch.equal(ops.unpack_bfrag(ops.pack_bfrag(W), N, K), W)
    with pytest.raises(ValueError):
        ops.pack_bfrag(W[:, :100])


def test_pack_frag32_layout():
    # fragment (n32, k64, s), lane (r, h), value e = W[32 n32 + r, 64 k64 + 16 s + 8 h + e]
    N, K = 96, 192
    W = torch.arange(N * K, dtype=torch.float32).view(N, K).to(torch.bfloat16)
    P = ops.pack_frag32(W).view(N // 32, K // 64, 4, 64, 8)
    for n32, k64, s, lane in ((0, 0, 0, 0), (2, 1, 3, 37), (1, 2, 1, 63), (2, 2, 2, 31), (0, 1, 0, 32)):
        r, h = lane & 31, lane >> 5
        want = W[32 * n32 + r, 64 * k64 + 16 * s + 8 * h: 64 * k64 + 16 * s + 8 * h + 8]
        assert torch.equal(P[n32, k64, s, lane], want)
    with pytest.raises(ValueError):
        ops.pack_frag32(W[:80])


def test_dense_packed_layouts_are_cached_per_layout():
    from distributed_tf_serving_amd.models.layers import Dense

    d = Dense(128, 64, "relu", torch.bfloat16, "cpu", torch.Generator().manual_seed(0))
    p16, p32 = d.packed("16"), d.packed("32")
    assert torch.equal(p16, ops.pack_bfrag(d.weight)) and torch.equal(p32, ops.pack_frag32(d.weight))
    assert d.packed("32") is p32
    with torch.no_grad():
        d.weight.add_(1.0)  # bumps the version: both layouts are re-packed IN PLACE
    assert torch.equal(d.packed("32"), ops.pack_frag32(d.weight)) and torch.equal(d.packed("16"), ops.pack_bfrag(d.weight))
    # same buffers: HIP graphs captured before the update read the new weights
    assert d.packed("16") is p16 and d.packed("32") is p32


def test_mlp_tail_only_on_gpu_shapes():
    from distributed_tf_serving_amd.config import ModelConfig
    from distributed_tf_serving_amd.models import build_model

    m = build_model(ModelConfig(family="deepfm", vocab_size=1000), "cpu")
    l2, l3 = m.mlp.layers[1], m.mlp.layers[2]
    x = torch.zeros(16384, 1024, dtype=torch.bfloat16)
    assert not ops.mlp_tail_ok(x, l2, l3)  # CPU tensors take the reference path
    # the packed copy follows the weight (re-packed after an in-place update)
    p1 = l2.packed()
    assert l2.packed() is p1
    with torch.no_grad():
        l2.weight.add_(1.0)
    p2 = l2.packed()
    assert p2 is p1 and torch.equal(ops.unpack_bfrag(p2, 512, 1024), l2.weight)  # re-packed in place
