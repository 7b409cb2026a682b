"""OCP MX-fp8 reference path (CPU): block quantisation round trip, the GEMM's
block-scaled input, and the DCN-v2 cross chain that hands MX-fp8 operands from
one layer's epilogue to the next (GPU kernels: tests/test_kernels_gpu.py)."""
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
