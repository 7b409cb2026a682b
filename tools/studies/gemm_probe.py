"""Run one GEMM shape/variant N times (for rocprofv3 counter collection).

    python -m tools.studies.gemm_probe M N K variant [iters] [bf16|fp8]
"""
import sys

import torch

from distributed_tf_serving_amd import ops


def main():
    M, N, K, v = (int(x) for x in sys.argv[1:5])
    iters = int(sys.argv[5]) if len(sys.argv) > 5 else 20
    dtype = sys.argv[6] if len(sys.argv) > 6 else "bf16"
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    W = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device="cuda")
    h = ops.hip()
    if dtype == "fp8":
        xq, sx = ops.quant_rows_fp8(x, ops.FP8_K_PAD)
        wq, sw = ops.quant_rows_fp8(W, ops.FP8_K_PAD)
        for _ in range(iters):
            h.gemm(xq, wq, b, 1, None, None, False, sx, sw, None, v)
    else:
        for _ in range(iters):
            h.gemm(x, W, b, 1, None, None, False, None, None, None, v)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
