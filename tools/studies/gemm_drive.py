"""Replays one GEMM form at a serving shape for counter collection
(rocprofv3 --pmc): the bf16 8-phase MLP GEMM, the same shape in fp8, and the
fp8 DCN-v2 cross layer (16384 x 2752 x 2816, x0 / xl epilogue).

    rocprofv3 --pmc ... -- python3 -m tools.studies.gemm_drive --form fp8 --variant 17
"""
from __future__ import annotations

import argparse

import torch

from distributed_tf_serving_amd import ops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--form", default="bf16", choices=["bf16", "fp8", "fp8cross"])
    ap.add_argument("--variant", type=int, default=17)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(0)
    h = ops.hip()
    if a.form == "fp8cross":
        M, N, K = 16384, 2752, 2816
    else:
        M, N, K = 16384, 1024, 2752 if a.form == "bf16" else 2816
    x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev, generator=g) / K ** 0.5).to(torch.bfloat16)
    b = torch.zeros(N, device=dev)
    if a.form == "bf16":
        fn = lambda: h.gemm(x, W, b, 1, None, None, False, None, None, None, a.variant)  # noqa: E731
    else:
        xq, sx = ops.quant_rows_fp8(x, ops.FP8_K_PAD)
        wq, sw = ops.quant_rows_fp8(W, ops.FP8_K_PAD)
        if a.form == "fp8":
            fn = lambda: h.gemm(xq, wq, b, 1, None, None, False, sx, sw, None, a.variant)  # noqa: E731
        else:
            x0 = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
            xl = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
            fn = lambda: h.gemm(xq, wq, b, 3, x0, xl, False, sx, sw, None, a.variant)  # noqa: E731
    for _ in range(a.iters):
        fn()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
