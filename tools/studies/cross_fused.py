"""DCN-v2 fp8 cross layer at the served shape (M x 2752 x 2816): one-launch
GEMM + LDS-staged cross epilogue (ops.cross_gemm_fp8) vs the split form
(plain 8-phase GEMM + cross_combine), interleaved rounds, CUDA-event timing.

    python -m tools.studies.cross_fused [M]

Prints one JSON line per form (median us over rounds): middle layer (z + e4m3
z for the next layer) and last layer (partial logits only).
"""
import json
import statistics
import sys

import torch

from distributed_tf_serving_amd import ops


def _t(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    N, dev = 2752, "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    x0 = (torch.randn(M, N, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    xl = (torch.randn(M, N, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    W = (torch.randn(N, N, device=dev, generator=g) / N ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=dev, generator=g) * 0.1
    hw = torch.randn(N, device=dev, generator=g) * 0.05
    wq, sw = ops.quant_rows_fp8(W, ops.FP8_K_PAD)
    q, sx = ops.quant_rows_fp8(xl, ops.FP8_K_PAD)

    forms = {
        "split_mid": lambda: ops.cross_combine(ops.linear_fp8(q, sx, wq, sw, b), x0, xl, True, ops.FP8_K_PAD),
        "fused_mid": lambda: ops.quant_rows_fp8(ops.cross_gemm_fp8(q, sx, wq, sw, b, x0, xl, True)[0],
                                                ops.FP8_K_PAD),
        "fused_mid_gemm_only": lambda: ops.cross_gemm_fp8(q, sx, wq, sw, b, x0, xl, True),
        "plain_gemm": lambda: ops.linear_fp8(q, sx, wq, sw, b),
        "split_last": lambda: ops.cross_combine(ops.linear_fp8(q, sx, wq, sw, b), x0, xl, False, 0, hw),
        "fused_last": lambda: ops.cross_gemm_fp8(q, sx, wq, sw, b, x0, xl, False, hw),
    }
    w2 = [ops.quant_rows_fp8((torch.randn(N, N, device=dev, generator=g) / N ** 0.5).to(torch.bfloat16),
                             ops.FP8_K_PAD) for _ in range(3)]

    def chain():
        """3 cross layers from x0 (row-scaled e4m3 x0, as the gather writes it)"""
        qq, ss = ops.quant_rows_fp8(x0, ops.FP8_K_PAD)
        xl_ = x0
        for i, (wq_, sw_) in enumerate(w2):
            last = i == 2
            z, d = ops.cross_gemm_fp8(qq, ss, wq_, sw_, b, x0, xl_, not last, hw if last else None)
            if not last:
                qq, ss = ops.quant_rows_fp8(z, ops.FP8_K_PAD)
            xl_ = z
        return d

    forms["chain_quant_rows"] = chain
    res = {k: [] for k in forms}
    for _ in range(5):
        for k, fn in forms.items():
            res[k].append(_t(fn))
    for k, v in res.items():
        print(json.dumps({"form": k, "M": M, "N": N, "K": q.shape[1], "us_median": round(statistics.median(v), 1),
                          "us_all": [round(x, 1) for x in v]}))


if __name__ == "__main__":
    main()
