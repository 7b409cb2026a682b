"""Is the DCN-v2 fp8 cross layer cheaper as GEMM + separate combine pass?

Times, at the served shape (M x 2752 x 2816, fp8 operands, interleaved rounds):
  fused   - the cross epilogue inside the GEMM (x0 * (xl W^T + b) + xl), variants 14 / 17
  plain   - the same GEMM with a plain bf16 epilogue (y = xl W^T + b), variants 14 / 17
  combine - x0 * y + xl as one torch elementwise pass (a stand-in for a fused
            combine + next-layer quantisation kernel), and quant_rows on its output

    python -m tools.studies.cross_split [M]
"""
import json
import statistics
import sys

import torch

from distributed_tf_serving_amd import ops


def _t(fn, iters=30):
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
    x0 = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
    xl = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
    W = (torch.randn(N, N, device=dev, generator=g) / N ** 0.5).to(torch.bfloat16)
    b = torch.zeros(N, device=dev)
    wq, sw = ops.quant_rows_fp8(W, ops.FP8_K_PAD)
    qr, sr = ops.quant_rows_fp8(xl, ops.FP8_K_PAD)
    h = ops.hip()
    y = h.gemm(qr, wq, b, 0, None, None, False, sr, sw, None, 14)
    forms = {}
    for v in (14, 17):
        forms[f"fused_v{v}"] = (lambda v=v: h.gemm(qr, wq, b, 3, x0, xl, False, sr, sw, None, v))
        forms[f"plain_v{v}"] = (lambda v=v: h.gemm(qr, wq, b, 0, None, None, False, sr, sw, None, v))
    forms["combine_torch"] = lambda: torch.addcmul(xl, x0, y)
    forms["quant_rows"] = lambda: ops.quant_rows_fp8(xl, ops.FP8_K_PAD)
    times = {k: [] for k in forms}
    for _ in range(3):
        for k, fn in forms.items():
            times[k].append(_t(fn))
    print(json.dumps({"M": M, "N": N, "K": 2816, **{k: round(statistics.median(v), 1) for k, v in times.items()}}))


if __name__ == "__main__":
    main()
