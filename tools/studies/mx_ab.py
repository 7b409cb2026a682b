"""A/B of the DCN-v2 cross GEMM (16384 x 2752 x 2816, fp8) operand forms:
per-row scaled e4m3 A vs OCP MX-fp8 A (E8M0 block scales into the MFMA),
with and without the MX-fp8 epilogue output. Prints one JSON line per form.

    python -m tools.studies.mx_ab
"""
import json

import torch

from distributed_tf_serving_amd import ops


def _time(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    import sys
    M, N = (int(sys.argv[1]) if len(sys.argv) > 1 else 16384), 2752
    K = 2816
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(0)
    x0 = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
    xl = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
    W = (torch.randn(N, N, device=dev, generator=g) / N ** 0.5).to(torch.bfloat16)
    b = torch.zeros(N, device=dev)
    wq, sw = ops.quant_rows_fp8(W, ops.FP8_K_PAD)
    qr, sr = ops.quant_rows_fp8(xl, ops.FP8_K_PAD)
    qm, sm = ops.quant_mx_fp8(xl, K)
    s127 = torch.full_like(sm, 127)
    ones = torch.ones_like(sr)
    h = ops.hip()
    flops = 2.0 * M * N * K
    forms = {
        "row_scaled": lambda: h.gemm(qr, wq, b, 3, x0, xl, False, sr, sw, None, 0),
        "row_scaled_variant14": lambda: h.gemm(qr, wq, b, 3, x0, xl, False, sr, sw, None, 14),
        "row_q_with_unit_block_scales": lambda: h.gemm(qr, wq, b, 3, x0, xl, False, sr, sw, None, 0, s127),
        "mx_q_unit_scales(wrong values, same data)": lambda: h.gemm(qm, wq, b, 3, x0, xl, False, ones, sw, None, 0),
        "mx_q_block_scales": lambda: h.gemm(qm, wq, b, 3, x0, xl, False, None, sw, None, 0, sm),
    }
    q_out = torch.empty(M, K, dtype=torch.float8_e4m3fn, device=dev)
    sq_out = torch.empty(M, K // 32, dtype=torch.uint8, device=dev)
    forms["row_in_mx_out"] = lambda: h.gemm(qr, wq, b, 3, x0, xl, False, sr, sw, None, 0, None, q_out, sq_out)
    forms["mx_in_mx_out"] = lambda: h.gemm(qm, wq, b, 3, x0, xl, False, None, sw, None, 0, sm, q_out, sq_out)
    forms["quant_rows"] = lambda: ops.quant_rows_fp8(xl, ops.FP8_K_PAD)
    for v in (4, 10, 14, 17):
        forms[f"row_scaled_variant{v}"] = (lambda v=v: h.gemm(qr, wq, b, 3, x0, xl, False, sr, sw, None, v))
    for name, fn in forms.items():
        us = _time(fn)
        print(json.dumps({"form": name, "us": round(us, 2), "pflops": round(flops / us / 1e9, 3)}), flush=True)


if __name__ == "__main__":
    main()
