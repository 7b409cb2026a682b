"""Fixed vs per-K-tile cost of a GEMM kernel: time M x N x K for several K at
one tile variant, bf16 and fp8 (row-scaled e4m3), and fit t(K) = F + nk * t_tile
(nk = K tiles of 128 bytes). Separates the prologue / epilogue / tail share
from the main-loop rate.

    python -m tools.studies.gemm_kscan [M N variant]
"""
import json
import sys

import numpy as np
import torch

from distributed_tf_serving_amd import ops


def _time(fn, iters=30):
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
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    v = int(sys.argv[3]) if len(sys.argv) > 3 else 17
    h = ops.hip()
    dev = "cuda"
    for dt in ("bf16", "fp8"):
        pts = []
        for nk in (11, 22, 44, 88):
            K = nk * (128 if dt == "fp8" else 64)
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            W = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
            b = torch.zeros(N, device=dev)
            if dt == "fp8":
                xq, sx = ops.quant_rows_fp8(x, ops.FP8_K_PAD)
                wq, sw = ops.quant_rows_fp8(W, ops.FP8_K_PAD)
                us = _time(lambda: h.gemm(xq, wq, b, 1, None, None, False, sx, sw, None, v))
            else:
                us = _time(lambda: h.gemm(x, W, b, 1, None, None, False, None, None, None, v))
            pts.append((nk, us))
            print(json.dumps({"dtype": dt, "M": M, "N": N, "K": K, "k_tiles": nk, "variant": v, "us": round(us, 2),
                              "pflops": round(2.0 * M * N * K / us / 1e9, 3)}), flush=True)
        a = np.array(pts)
        t_tile, F = np.polyfit(a[:, 0], a[:, 1], 1)
        print(json.dumps({"dtype": dt, "fit": {"fixed_us": round(float(F), 2), "us_per_k_tile": round(float(t_tile), 3)}}),
              flush=True)


if __name__ == "__main__":
    main()
