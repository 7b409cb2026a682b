"""Run one GEMM shape/variant N times (for rocprofv3 counter collection)."""
import sys

import torch

from .. import ops


def main():
    M, N, K, v = (int(x) for x in sys.argv[1:5])
    iters = int(sys.argv[5]) if len(sys.argv) > 5 else 20
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    W = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device="cuda")
    h = ops.hip()
    for _ in range(iters):
        h.gemm(x, W, b, 1, None, None, False, None, None, None, v)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
