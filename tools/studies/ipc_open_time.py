"""How long does mapping a peer's allocation take (hipIpcGetMemHandle /
hipIpcOpenMemHandle, the peer exchange's start-up, parallel/hot_cache.py)?
torchrun N ranks; each exports a buffer of each size, every rank maps the
others' and reports the open time. Prints one JSON line per size (rank 0)."""
from __future__ import annotations

import argparse
import json
import time

import torch
import torch.distributed as dist


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", default="0.25,0.5,1,2")
    a = ap.parse_args()
    from distributed_tf_serving_amd.ops import hip
    from distributed_tf_serving_amd.parallel.dist import init_from_env

    ctx = init_from_env()
    dev = ctx.device
    for g in (float(x) for x in a.gib.split(",")):
        n = int(g * (1 << 30))
        buf = torch.empty(n, dtype=torch.uint8, device=dev)
        buf[:: 1 << 20].fill_(ctx.rank + 1)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        h, off = hip().ipc_export(buf)
        t_exp = time.perf_counter() - t0
        allv = [None] * ctx.world
        dist.all_gather_object(allv, (h, off, n))
        t0 = time.perf_counter()
        peers = [hip().ipc_open(hh, oo, [nn], buf) for r, (hh, oo, nn) in enumerate(allv) if r != ctx.rank]
        t_open = time.perf_counter() - t0
        ok = all(int(p[0]) != 0 for p in peers)
        t0 = time.perf_counter()
        s = sum(float(p[:: 1 << 20].float().sum()) for p in peers)
        torch.cuda.synchronize(dev)
        t_read = time.perf_counter() - t0
        res = [None] * ctx.world
        dist.all_gather_object(res, {"rank": ctx.rank, "export_s": round(t_exp, 4), "open_s": round(t_open, 3),
                                     "first_touch_s": round(t_read, 3), "ok": ok, "sum": s})
        if ctx.rank == 0:
            print(json.dumps({"gib": g, "ranks": res}), flush=True)
        del peers
        dist.barrier()
        del buf
        torch.cuda.empty_cache()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
