"""Kernel micro-benchmarks on one GPU (hot ops vs the library baseline).

    python -m tools.studies.microbench [--quick]

Prints one JSON line per measurement: the op, its shape, mean microseconds
over interleaved rounds (cdna_hip_programming.md §5.4 rule 24), achieved
TFLOP/s or GB/s, and for GEMMs the hipBLASLt (torch.matmul) time on the same
random operands.
"""
from __future__ import annotations

import argparse
import json
import statistics

import torch

from distributed_tf_serving_amd import ops


def _time(fn, iters=50, rounds=5):
    fn()
    torch.cuda.synchronize()
    res = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e) * 1e3 / iters)
    return statistics.median(res)


def bench_gemm(M, N, K, act="relu", dev="cuda"):
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    ours = _time(lambda: ops.linear(x, W, b, act))
    lib = _time(lambda: torch.relu(torch.addmm(b.to(torch.bfloat16), x, W.t())))
    flops = 2.0 * M * N * K
    xq, sx = ops.quant_rows_fp8(x)
    wq, sw = ops.quant_rows_fp8(W)
    f8 = _time(lambda: ops.linear_fp8(xq, sx, wq, sw, b, act))
    out = {"op": "gemm", "M": M, "N": N, "K": K, "us": round(ours, 2), "tflops": round(flops / ours / 1e6, 1),
           "hipblaslt_us": round(lib, 2), "hipblaslt_tflops": round(flops / lib / 1e6, 1),
           "fp8_us": round(f8, 2), "fp8_tflops": round(flops / f8 / 1e6, 1)}
    try:  # hipBLASLt fp8 (e4m3, per-tensor scales) on the same shape
        a8 = x.float().clamp(-448, 448).to(torch.float8_e4m3fn)
        w8 = W.float().mul(K ** 0.5).clamp(-448, 448).to(torch.float8_e4m3fn)
        one = torch.ones((), device=dev)
        lib8 = _time(lambda: torch._scaled_mm(a8, w8.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16))
        out.update(hipblaslt_fp8_us=round(lib8, 2), hipblaslt_fp8_tflops=round(flops / lib8 / 1e6, 1))
    except Exception as e:  # noqa: BLE001 - not every torch build has a fp8 hipBLASLt path
        out["hipblaslt_fp8"] = f"unavailable: {type(e).__name__}: {str(e)[:80]}"
    return out


def bench_gemm_variants(M, N, K, dev="cuda", variants=(0, 4, 8, 10, 14, 17)):
    """Interleaved A/B of the GEMM kernel variants in one process (rule 24)."""
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    h = ops.hip()
    ref = h.gemm(x, W, b, 1, None, None, True, None, None, None, 0)
    res = {"op": "gemm_variants", "M": M, "N": N, "K": K}
    # variant >= 100: same kernel as (variant - 100) with the legacy M-fastest tile order
    def call(v, f32=False):
        return h.gemm(x, W, b, 1 | (16 if v >= 100 else 0), None, None, f32, None, None, None, v % 100)
    fns = {v: (lambda v=v: call(v)) for v in variants}
    for v in variants:
        out = call(v, True)
        err = (out - ref).abs().max().item()
        res[f"v{v}_maxerr"] = round(err, 5)
    times = {v: [] for v in variants}
    for _ in range(5):
        for v in variants:
            times[v].append(_time(fns[v], iters=20, rounds=1))
    for v in variants:
        us = statistics.median(times[v])
        res[f"v{v}_us"] = round(us, 2)
        res[f"v{v}_tf"] = round(2.0 * M * N * K / us / 1e6, 1)
    lib = _time(lambda: torch.addmm(b.to(torch.bfloat16), x, W.t()))
    res["hipblaslt_us"] = round(lib, 2)
    return res


def bench_embed(B, F=43, D=64, V=1_000_000, dev="cuda"):
    table = torch.randn(V, D, device=dev).to(torch.bfloat16)
    lin = torch.randn(V, device=dev)
    ids = torch.randint(0, V, (B, F), device=dev, dtype=torch.int32)
    wts = torch.rand(B, F, device=dev)
    us = _time(lambda: ops.embed(table, ids, wts, lin=lin, modulo=V, want_x=True, want_fm=True, fm2=True))
    byts = B * F * (D * 2 * 2 + 4 + 4 + 4)
    ref = _time(lambda: (table[ids.long()] * wts.unsqueeze(-1).to(torch.bfloat16)).view(B, -1))
    return {"op": "embed_fm", "B": B, "F": F, "D": D, "us": round(us, 2), "GBps": round(byts / us / 1e3, 1),
            "torch_gather_us": round(ref, 2)}


def bench_model(family, B, dev="cuda", graphs=True):
    from distributed_tf_serving_amd.config import ModelConfig
    from distributed_tf_serving_amd.models import build_model

    cfg = ModelConfig(family=family)
    if family == "dlrm":
        cfg.table_rows = 1_000_000
    m = build_model(cfg, dev)
    ids = torch.randint(0, 1 << 30, (B, cfg.num_fields), device=dev)
    wts = torch.rand(B, cfg.num_fields, device=dev)
    eager = _time(lambda: m(ids, wts), iters=20)
    out = {"op": f"model_{family}", "B": B, "eager_us": round(eager, 1)}
    if graphs:
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                m(ids, wts)
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(g):
            m(ids, wts)
        gt = _time(lambda: g.replay(), iters=50)
        out["graph_us"] = round(gt, 1)
        out["Mscores_per_s"] = round(B / gt, 2)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--gemm-variants", action="store_true")
    ap.add_argument("--embed-study", action="store_true")
    ap.add_argument("--gather-gemm", action="store_true", help="K1 fused into K4 vs gather + GEMM")
    ap.add_argument("--gg-id-space", type=int, default=1 << 40, help="--gather-gemm: ids drawn (zipf) from [0, this)")
    ap.add_argument("--gg-rows", default="2048,4096,8192,16384", help="--gather-gemm: row counts")
    ap.add_argument("--gather-locality", action="store_true",
                    help="gather-GEMM time by where the table rows come from (L2 / MALL / HBM)")
    ap.add_argument("--variants", default="", help="M,N,K:v1,v2,... interleaved A/B of GEMM variants")
    ap.add_argument("--tail", action="store_true",
                    help="MLP tail 1024 -> 512 -> 256 -> score: GEMM2 + fused head vs the one-kernel tail")
    ap.add_argument("--serving", action="store_true",
                    help="the serving-step GEMM shapes (DeepFM 16384 rows, DCN-v2 8192 rows) vs hipBLASLt")
    ap.add_argument("--dcn", action="store_true",
                    help="DCN-v2 fp8: 8-phase vs one-wave cross layer, and graph-captured forwards per variant")
    ap.add_argument("--dcn-rows", default="2048,8192,16384")
    a = ap.parse_args()
    torch.manual_seed(0)
    if a.dcn:
        dcn_study(rows=tuple(int(x) for x in a.dcn_rows.split(",")))
        return
    if a.serving:
        for s in ((16384, 1024, 2752), (16384, 512, 1024), (16384, 256, 512), (8192, 2752, 2752),
                  (8192, 1024, 2752)):
            print(json.dumps(bench_gemm(*s)), flush=True)
        print(json.dumps(bench_embed(16384)), flush=True)
        return
    if a.variants:
        shape, vs = a.variants.split(":")
        M, N, K = (int(x) for x in shape.split(","))
        print(json.dumps(bench_gemm_variants(M, N, K, variants=tuple(int(v) for v in vs.split(",")))), flush=True)
        return
    if a.tail:
        for r in tail_study():
            print(json.dumps(r), flush=True)
        return
    if a.gather_locality:
        for r in gather_locality_study():
            print(json.dumps(r), flush=True)
    if a.gather_gemm:
        for r in gather_gemm_study(rows=tuple(int(x) for x in a.gg_rows.split(",")), id_space=a.gg_id_space):
            print(json.dumps(r), flush=True)
        return
    if a.embed_study:
        for r in embed_study():
            print(json.dumps(r), flush=True)
        return
    if a.gemm_variants:
        narrow = (0, 10, 14, 17)
        wide = (0, 4, 14, 17)
        for s, v in [((8192, 512, 1024), narrow), ((16384, 512, 1024), narrow), ((8192, 256, 512), narrow),
                     ((8192, 1024, 2752), wide), ((16384, 1024, 2752), wide), ((8192, 2752, 2752), wide)]:
            print(json.dumps(bench_gemm_variants(*s, variants=v)), flush=True)
        return
    shapes = [(512, 1024, 2752), (512, 512, 1024), (512, 256, 512), (4096, 1024, 2752), (8192, 1024, 2752),
              (4096, 2752, 2752)]
    if a.quick:
        shapes = shapes[:2]
    for s in shapes:
        print(json.dumps(bench_gemm(*s)), flush=True)
    for B in ([512] if a.quick else [512, 4096, 8192]):
        print(json.dumps(bench_embed(B)), flush=True)
    for fam in (["deepfm"] if a.quick else ["deepfm", "dcn", "dcn_v2", "wdl", "dlrm"]):
        for B in ([512] if a.quick else [512, 4096]):
            print(json.dumps(bench_model(fam, B)), flush=True)



def tail_study(rows=(2048, 8192, 16384), dev="cuda", rounds=5):
    """DeepFM / WDL / DCN MLP tail (h1 [M, 1024] -> 512 -> 256 -> sigmoid score):
    GEMM2 (ops.linear) + fused last layer/head (ops.linear_head) vs ONE
    ops.mlp_tail launch, interleaved; both checked against an fp32 reference."""
    out = []
    for M in rows:
        g = torch.Generator(device="cpu").manual_seed(M)
        x = (torch.rand(M, 1024, generator=g) - 0.5).to(torch.bfloat16).to(dev)
        W2 = ((torch.rand(512, 1024, generator=g) - 0.5) / 16).to(torch.bfloat16).to(dev)
        W3 = ((torch.rand(256, 512, generator=g) - 0.5) / 11).to(torch.bfloat16).to(dev)
        b2 = ((torch.rand(512, generator=g) - 0.5) * 0.1).to(dev)
        b3 = ((torch.rand(256, generator=g) - 0.5) * 0.1).to(dev)
        hw = ((torch.rand(256, generator=g) - 0.5) * 0.1).to(dev)
        extra = (torch.rand(2, M, generator=g) - 0.5).to(dev)
        W2p, W3p = ops.pack_bfrag(W2), ops.pack_bfrag(W3)
        h2 = torch.relu(x.float() @ W2.float().t() + b2).to(torch.bfloat16).float()
        ref = torch.sigmoid(torch.relu(h2 @ W3.float().t() + b3) @ hw + extra.sum(0))

        def two():
            return ops.linear_head(ops.linear(x, W2, b2, "relu"), W3, b3, "relu", hw, 0.0, extra=extra)

        def one():
            return ops.mlp_tail(x, W2p, b2, "relu", W3p, b3, "relu", hw, 0.0, extra=extra)

        times = {"two_kernels": [], "mlp_tail": []}
        for _ in range(rounds):
            times["two_kernels"].append(_time(two, rounds=1))
            times["mlp_tail"].append(_time(one, rounds=1))
        res = {"op": "mlp_tail", "M": M}
        for k, fn in (("two_kernels", two), ("mlp_tail", one)):
            y = fn()
            torch.cuda.synchronize()
            res[f"{k}_us"] = round(statistics.median(times[k]), 2)
            res[f"{k}_maxdiff_fp32"] = float((y - ref).abs().max())
        flops = 2.0 * M * (1024 * 512 + 512 * 256)
        res["mlp_tail_tflops"] = round(flops / res["mlp_tail_us"] / 1e6, 1)
        out.append(res)
    return out


def dcn_study(rows=(2048, 8192, 16384), dev="cuda", rounds=5):
    """DCN-v2 fp8 (preset dcn_v2_fp8): one cross layer on the fused 8-phase
    kernel (ops.cross_gemm_fp8), then the whole forward as a captured graph,
    interleaved rounds."""
    from distributed_tf_serving_amd.client.synth import SyntheticRequests
    from distributed_tf_serving_amd.config import load_preset
    from distributed_tf_serving_amd.models import build_model

    cfg = load_preset("dcn_v2_fp8").model
    m = build_model(cfg, dev)
    out = []
    for B in rows:
        ids_np, wts_np = SyntheticRequests(fields=cfg.num_fields, id_space=1 << 40, dist="zipf", seed=B).arrays(B)
        ids, wts = torch.from_numpy(ids_np).to(dev), torch.from_numpy(wts_np).to(dev)
        # one cross layer alone (the middle one: writes z)
        x0 = (torch.randn(B, m.d, device=dev) * 0.5).to(torch.bfloat16)
        q, sx = ops.quant_rows_fp8(x0, ops.FP8_K_PAD)
        layer = m.cross[1]

        def c8():
            return ops.cross_gemm_fp8(q, sx, layer.w_fp8, layer.w_scale, layer.bias, x0, x0, want_z=True)

        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                m(ids, wts)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            m(ids, wts)
        tc, tg = [], []
        for _ in range(rounds):
            tc.append(_time(c8, 20, 1))
            tg.append(_time(g.replay, 20, 1))
        r = {"op": "dcn_v2", "B": B, "cross_us": round(statistics.median(tc), 2),
             "graph_forward_us": round(statistics.median(tg), 1)}
        r["cross_tflops"] = round(2.0 * B * m.d * q.shape[1] / r["cross_us"] / 1e6, 1)
        out.append(r)
        print(json.dumps(r), flush=True)
        del g
    return out


def gather_gemm_study(rows=(2048, 4096, 8192, 16384), F=43, V=1_000_000, N=1024, dev="cuda", id_space=1 << 40):
    """K1 fused into K4 vs the separate gather + GEMM at the DeepFM serving
    shape (Zipf ids, 1M x 64 table): resolve + gather-GEMM vs embed(x, FM) +
    8-phase GEMM, interleaved rounds; also each half alone."""
    from distributed_tf_serving_amd.client.synth import SyntheticRequests

    table = (torch.randn(V, 64, device=dev) * 0.05).to(torch.bfloat16)
    lin = torch.randn(V, device=dev) * 0.01
    W = (torch.randn(N, F * 64, device=dev) * 0.02).to(torch.bfloat16)
    b = torch.randn(N, device=dev) * 0.01
    out = []
    for B in rows:
        ids_np, wts_np = SyntheticRequests(fields=F, id_space=id_space, dist="zipf", seed=B).arrays(B)
        ids, wts = torch.from_numpy(ids_np).to(dev), torch.from_numpy(wts_np).to(dev)

        def unfused():
            x, fm = ops.embed(table, ids, wts, lin=lin, modulo=V, want_x=True, want_fm=True, fm2=True)
            return ops.linear(x, W, b, "relu")

        def fused():
            return ops.embed_gemm(table, ids, wts, lin, V, 0.0, W, b, "relu", fm2=True)

        def fused_nofm():
            return ops.embed_gemm(table, ids, wts, lin, V, 0.0, W, b, "relu", fm2=False)

        Wp = ops.pack_frag32(W)
        res = ops.embed_gemm_resolve(table, ids, wts, lin, V, 0.0, True)

        def gg8():  # the GEMM half alone, 8-phase (gemm.hip)
            return ops.embed_gemm(table, ids, wts, lin, V, 0.0, W, b, "relu", fm2=True, resolved=res)

        def gg1w():  # the GEMM half alone, one wave per SIMD (gather_gemm.hip)
            return ops.embed_gemm(table, ids, wts, lin, V, 0.0, W, b, "relu", fm2=True, resolved=res,
                                  packed_w=lambda: Wp)

        torch.testing.assert_close(gg1w()[0].float(), gg8()[0].float(), atol=1e-2, rtol=1e-2)
        x, _ = ops.embed(table, ids, wts, lin=lin, modulo=V, want_x=True, want_fm=True, fm2=True)
        t = {k: [] for k in ("unfused", "fused", "embed", "gemm", "fused_nofm", "gg8", "gg1w")}
        for _ in range(5):  # interleaved
            t["gg8"].append(_time(gg8, 20, 1))
            t["gg1w"].append(_time(gg1w, 20, 1))
            t["unfused"].append(_time(unfused, 20, 1))
            t["fused"].append(_time(fused, 20, 1))
            t["fused_nofm"].append(_time(fused_nofm, 20, 1))
            t["embed"].append(_time(lambda: ops.embed(table, ids, wts, lin=lin, modulo=V, want_x=True,
                                                      want_fm=True, fm2=True), 20, 1))
            t["gemm"].append(_time(lambda: ops.linear(x, W, b, "relu"), 20, 1))
        r = {"op": "gather_gemm", "B": B, "N": N, "K": F * 64, "id_space": id_space}
        for k, v in t.items():
            r[f"{k}_us"] = round(statistics.median(v), 2)
        r["fused_tflops"] = round(2.0 * B * N * F * 64 / r["fused_us"] / 1e6, 1)
        r["gg1w_tflops"] = round(2.0 * B * N * F * 64 / r["gg1w_us"] / 1e6, 1)
        out.append(r)
    return out


def gather_locality_study(rows=(2048, 16384), F=43, V=1_000_000, N=1024, dev="cuda"):
    """Is the gather-GEMM bound by where its A rows come from? The same fused
    kernel on ids whose table rows are: all within 256 rows (L2-resident),
    sequential (row = 43 m + f), Zipf over 2^40 (the bench), uniform over the
    1M-row table; plus the dense 8-phase GEMM on the materialised x. ids map
    to rows by id mod V (K0), so the row pattern is chosen exactly."""
    from distributed_tf_serving_amd.client.synth import SyntheticRequests

    table = (torch.randn(V, 64, device=dev) * 0.05).to(torch.bfloat16)
    lin = torch.randn(V, device=dev) * 0.01
    W = (torch.randn(N, F * 64, device=dev) * 0.02).to(torch.bfloat16)
    b = torch.randn(N, device=dev) * 0.01
    out = []
    for B in rows:
        g = torch.Generator(device="cpu").manual_seed(B)
        zipf_np, wts_np = SyntheticRequests(fields=F, id_space=1 << 40, dist="zipf", seed=B).arrays(B)
        wts = torch.from_numpy(wts_np).to(dev)
        pats = {
            "l2_hot256": torch.randint(0, 256, (B, F), generator=g),
            "sequential": (torch.arange(B * F).view(B, F) % V),
            "zipf": torch.from_numpy(zipf_np),
            "uniform": torch.randint(0, V, (B, F), generator=g),
        }
        pats = {k: v.to(torch.int64).to(dev) for k, v in pats.items()}
        x, _ = ops.embed(table, pats["zipf"], wts, lin=lin, modulo=V, want_x=True, want_fm=True, fm2=True)
        t = {k: [] for k in list(pats) + ["dense_gemm"]}
        for _ in range(5):
            for k, ids in pats.items():
                t[k].append(_time(lambda: ops.embed_gemm(table, ids, wts, lin, V, 0.0, W, b, "relu", fm2=True), 20, 1))
            t["dense_gemm"].append(_time(lambda: ops.linear(x, W, b, "relu"), 20, 1))
        r = {"op": "gather_locality", "B": B, "N": N, "K": F * 64}
        for k, v in t.items():
            r[f"{k}_us"] = round(statistics.median(v), 2)
        out.append(r)
    return out


def embed_study(B=16384, F=43, D=64, V=1_000_000, dev="cuda"):
    """Where the K1 time goes at the bench shape: id distribution, x write, FM terms."""
    from distributed_tf_serving_amd.client.synth import SyntheticRequests

    table = torch.randn(V, D, device=dev).to(torch.bfloat16)
    lin = torch.randn(V, device=dev)
    out = []
    for dist in ("zipf", "uniform"):
        ids_np, wts_np = SyntheticRequests(fields=F, id_space=1 << 40, dist=dist).arrays(B)
        ids = torch.from_numpy(ids_np).to(dev)
        wts = torch.from_numpy(wts_np).to(dev)
        for name, kw in (("x+fm", dict(want_x=True, want_fm=True, fm2=True, lin=lin)),
                         ("fm_only", dict(want_x=False, want_fm=True, fm2=True, lin=lin)),
                         ("x_only", dict(want_x=True, want_fm=False))):
            us = _time(lambda: ops.embed(table, ids, wts, modulo=V, **kw))
            out.append({"op": "embed_study", "dist": dist, "variant": name, "B": B, "us": round(us, 2)})
    # resident-wave cap of the pipelined gather (rows per wave = B / cap; 0 = one row per wave)
    ids_np, wts_np = SyntheticRequests(fields=F, id_space=1 << 40, dist="zipf").arrays(B)
    ids, wts = torch.from_numpy(ids_np).to(dev), torch.from_numpy(wts_np).to(dev)
    h = ops.hip()
    for cap in (0, 2048, 4096, 8192, 16384):
        h.set_embed_wave_cap(cap)
        us = _time(lambda: ops.embed(table, ids, wts, modulo=V, want_x=True, want_fm=True, fm2=True, lin=lin))
        out.append({"op": "embed_study", "dist": "zipf", "variant": f"x+fm wave_cap={cap}", "B": B, "us": round(us, 2)})
    h.set_embed_wave_cap(4096)
    x = torch.empty(B, F * D, device=dev, dtype=torch.bfloat16)
    us = _time(lambda: x.fill_(1.0))
    out.append({"op": "embed_study", "variant": "fill_x (write-BW floor)", "us": round(us, 2),
                "GBps": round(x.numel() * 2 / us / 1e3, 1)})
    return out



if __name__ == "__main__":
    main()
