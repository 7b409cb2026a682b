"""Summarise rocprofv3 counter passes (scripts/gpu_study.sh counters) per kernel.

Reads every ``*counter_collection.csv`` under a directory (one rocprofv3 run
per counter pass), averages each counter per dispatch of each kernel, and
prints a markdown table with the derived metrics:

* ``mfma_busy``   SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x kernel cycles), kernel
                  cycles = GRBM_GUI_ACTIVE / 8 XCDs (MI355X_MICROARCH.md, DVFS)
* ``clock_ghz``   GRBM_GUI_ACTIVE / 8 / kernel duration
* ``lds_conflict`` SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles per LDS cycle)
* ``hbm_read_MB`` FETCH_SIZE x 2 / 1e3 (gfx950 FETCH_SIZE counts half the bytes of
                  wide streaming reads; MI355X_MICROARCH.md §HBM) - an estimate
* ``write_MB``    WRITE_SIZE / 1e3 (KB units)
* ``l2_hit``      TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
* ``waves/CU``    4 x SQ_WAVE_CYCLES / (256 CUs x kernel cycles): mean resident waves per CU (SQ_WAVE_CYCLES
                  counts quad-cycles)
* ``wait / stall / active``  SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY as shares of SQ_WAVE_CYCLES
                  (disjoint; wait = parked on s_waitcnt / barrier, stall = issue stall, active = issuing)
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os
import statistics

SIMDS = 256 * 4


def short(name: str) -> str:
    for key in ("gemm_gather", "dot_interact_gather", "bottom_mlp3", "embed_resolve", "gemm_8ph", "gemm_glds", "gemm_head", "embed_pipe", "arena_varint", "quant_rows", "gemm_fp8",
                "gemm_mx", "cross", "head_kernel", "dot_inter", "unpack"):
        if key in name:
            return key + (" (fp8)" if "DF16" not in name and "fp8" in name.lower() else "")
    return name[:48]


def load(root: str, only: str = ""):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    names = {}
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        if only and only not in os.path.relpath(path, root):
            continue
        with open(path) as f:
            for row in csv.DictReader(f):
                k = row.get("Kernel_Name", "")
                names[short(k)] = k
                cn, cv = row.get("Counter_Name"), row.get("Counter_Value")
                if cn is None or cv is None:
                    continue
                per[short(k)][cn].append(float(cv))
                try:
                    d = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-3
                    if d > 0:
                        dur[short(k)].append(d)
                except (KeyError, ValueError):
                    pass
    return per, dur, names


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--title", default="kernel counters")
    ap.add_argument("--only", default="", help="only counter files whose path under root contains this")
    a = ap.parse_args(argv)
    per, dur, names = load(a.root, a.only)
    print(f"# {a.title}\n")
    print("| kernel | us (profiled) | clock GHz | mfma_busy | waves/CU | wait / stall / active | LDS conflict | "
          "HBM read MB (est) | write MB | L2 hit | VALU insts | waves |")
    print("|---|---:|---:|---:|---:|---|---:|---:|---:|---:|---:|---:|")
    for k in sorted(per, key=lambda k: -statistics.mean(dur[k]) if dur[k] else 0):
        c = {n: statistics.mean(v) for n, v in per[k].items()}
        us = statistics.median(dur[k]) if dur[k] else float("nan")
        gui = c.get("GRBM_GUI_ACTIVE")
        cyc = gui / 8 if gui else None
        clk = (cyc / (us * 1e3)) if cyc and us == us else None
        mfma = c.get("SQ_VALU_MFMA_BUSY_CYCLES")
        busy = mfma / (SIMDS * cyc) if mfma is not None and cyc else None
        ldsc = (c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]) if c.get("SQ_LDS_IDX_ACTIVE") else None
        fetch = c.get("FETCH_SIZE")
        wr = c.get("WRITE_SIZE")
        hit, miss = c.get("TCC_HIT_sum"), c.get("TCC_MISS_sum")
        l2 = hit / (hit + miss) if hit is not None and miss and hit + miss > 0 else None

        def f(x, fmt):
            return fmt.format(x) if x is not None else "-"

        wc = c.get("SQ_WAVE_CYCLES")
        occ = 4 * wc / (256 * cyc) if wc and cyc else None
        wsa = "-"
        if wc and c.get("SQ_WAIT_ANY") is not None:
            wsa = " / ".join(f(c.get(n, 0) / wc, "{:.0%}") for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"))

        print(f"| `{k}` | {us:.1f} | {f(clk, '{:.2f}')} | {f(busy, '{:.1%}')} | {f(occ, '{:.1f}')} | {wsa} | {f(ldsc, '{:.3f}')} | "
              f"{f(fetch * 2 / 1e3 if fetch is not None else None, '{:.1f}')} | {f(wr / 1e3 if wr is not None else None, '{:.1f}')} | "
              f"{f(l2, '{:.1%}')} | {f(c.get('SQ_INSTS_VALU'), '{:.3g}')} | {f(c.get('SQ_WAVES'), '{:.0f}')} |")
    print()


if __name__ == "__main__":
    main()
