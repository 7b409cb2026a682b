"""Static check of hand-scheduled gfx950 kernels for asynchronous-load register
hazards: an instruction that reads or writes a VGPR / AGPR that is still the
destination of an in-flight VMEM or LDS load (before the s_waitcnt that
retires it).

Why: the kernels issue their loads from inline asm and retire them with
counted s_waitcnt. The compiler models an asm output as written when the asm
statement ends, so it may copy, spill or reuse such a register before the
data has arrived; a late return then overwrites whatever the register holds
by then - e.g. an address, which faulted the GPU (memory aperture violation)
only when load latencies were long (graph replays).

    hipcc --offload-arch=gfx950 -O3 --cuda-device-only -S k.hip -o k.s ...
    python -m tools.isa_hazards k.s [--kernel NAME]

Only loads issued from inline asm are tracked (the compiler places its own
waits for its own loads, on every control-flow path). Walks each kernel's
instructions in textual order, running every loop body (a backward
branch) twice so loads in flight across the back edge are covered. vmcnt counts
VMEM loads and stores in order (gfx9 has no separate store counter); lgkmcnt
counts LDS ops in order (SMEM loads are retired by the compiler's lgkmcnt(0)).
Exit status 1 if any hazard is found.
"""
from __future__ import annotations

import argparse
import re
import sys
from collections import deque

_REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)(?!\w))")
_WAIT = re.compile(r"s_waitcnt\s+(.*)")
_CNT = re.compile(r"(vmcnt|lgkmcnt|expcnt)\((\d+)\)")


def regs(text: str):
    out = set()
    for m in _REG.finditer(text):
        kind = m.group(1)
        if m.group(4) is not None:
            out.add((kind, int(m.group(4))))
        else:
            for r in range(int(m.group(2)), int(m.group(3)) + 1):
                out.add((kind, r))
    return out


def parse_kernels(lines):
    """{kernel name: [(lineno, text, from_asm)]} of instructions and labels."""
    kernels, cur, name = {}, None, None
    in_asm = False
    for i, raw in enumerate(lines, 1):
        if ";;#ASMSTART" in raw:
            in_asm = True
        elif ";;#ASMEND" in raw:
            in_asm = False
        line = raw.split(";")[0].rstrip()
        m = re.match(r"^([A-Za-z_.$][\w.$]*):", line)
        if m:  # a label at column 0: a kernel symbol, or a local .L / $ label
            label = m.group(1)
            if not label.startswith(".L") and not label.startswith("$"):
                name = label
                cur = kernels.setdefault(name, [])
                continue
            if cur is not None:
                cur.append((i, label + ":", False))
            continue
        s = line.strip()
        if not s or s.startswith(".") or cur is None:
            if s.startswith(".Lfunc_end") or s.startswith(".size"):
                cur = None
            continue
        cur.append((i, s, in_asm))
    return kernels


def is_vmem(op):
    return op.startswith(("global_", "buffer_", "flat_", "scratch_"))


def is_lds(op):
    return op.startswith("ds_")


def writes_dest(op):
    if op.startswith(("global_store", "buffer_store", "flat_store", "scratch_store", "ds_write", "ds_store")):
        return False
    if "_lds_" in op or op.endswith("_lds"):
        return False  # LDS-DMA: no register destination
    return "load" in op or op.startswith("ds_read") or op.startswith("ds_bpermute") or op.startswith("ds_swizzle")


def check(instrs, limit=50):
    labels = {t[:-1]: k for k, (_, t, _) in enumerate(instrs) if t.endswith(":")}
    vm, lg = deque(), deque()  # pending: (dest regs, lineno, text)
    found = []
    seen_back = set()
    k = 0
    steps = 0
    while k < len(instrs) and steps < 200000:
        steps += 1
        ln, t, from_asm = instrs[k]
        k += 1
        if t.endswith(":"):
            continue
        op = t.split()[0]
        if op == "s_waitcnt":
            for c, n in _CNT.findall(t):
                n = int(n)
                q = vm if c == "vmcnt" else lg if c == "lgkmcnt" else None
                if q is not None:
                    while len(q) > n:
                        q.popleft()
            continue
        rs = regs(t.split(None, 1)[1] if " " in t else "")
        for q, qn in ((vm, "vmcnt"), (lg, "lgkmcnt")):
            for dest, pln, ptxt in q:
                hit = dest & rs
                if hit:
                    found.append((ln, t, pln, ptxt, qn, sorted(hit)[:4]))
        # only loads from inline asm are tracked for hazards (the compiler's own
        # loads get its own waits); every load still takes a counter slot
        if is_vmem(op):
            vm.append((regs(t.split(None, 1)[1].split(",")[0]) if writes_dest(op) and from_asm else set(), ln, t))
        elif is_lds(op):
            lg.append((regs(t.split(None, 1)[1].split(",")[0]) if writes_dest(op) and from_asm else set(), ln, t))
        if op.startswith("s_cbranch") or op == "s_branch":
            target = t.split()[-1]
            tk = labels.get(target)
            if tk is not None and tk < k and (ln not in seen_back):
                seen_back.add(ln)  # run the loop body once more with what is in flight
                k = tk
        if op == "s_endpgm":
            break
        if len(found) >= limit:
            break
    return found


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--kernel", default="")
    a = ap.parse_args(argv)
    with open(a.asm) as f:
        kernels = parse_kernels(f.read().splitlines())
    bad = 0
    for name, instrs in kernels.items():
        if a.kernel and a.kernel not in name:
            continue
        found = check(instrs)
        print(f"{name[:80]}: {len(instrs)} lines, {len(found)} hazard(s)")
        for ln, t, pln, ptxt, qn, hit in found[:20]:
            print(f"  line {ln}: `{t}` touches {hit} of the {qn} load at line {pln}: `{ptxt}`")
        bad += len(found)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
