"""Compile-time resource checks of the hand-scheduled gfx950 kernels (CPU:
hipcc cross-compiles, no GPU needed).

The one-wave-per-SIMD kernels run at the 512-register limit, where the
register allocator starts spilling to scratch around loop exits; a scratch
spill is slow and, captured into the served step's HIP graph, the round-5
gather-GEMM with 32 bytes of scratch per lane faulted the GPU (memory aperture
violation) while the same kernel passed every eager test. These kernels must
stay scratch-free.
"""
import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"

pytestmark = pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")


def _flags(path):
    with open(path) as f:
        for _, line in zip(range(60), f):
            if line.startswith("// hipcc-flags:"):
                return line.split(":", 1)[1].split()
    return []


def _resources(src: str):
    """{kernel symbol: {"scratch": bytes/lane, "vgprs": n, "agprs": n, "lds": bytes}}"""
    path = os.path.join(REPO, "csrc", "kernels", src)
    out = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-c", path,
                          "-o", os.devnull, "-I" + os.path.join(REPO, "csrc"), *_flags(path),
                          "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    res, cur = {}, None
    for line in out.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = res.setdefault(m.group(1), {})
            continue
        for key, pat in (("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"), ("vgprs", r"\bVGPRs: (\d+)"),
                         ("agprs", r"AGPRs: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
            m = re.search(pat, line)
            if m and cur is not None:
                cur[key] = int(m.group(1))
    return res


@pytest.mark.parametrize("src", ["gather_gemm.hip", "gather_mlp.hip", "mlp_tail.hip"])
def test_one_wave_kernels_are_scratch_free(src):
    res = _resources(src)
    assert res, f"no kernels found in {src}"
    for name, r in res.items():
        assert r.get("scratch") == 0, f"{src}: {name} spills {r.get('scratch')} bytes/lane to scratch"


@pytest.mark.parametrize("src", ["gather_gemm.hip", "gather_mlp.hip", "mlp_tail.hip", "gemm.hip", "embedding.hip"])
def test_inline_asm_loads_have_no_register_hazards(src, tmp_path):
    """No instruction touches a register an inline-asm load is still filling
    (tools/isa_hazards.py on the compiled gfx950 code): the round-5 one-wave
    cross kernel faulted the GPU in graph replays because the compiler had put
    epilogue address math into a register of a prefetch still in flight."""
    import sys

    sys.path.insert(0, REPO)
    from tools import isa_hazards

    path = os.path.join(REPO, "csrc", "kernels", src)
    asm = str(tmp_path / "k.s")
    out = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S", path,
                          "-o", asm, "-I" + os.path.join(REPO, "csrc"), *_flags(path)],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    with open(asm) as f:
        kernels = isa_hazards.parse_kernels(f.read().splitlines())
    bad = {name: isa_hazards.check(instrs) for name, instrs in kernels.items()}
    bad = {k: v[:3] for k, v in bad.items() if v}
    assert not bad, bad


def test_gather_gemm_uses_one_wave_per_simd_budget():
    # 256 AGPRs hold the 128 x 128 accumulator tile per wave; LDS: the 133 KB epilogue staging
    res = _resources("gather_gemm.hip")
    for name, r in res.items():
        assert r["agprs"] == 256 and r["vgprs"] <= 256, (name, r)
        assert r["lds"] <= 160 * 1024, (name, r)
