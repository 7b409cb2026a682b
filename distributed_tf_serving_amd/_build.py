"""In-tree native build: host runtime (`_native`) and gfx950 HIP kernels (`_hip`).

No hipify, no setuptools CUDAExtension: every ``.hip`` translation unit under
``csrc/kernels`` is compiled directly with ``hipcc --offload-arch=gfx950`` into
an object, host-side C++ with the system compiler, and both are linked into
Python extension modules that land next to this file (so the ``.so`` travels
with the repo snapshot to the GPU box and is what the tests load).

Incremental: an object is rebuilt when its source or any header under
``csrc/`` is newer. Compiles run in parallel (``MAX_JOBS``, default 8).

    python -m distributed_tf_serving_amd._build          # build both
    python -m distributed_tf_serving_amd._build --clean
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
CSRC = os.path.join(REPO, "csrc")
BUILD = os.path.join(REPO, "build", "native")
ARCH = "gfx950"  # the only target (MI355X / CDNA4)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"

NATIVE_SOURCES = [
    "bindings_native.cpp",
    "wire/tensor_codec.cpp",
    "runtime/batcher.cpp",
    "runtime/thread_pool.cpp",
    "runtime/arena.cpp",
    "runtime/trace.cpp",
    "runtime/live_server.cpp",
    "runtime/loadgen.cpp",
    "runtime/narrow.cpp",
    "runtime/step_control.cpp",
    "net/hpack.cpp",
    "net/h2_server.cpp",
    "net/h2_client.cpp",
    "runtime/numa.cpp",
    "runtime/shared_scatter.cpp",
]
HIP_HOST_SOURCES = ["bindings_hip.cpp", "runtime/step_runner.cpp", "comm/rccl_comm.cpp",
                    "runtime/kernel_seq.cpp",
                    # shared with _native (the loop parses arenas / encodes responses itself)
                    "runtime/arena.cpp", "runtime/thread_pool.cpp", "wire/tensor_codec.cpp", "runtime/trace.cpp",
                    "runtime/batcher.cpp", "runtime/live_server.cpp", "runtime/loadgen.cpp", "runtime/narrow.cpp",
                    "runtime/step_control.cpp", "net/hpack.cpp", "net/h2_server.cpp", "runtime/numa.cpp",
                    "runtime/shared_scatter.cpp"]


def _torch_paths():
    import torch

    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    return tdir, inc, os.path.join(tdir, "lib"), int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _common_defs(name: str, abi: int):
    return [
        f"-DTORCH_EXTENSION_NAME={name}",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
    ]


def _headers_mtime() -> float:
    hs = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    hs += glob.glob(os.path.join(CSRC, "**", "*.cuh"), recursive=True)
    hs += glob.glob(os.path.join(CSRC, "**", "*.hpp"), recursive=True)
    return max([os.path.getmtime(h) for h in hs] + [0.0])


def _stale(obj: str, src: str, hdr_mtime: float) -> bool:
    if not os.path.exists(obj):
        return True
    m = os.path.getmtime(obj)
    return m < os.path.getmtime(src) or m < hdr_mtime


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}):\n{' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def _compile_all(jobs, verbose):
    n = int(os.environ.get("MAX_JOBS", "8"))
    with cf.ThreadPoolExecutor(max_workers=max(1, min(n, 16))) as ex:
        futs = [ex.submit(_run, cmd, verbose) for cmd in jobs]
        for f in futs:
            f.result()


def _py_includes():
    return [sysconfig.get_paths()["include"]]


SANITIZE_FLAGS = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"]
TSAN_FLAGS = ["-fsanitize=thread", "-fno-omit-frame-pointer"]


def build_native(verbose=False, force=False, sanitize=False) -> str:
    """``sanitize``: ASan + UBSan (True / "address") or ThreadSanitizer
    ("thread") host build of the native runtime, into its
    own object dir. Run it with the sanitizer runtime
    preloaded and ``DTFS_NATIVE_SO`` pointing at it, e.g.
    ``scripts/sanitize_native.sh`` (the in-tree .so is left alone)."""
    tdir, tinc, tlib, abi = _torch_paths()
    san = [] if not sanitize else (TSAN_FLAGS if sanitize == "thread" else SANITIZE_FLAGS)
    odir = os.path.join(BUILD, {"thread": "native_tsan"}.get(sanitize, "native_asan") if sanitize else "native")
    # a sanitizer build lands in its own directory, never over the in-tree .so
    # (GPU runs ship the package directory); load it with DTFS_NATIVE_SO=<path>
    out = os.path.join(odir if sanitize else PKG_DIR, "_native" + EXT_SUFFIX)
    os.makedirs(odir, exist_ok=True)
    hdr = _headers_mtime()
    flags = ["-O1" if sanitize else "-O3", "-g" if sanitize else "-g0", "-std=c++17", "-fPIC", "-Wall",
             "-Wno-unused-function", "-fvisibility=hidden",
             f"-I{CSRC}"] + [f"-I{p}" for p in tinc + _py_includes()] + _common_defs("_native", abi)
    if sanitize:
        flags += san
        force = True  # the output name is shared with the normal build
    objs, jobs = [], []
    for s in NATIVE_SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(odir, s.replace("/", "_") + ".o")
        objs.append(obj)
        if force or _stale(obj, src, hdr):
            jobs.append([CXX, *flags, "-c", src, "-o", obj])
    _compile_all(jobs, verbose)
    if force or jobs or not os.path.exists(out):
        _run([CXX, "-shared", "-o", out, *objs, *san, f"-L{tlib}", "-lc10",
              "-ltorch", "-ltorch_cpu", "-ltorch_python", "-ldl", f"-Wl,-rpath,{tlib}"], verbose)
    return out


def _file_flags(src: str):
    """Per-kernel-file compiler flags: a ``// hipcc-flags: ...`` line in the
    file's first 60 lines (e.g. gather_gemm.hip turns SLP vectorisation off:
    packed f32 VALU beside MFMAs costs more issue cycles than scalar)."""
    with open(src) as f:
        for _, line in zip(range(60), f):
            if line.startswith("// hipcc-flags:"):
                return line.split(":", 1)[1].split()
    return []


def build_hip(verbose=False, force=False) -> str:
    tdir, tinc, tlib, abi = _torch_paths()
    out = os.path.join(PKG_DIR, "_hip" + EXT_SUFFIX)
    odir = os.path.join(BUILD, "hip")
    os.makedirs(odir, exist_ok=True)
    hdr = _headers_mtime()
    dev_flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-x", "hip", f"-I{CSRC}",
                 "-munsafe-fp-atomics", "-Wno-unused-result"]
    host_flags = ["-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", f"--offload-arch={ARCH}", f"-I{CSRC}",
                  "-D__HIP_PLATFORM_AMD__=1",
                  "-DUSE_ROCM=1", "-DHIPBLAS_V2", "-I/opt/rocm/include", "-Wno-unused-result"] + \
                 [f"-I{p}" for p in tinc + _py_includes()] + _common_defs("_hip", abi)
    objs, jobs = [], []
    for src in sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip"))):
        obj = os.path.join(odir, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _stale(obj, src, hdr):
            jobs.append([HIPCC, *dev_flags, *_file_flags(src), "-c", src, "-o", obj])
    for s in HIP_HOST_SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(odir, s.replace("/", "_") + ".o")
        objs.append(obj)
        if force or _stale(obj, src, hdr):
            jobs.append([HIPCC, *host_flags, "-c", src, "-o", obj])
    _compile_all(jobs, verbose)
    if force or jobs or not os.path.exists(out):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "--hip-link", "-o", out, *objs,
              f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
              # RCCL is not linked: csrc/comm resolves it from torch's loaded copy
              "-lamdhip64", "-ldl", f"-Wl,-rpath,{tlib}"], verbose)
    return out


def build_all(verbose=False, force=False):
    return build_native(verbose, force), build_hip(verbose, force)


def clean():
    shutil.rmtree(os.path.join(REPO, "build"), ignore_errors=True)
    for f in glob.glob(os.path.join(PKG_DIR, "_native*.so")) + glob.glob(os.path.join(PKG_DIR, "_hip*.so")):
        os.remove(f)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--native-only", action="store_true")
    ap.add_argument("--sanitize", nargs="?", const="address", default=None, choices=["address", "thread"],
                    help="ASan+UBSan (default) or TSan host build of _native (implies --native-only)")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    if a.clean:
        clean()
        sys.exit(0)
    print(build_native(a.verbose, a.force or bool(a.sanitize), sanitize=a.sanitize or False))
    if a.sanitize:
        sys.exit(0)
    if not a.native_only:
        print(build_hip(a.verbose, a.force))
