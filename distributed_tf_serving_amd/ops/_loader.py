"""Locate the in-tree native extensions.

``_hip`` holds the gfx950 kernels. GPU tensors are NEVER silently routed to a
PyTorch fallback: if the extension is missing or fails to load while a GPU op
is requested, :func:`hip` raises. CPU tensors use the reference math in the
op modules (that is the CPU backend, config 1 of BASELINE.json).
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_hip_mod = None
_hip_err = None
_native_mod = None
_native_err = None


def _autobuild_allowed() -> bool:
    return os.environ.get("DTFS_NO_AUTOBUILD", "0") != "1"


def hip():
    """The `_hip` extension module; raises RuntimeError if it cannot be loaded."""
    global _hip_mod, _hip_err
    if _hip_mod is not None:
        return _hip_mod
    with _lock:
        if _hip_mod is None:
            try:
                _hip_mod = importlib.import_module("distributed_tf_serving_amd._hip")
            except ImportError as e:  # pragma: no cover - depends on build state
                if _autobuild_allowed():
                    from .. import _build

                    _build.build_hip()
                    _hip_mod = importlib.import_module("distributed_tf_serving_amd._hip")
                else:
                    _hip_err = e
                    raise RuntimeError(
                        "gfx950 kernels (_hip) are not built: run `python -m distributed_tf_serving_amd._build`"
                    ) from e
            _hip_mod.rccl_set_library(_torch_rccl_path())
    return _hip_mod


def _torch_rccl_path() -> str:
    """PyTorch's bundled librccl (the one ProcessGroupNCCL uses); the system
    copy only when torch ships none."""
    import torch

    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return p if os.path.exists(p) else "librccl.so.1"


def _load_native_from(path: str):
    """A sanitizer build of `_native` kept out of the package directory
    (scripts/sanitize_native.sh sets DTFS_NATIVE_SO): the in-tree .so, which
    GPU runs ship, is never replaced by an instrumented one."""
    import importlib.util
    import sys

    spec = importlib.util.spec_from_file_location("distributed_tf_serving_amd._native", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    sys.modules["distributed_tf_serving_amd._native"] = mod
    return mod


def native():
    """The `_native` host runtime (wire codec, batcher)."""
    global _native_mod
    if _native_mod is not None:
        return _native_mod
    with _lock:
        if _native_mod is None and os.environ.get("DTFS_NATIVE_SO"):
            _native_mod = _load_native_from(os.environ["DTFS_NATIVE_SO"])
        if _native_mod is None:
            try:
                _native_mod = importlib.import_module("distributed_tf_serving_amd._native")
            except ImportError:
                if not _autobuild_allowed():
                    raise
                from .. import _build

                _build.build_native()
                _native_mod = importlib.import_module("distributed_tf_serving_amd._native")
    return _native_mod


def hip_loaded() -> bool:
    return _hip_mod is not None
