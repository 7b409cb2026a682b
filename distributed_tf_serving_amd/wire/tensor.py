"""TensorProto <-> numpy / torch conversion (the Python reference codec).

Semantics follow TF's ``tensor_util``:

* ``tensor_content`` (raw little-endian bytes) wins when present and must hold
  exactly ``prod(shape) * itemsize`` bytes.
* Otherwise the typed ``*_val`` field is used. If it holds FEWER values than the
  shape needs, the remaining elements repeat the LAST value (an empty field
  yields zeros); the reference smoke client relies on this
  (reference DCNClientSimple.java:33-51 declares ``[1500,43]`` but sends 87
  ids). MORE values than the shape needs is an INVALID_ARGUMENT error.

The hot path uses the native decoder in ``csrc/wire/tensor_codec.cpp``; this
module is its golden reference and the general (any dtype) path.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np

from . import schema as pb


class InvalidArgument(ValueError):
    """Maps to gRPC INVALID_ARGUMENT / TF-Serving error::INVALID_ARGUMENT."""


# dtype enum -> (numpy dtype, typed field name)
_DT = {
    pb.DT_FLOAT: (np.float32, "float_val"),
    pb.DT_DOUBLE: (np.float64, "double_val"),
    pb.DT_INT32: (np.int32, "int_val"),
    pb.DT_UINT8: (np.uint8, "int_val"),
    pb.DT_INT16: (np.int16, "int_val"),
    pb.DT_INT8: (np.int8, "int_val"),
    pb.DT_UINT16: (np.uint16, "int_val"),
    pb.DT_INT64: (np.int64, "int64_val"),
    pb.DT_BOOL: (np.bool_, "bool_val"),
    pb.DT_HALF: (np.float16, "half_val"),
    pb.DT_BFLOAT16: (np.uint16, "half_val"),  # bit pattern; see to_torch()
    pb.DT_UINT32: (np.uint32, "uint32_val"),
    pb.DT_UINT64: (np.uint64, "uint64_val"),
}

_NP2DT = {
    np.dtype(np.float32): pb.DT_FLOAT,
    np.dtype(np.float64): pb.DT_DOUBLE,
    np.dtype(np.int32): pb.DT_INT32,
    np.dtype(np.uint8): pb.DT_UINT8,
    np.dtype(np.int16): pb.DT_INT16,
    np.dtype(np.int8): pb.DT_INT8,
    np.dtype(np.uint16): pb.DT_UINT16,
    np.dtype(np.int64): pb.DT_INT64,
    np.dtype(np.bool_): pb.DT_BOOL,
    np.dtype(np.float16): pb.DT_HALF,
    np.dtype(np.uint32): pb.DT_UINT32,
    np.dtype(np.uint64): pb.DT_UINT64,
}


def numpy_dtype(dt: int):
    try:
        return _DT[dt][0]
    except KeyError:
        raise InvalidArgument(f"unsupported dtype {pb.DataTypeName.get(dt, dt)}") from None


def shape_of(tp) -> tuple:
    if tp.tensor_shape.unknown_rank:
        raise InvalidArgument("tensor with unknown rank")
    dims = tuple(int(d.size) for d in tp.tensor_shape.dim)
    if any(d < 0 for d in dims):
        raise InvalidArgument(f"negative dimension in shape {dims}")
    return dims


def make_shape(shape: Sequence[int]):
    s = pb.TensorShapeProto()
    for d in shape:
        s.dim.add().size = int(d)
    return s


def make_tensor_proto(values, dtype: Optional[int] = None, shape: Optional[Sequence[int]] = None,
                      raw: bool = False):
    """Build a TensorProto. ``raw=True`` uses ``tensor_content`` (fast path for
    large numeric tensors); otherwise the typed field, like the reference
    client's ``addAllInt64Val``/``addAllFloatVal`` (DCNClient.java:98-108)."""
    arr = np.asarray(values)
    if dtype is None:
        if arr.dtype not in _NP2DT:
            raise InvalidArgument(f"no TF dtype for numpy {arr.dtype}")
        dtype = _NP2DT[arr.dtype]
    np_dt, field = _DT[dtype]
    arr = np.ascontiguousarray(arr.astype(np_dt, copy=False))
    tp = pb.TensorProto()
    tp.dtype = dtype
    tp.tensor_shape.CopyFrom(make_shape(arr.shape if shape is None else shape))
    if raw:
        tp.tensor_content = arr.astype(arr.dtype.newbyteorder("<"), copy=False).tobytes()
    else:
        flat = arr.reshape(-1)
        if dtype == pb.DT_HALF:
            flat = flat.view(np.uint16).astype(np.int32)
        elif dtype == pb.DT_BFLOAT16:
            flat = flat.astype(np.int32)
        getattr(tp, field).extend(flat.tolist())
    return tp


def to_ndarray(tp) -> np.ndarray:
    """Decode a TensorProto into a numpy array (fill semantics, see module doc)."""
    if tp.dtype not in _DT:
        if tp.dtype == pb.DT_STRING:
            shape = shape_of(tp)
            vals = list(tp.string_val)
            return _fill(np.array(vals, dtype=object), shape, object)
        raise InvalidArgument(f"unsupported dtype {pb.DataTypeName.get(tp.dtype, tp.dtype)}")
    np_dt, field = _DT[tp.dtype]
    shape = shape_of(tp)
    n = int(np.prod(shape, dtype=np.int64)) if shape else 1
    if tp.tensor_content:
        want = n * np.dtype(np_dt).itemsize
        if len(tp.tensor_content) != want:
            raise InvalidArgument(
                f"tensor_content has {len(tp.tensor_content)} bytes, shape {shape} needs {want}")
        return np.frombuffer(tp.tensor_content, dtype=np.dtype(np_dt).newbyteorder("<")).astype(
            np_dt, copy=True).reshape(shape)
    vals = getattr(tp, field)
    if tp.dtype == pb.DT_HALF:
        src = np.asarray(vals, dtype=np.int32).astype(np.uint16).view(np.float16)
    elif tp.dtype == pb.DT_BFLOAT16:
        src = np.asarray(vals, dtype=np.int32).astype(np.uint16)
    else:
        src = np.asarray(vals, dtype=np_dt)
    return _fill(src, shape, np_dt)


def _fill(src: np.ndarray, shape: tuple, np_dt) -> np.ndarray:
    n = int(np.prod(shape, dtype=np.int64)) if shape else 1
    k = src.shape[0]
    if k > n:
        raise InvalidArgument(f"{k} values supplied for a tensor of {n} elements (shape {shape})")
    if k == n:
        return src.reshape(shape)
    out = np.empty(n, dtype=np_dt)
    if k == 0:
        out[...] = np.zeros((), dtype=np_dt) if np_dt is not object else b""
    else:
        out[:k] = src
        out[k:] = src[-1]
    return out.reshape(shape)


def to_torch(tp):
    """Decode into a torch tensor (bf16 bit patterns become torch.bfloat16)."""
    import torch

    arr = to_ndarray(tp)
    if tp.dtype == pb.DT_BFLOAT16:
        return torch.from_numpy(arr.astype(np.int16, copy=False).view(np.int16)).view(torch.bfloat16)
    if arr.dtype in (np.uint16, np.uint32, np.uint64):
        arr = arr.astype(np.int64)
    return torch.from_numpy(np.ascontiguousarray(arr))


def from_torch(t, raw: bool = True):
    import torch

    t = t.detach().cpu().contiguous()
    if t.dtype == torch.bfloat16:
        bits = t.view(torch.int16).numpy().view(np.uint16)
        return make_tensor_proto(bits, dtype=pb.DT_BFLOAT16, raw=raw)
    return make_tensor_proto(t.numpy(), raw=raw)
