"""Compile the vendored serving schema into a FileDescriptorSet.

There is no ``grpc_tools`` in this image and no C++ protobuf headers, so the
schema is compiled once with the ``protoc`` that ships inside the torch wheel
and the resulting descriptor set (``serving_apis.desc``) is committed. At
runtime :mod:`.schema` builds message classes from it with
``google.protobuf.message_factory``; no generated ``_pb2`` modules exist.

The well-known types (``Any``, ``Int64Value``) are fed to protoc through
``--descriptor_set_in`` from the descriptors the Python protobuf runtime
already carries, because the torch wheel ships no ``google/protobuf/*.proto``.

Run: ``python -m distributed_tf_serving_amd.wire.gen_descriptors``
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
PROTO_DIR = os.path.join(HERE, "protos")
OUT = os.path.join(HERE, "serving_apis.desc")


def find_protoc() -> str:
    import torch

    cand = os.path.join(os.path.dirname(torch.__file__), "bin", "protoc")
    if os.path.exists(cand):
        return cand
    for p in os.environ.get("PATH", "").split(os.pathsep):
        c = os.path.join(p, "protoc")
        if os.path.exists(c):
            return c
    raise FileNotFoundError("protoc not found (expected torch/bin/protoc)")


def wkt_descriptor_set() -> bytes:
    from google.protobuf import any_pb2, descriptor_pb2, wrappers_pb2

    fds = descriptor_pb2.FileDescriptorSet()
    for mod in (any_pb2, wrappers_pb2):
        fdp = fds.file.add()
        mod.DESCRIPTOR.CopyToProto(fdp)
    return fds.SerializeToString()


def generate(out_path: str = OUT) -> str:
    protoc = find_protoc()
    with tempfile.TemporaryDirectory() as td:
        wkt = os.path.join(td, "wkt.desc")
        with open(wkt, "wb") as f:
            f.write(wkt_descriptor_set())
        tmp_out = os.path.join(td, "out.desc")
        cmd = [
            protoc,
            f"--proto_path={PROTO_DIR}",
            f"--descriptor_set_in={wkt}",
            f"--descriptor_set_out={tmp_out}",
            "tf_core.proto",
            "serving_apis.proto",
        ]
        subprocess.run(cmd, check=True)
        with open(tmp_out, "rb") as f:
            data = f.read()
    with open(out_path, "wb") as f:
        f.write(data)
    return out_path


if __name__ == "__main__":
    print(generate(sys.argv[1] if len(sys.argv) > 1 else OUT))
