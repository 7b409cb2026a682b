"""Message classes for the serving API, built from the committed descriptor set.

The classes live in a private ``DescriptorPool`` so that they never collide with
another copy of ``tensorflow.TensorProto`` (tensorboard registers one in the
default pool). Usage::

    from distributed_tf_serving_amd.wire import schema as pb
    req = pb.PredictRequest()
    req.model_spec.name = "DCN"

Mirrors what protoc-generated Java gives the reference client
(``Predict.PredictRequest``, ``Model.ModelSpec``, ``TensorProto``...;
reference DCNClient.java:83-115).
"""
from __future__ import annotations

import os

from google.protobuf import any_pb2, descriptor_pb2, descriptor_pool, message_factory, wrappers_pb2

_DESC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "serving_apis.desc")

POOL = descriptor_pool.DescriptorPool()


def _load_pool() -> None:
    for mod in (any_pb2, wrappers_pb2):
        fdp = descriptor_pb2.FileDescriptorProto()
        mod.DESCRIPTOR.CopyToProto(fdp)
        POOL.Add(fdp)
    if not os.path.exists(_DESC):  # dev checkout without the generated blob
        from .gen_descriptors import generate

        generate(_DESC)
    fds = descriptor_pb2.FileDescriptorSet()
    with open(_DESC, "rb") as f:
        fds.ParseFromString(f.read())
    for fdp in fds.file:
        if fdp.name.startswith("google/protobuf/"):
            continue
        POOL.Add(fdp)


_load_pool()


def message_class(full_name: str):
    return message_factory.GetMessageClass(POOL.FindMessageTypeByName(full_name))


# --- tensorflow core -------------------------------------------------------
TensorProto = message_class("tensorflow.TensorProto")
TensorShapeProto = message_class("tensorflow.TensorShapeProto")
Example = message_class("tensorflow.Example")
Features = message_class("tensorflow.Features")
Feature = message_class("tensorflow.Feature")
TensorInfo = message_class("tensorflow.TensorInfo")
SignatureDef = message_class("tensorflow.SignatureDef")
_dt = POOL.FindEnumTypeByName("tensorflow.DataType")
DataType = {v.name: v.number for v in _dt.values}
DataTypeName = {v.number: v.name for v in _dt.values}
DT_FLOAT = DataType["DT_FLOAT"]
DT_DOUBLE = DataType["DT_DOUBLE"]
DT_INT32 = DataType["DT_INT32"]
DT_INT64 = DataType["DT_INT64"]
DT_BOOL = DataType["DT_BOOL"]
DT_HALF = DataType["DT_HALF"]
DT_BFLOAT16 = DataType["DT_BFLOAT16"]
DT_STRING = DataType["DT_STRING"]
DT_UINT8 = DataType["DT_UINT8"]
DT_INT8 = DataType["DT_INT8"]
DT_INT16 = DataType["DT_INT16"]
DT_UINT16 = DataType["DT_UINT16"]
DT_UINT32 = DataType["DT_UINT32"]
DT_UINT64 = DataType["DT_UINT64"]

# --- tensorflow.serving ----------------------------------------------------
ModelSpec = message_class("tensorflow.serving.ModelSpec")
PredictRequest = message_class("tensorflow.serving.PredictRequest")
PredictResponse = message_class("tensorflow.serving.PredictResponse")
Input = message_class("tensorflow.serving.Input")
ExampleList = message_class("tensorflow.serving.ExampleList")
ExampleListWithContext = message_class("tensorflow.serving.ExampleListWithContext")
ClassificationRequest = message_class("tensorflow.serving.ClassificationRequest")
ClassificationResponse = message_class("tensorflow.serving.ClassificationResponse")
RegressionRequest = message_class("tensorflow.serving.RegressionRequest")
RegressionResponse = message_class("tensorflow.serving.RegressionResponse")
InferenceTask = message_class("tensorflow.serving.InferenceTask")
MultiInferenceRequest = message_class("tensorflow.serving.MultiInferenceRequest")
MultiInferenceResponse = message_class("tensorflow.serving.MultiInferenceResponse")
SignatureDefMap = message_class("tensorflow.serving.SignatureDefMap")
GetModelMetadataRequest = message_class("tensorflow.serving.GetModelMetadataRequest")
GetModelMetadataResponse = message_class("tensorflow.serving.GetModelMetadataResponse")
Any = message_class("google.protobuf.Any")
Int64Value = message_class("google.protobuf.Int64Value")

SERVICE = POOL.FindServiceByName("tensorflow.serving.PredictionService")
SERVICE_NAME = SERVICE.full_name
#: method name -> (request class, response class)
METHODS = {
    m.name: (
        message_factory.GetMessageClass(m.input_type),
        message_factory.GetMessageClass(m.output_type),
    )
    for m in SERVICE.methods
}
