"""Message classes for polykey.v2 / common.v2 / grpc.health.v1 / grpc.reflection.

See :mod:`polykey_service_amd.proto.schema` for how these are built and how the
field names map to the reference's Go usage.
"""
from google.protobuf import struct_pb2
from google.protobuf.json_format import MessageToDict

from . import schema
from .schema import message_class

Struct = struct_pb2.Struct
Value = struct_pb2.Value

Status = message_class("common.v2.Status")
Metadata = message_class("common.v2.Metadata")
File = message_class("common.v2.File")

ExecuteToolRequest = message_class("polykey.v2.ExecuteToolRequest")
ExecuteToolResponse = message_class("polykey.v2.ExecuteToolResponse")

HealthCheckRequest = message_class("grpc.health.v1.HealthCheckRequest")
HealthCheckResponse = message_class("grpc.health.v1.HealthCheckResponse")

POLYKEY_SERVICE = "polykey.v2.PolykeyService"
HEALTH_SERVICE = "grpc.health.v1.Health"
REFLECTION_SERVICES = ("grpc.reflection.v1alpha.ServerReflection", "grpc.reflection.v1.ServerReflection")

EXECUTE_TOOL = f"/{POLYKEY_SERVICE}/ExecuteTool"
EXECUTE_TOOL_STREAM = f"/{POLYKEY_SERVICE}/ExecuteToolStream"
HEALTH_CHECK = f"/{HEALTH_SERVICE}/Check"
HEALTH_WATCH = f"/{HEALTH_SERVICE}/Watch"


def struct_from_dict(d) -> "Struct":
    s = Struct()
    if d:
        s.update(d)
    return s


def struct_to_dict(s) -> dict:
    if s is None:
        return {}
    return MessageToDict(s)


__all__ = [
    "schema", "Struct", "Value", "Status", "Metadata", "File", "ExecuteToolRequest",
    "ExecuteToolResponse", "HealthCheckRequest", "HealthCheckResponse", "POLYKEY_SERVICE",
    "HEALTH_SERVICE", "REFLECTION_SERVICES", "EXECUTE_TOOL", "EXECUTE_TOOL_STREAM",
    "HEALTH_CHECK", "HEALTH_WATCH", "struct_from_dict", "struct_to_dict",
]
