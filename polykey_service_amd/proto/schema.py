"""Wire schema for the polykey gRPC surface, built from descriptors at import time.

The reference (`/root/reference`) compiles against the external module
``github.com/spounge-ai/spounge-proto/gen/go v1.2.0`` (``go.mod:6``) which is not
vendored.  Message and field *names* are reconstructed from their Go usage
(SURVEY.md §2.2):

* ``ExecuteToolRequest``  — ``internal/server/server.go:29-32``, ``cmd/dev_client/main.go:246-258``
* ``ExecuteToolResponse`` — ``internal/service/mock.go:24-64``
* ``common.v2.{Status,Metadata,File}`` — ``mock.go:26,54``, ``dev_client/main.go:252``

Field numbers are ours (the upstream ones are unknown).  ``protoc`` is not available,
so ``FileDescriptorProto`` objects are assembled here with ``descriptor_pb2`` and
registered in the default pool; the same serialized descriptors feed the
reflection service (``server/reflection.py``).

New relative to the reference: ``ExecuteToolStream`` (server streaming) on the same
service, plus hand-built ``grpc.health.v1`` and ``grpc.reflection.v1alpha``/``v1``
schemas (the python ``grpcio-health-checking``/``grpcio-reflection`` packages are not
installed).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
from google.protobuf import struct_pb2  # noqa: F401  (registers google/protobuf/struct.proto)

F = descriptor_pb2.FieldDescriptorProto

_TYPES = {
    "string": F.TYPE_STRING,
    "bytes": F.TYPE_BYTES,
    "int32": F.TYPE_INT32,
    "int64": F.TYPE_INT64,
    "uint32": F.TYPE_UINT32,
    "bool": F.TYPE_BOOL,
    "double": F.TYPE_DOUBLE,
    "float": F.TYPE_FLOAT,
}


class _Field:
    __slots__ = ("name", "number", "type", "label", "oneof", "proto3_optional")

    def __init__(self, name, number, type_, label="optional", oneof=None, proto3_optional=False):
        self.name = name
        self.number = number
        self.type = type_
        self.label = label
        self.oneof = oneof
        self.proto3_optional = proto3_optional


def field(name, number, type_, *, repeated=False, oneof=None, optional=False) -> _Field:
    return _Field(name, number, type_, "repeated" if repeated else "optional", oneof, optional)


def _add_message(container, pkg: str, name: str, fields: Sequence[_Field],
                 enums: Sequence[Tuple[str, Sequence[Tuple[str, int]]]] = (),
                 nested: Sequence = ()) -> descriptor_pb2.DescriptorProto:
    msg = container.add()
    msg.name = name
    for ename, values in enums:
        e = msg.enum_type.add()
        e.name = ename
        for vname, vnum in values:
            v = e.value.add()
            v.name = vname
            v.number = vnum
    for nested_args in nested:
        _add_message(msg.nested_type, pkg, *nested_args)
    oneof_index: Dict[str, int] = {}
    synthetic: List[Tuple[_Field, descriptor_pb2.FieldDescriptorProto]] = []
    for f in fields:
        fd = msg.field.add()
        fd.name = f.name
        fd.number = f.number
        fd.json_name = _json_name(f.name)
        fd.label = F.LABEL_REPEATED if f.label == "repeated" else F.LABEL_OPTIONAL
        if f.type in _TYPES:
            fd.type = _TYPES[f.type]
        elif f.type.startswith("enum:"):
            fd.type = F.TYPE_ENUM
            fd.type_name = f.type[len("enum:"):]
        else:
            fd.type = F.TYPE_MESSAGE
            fd.type_name = f.type
        if f.oneof is not None:
            if f.oneof not in oneof_index:
                oneof_index[f.oneof] = len(msg.oneof_decl)
                msg.oneof_decl.add().name = f.oneof
            fd.oneof_index = oneof_index[f.oneof]
        if f.proto3_optional:
            synthetic.append((f, fd))
    # proto3 `optional` = synthetic oneof named _<field>, declared after real oneofs.
    for f, fd in synthetic:
        fd.proto3_optional = True
        fd.oneof_index = len(msg.oneof_decl)
        msg.oneof_decl.add().name = "_" + f.name
    return msg


def _json_name(name: str) -> str:
    parts = name.split("_")
    return parts[0] + "".join(p[:1].upper() + p[1:] for p in parts[1:])


def _add_service(fdp, name: str, methods: Sequence[Tuple[str, str, str, bool, bool]]):
    svc = fdp.service.add()
    svc.name = name
    for mname, inp, out, cstream, sstream in methods:
        m = svc.method.add()
        m.name = mname
        m.input_type = inp
        m.output_type = out
        if cstream:
            m.client_streaming = True
        if sstream:
            m.server_streaming = True


def _file(name: str, package: str, deps: Sequence[str] = ()) -> descriptor_pb2.FileDescriptorProto:
    fdp = descriptor_pb2.FileDescriptorProto()
    fdp.name = name
    fdp.package = package
    fdp.syntax = "proto3"
    fdp.dependency.extend(deps)
    return fdp


# --------------------------------------------------------------------------- common.v2
def _build_common() -> descriptor_pb2.FileDescriptorProto:
    fdp = _file("common/v2/common.proto", "common.v2")
    _add_message(fdp.message_type, "common.v2", "Status", [
        field("code", 1, "int32"),
        field("message", 2, "string"),
    ])
    # map<string,string> fields = 1  → nested FieldsEntry with map_entry option.
    md = _add_message(fdp.message_type, "common.v2", "Metadata", [
        field("fields", 1, ".common.v2.Metadata.FieldsEntry", repeated=True),
    ], nested=[("FieldsEntry", [field("key", 1, "string"), field("value", 2, "string")])])
    md.nested_type[0].options.map_entry = True
    _add_message(fdp.message_type, "common.v2", "File", [
        field("file_name", 1, "string"),
        field("mime_type", 2, "string"),
        field("content", 3, "bytes"),
    ])
    return fdp


# -------------------------------------------------------------------------- polykey.v2
def _build_polykey() -> descriptor_pb2.FileDescriptorProto:
    fdp = _file("polykey/v2/polykey.proto", "polykey.v2",
                ["google/protobuf/struct.proto", "common/v2/common.proto"])
    _add_message(fdp.message_type, "polykey.v2", "ExecuteToolRequest", [
        field("tool_name", 1, "string"),
        field("parameters", 2, ".google.protobuf.Struct"),
        field("secret_id", 3, "string", optional=True),
        field("metadata", 4, ".common.v2.Metadata"),
    ])
    _add_message(fdp.message_type, "polykey.v2", "ExecuteToolResponse", [
        field("status", 1, ".common.v2.Status"),
        field("string_output", 2, "string", oneof="output"),
        field("struct_output", 3, ".google.protobuf.Struct", oneof="output"),
        field("file_output", 4, ".common.v2.File", oneof="output"),
    ])
    _add_service(fdp, "PolykeyService", [
        ("ExecuteTool", ".polykey.v2.ExecuteToolRequest", ".polykey.v2.ExecuteToolResponse", False, False),
        # [NEW] incremental string_output chunks, final struct_output with usage.
        ("ExecuteToolStream", ".polykey.v2.ExecuteToolRequest", ".polykey.v2.ExecuteToolResponse", False, True),
    ])
    return fdp


# ---------------------------------------------------------------------- grpc.health.v1
def _build_health() -> descriptor_pb2.FileDescriptorProto:
    fdp = _file("grpc/health/v1/health.proto", "grpc.health.v1")
    _add_message(fdp.message_type, "grpc.health.v1", "HealthCheckRequest", [field("service", 1, "string")])
    _add_message(fdp.message_type, "grpc.health.v1", "HealthCheckResponse",
                 [field("status", 1, "enum:.grpc.health.v1.HealthCheckResponse.ServingStatus")],
                 enums=[("ServingStatus", [("UNKNOWN", 0), ("SERVING", 1), ("NOT_SERVING", 2),
                                           ("SERVICE_UNKNOWN", 3)])])
    _add_service(fdp, "Health", [
        ("Check", ".grpc.health.v1.HealthCheckRequest", ".grpc.health.v1.HealthCheckResponse", False, False),
        ("Watch", ".grpc.health.v1.HealthCheckRequest", ".grpc.health.v1.HealthCheckResponse", False, True),
    ])
    return fdp


# ------------------------------------------------------------------ grpc.reflection.*
def _build_reflection(version: str) -> descriptor_pb2.FileDescriptorProto:
    pkg = f"grpc.reflection.{version}"
    p = "." + pkg + "."
    fdp = _file(f"grpc/reflection/{version}/reflection.proto", pkg)
    m = fdp.message_type
    _add_message(m, pkg, "ServerReflectionRequest", [
        field("host", 1, "string"),
        field("file_by_filename", 3, "string", oneof="message_request"),
        field("file_containing_symbol", 4, "string", oneof="message_request"),
        field("file_containing_extension", 5, p + "ExtensionRequest", oneof="message_request"),
        field("all_extension_numbers_of_type", 6, "string", oneof="message_request"),
        field("list_services", 7, "string", oneof="message_request"),
    ])
    _add_message(m, pkg, "ExtensionRequest", [
        field("containing_type", 1, "string"), field("extension_number", 2, "int32")])
    _add_message(m, pkg, "ServerReflectionResponse", [
        field("valid_host", 1, "string"),
        field("original_request", 2, p + "ServerReflectionRequest"),
        field("file_descriptor_response", 4, p + "FileDescriptorResponse", oneof="message_response"),
        field("all_extension_numbers_response", 5, p + "ExtensionNumberResponse", oneof="message_response"),
        field("list_services_response", 6, p + "ListServiceResponse", oneof="message_response"),
        field("error_response", 7, p + "ErrorResponse", oneof="message_response"),
    ])
    _add_message(m, pkg, "FileDescriptorResponse", [field("file_descriptor_proto", 1, "bytes", repeated=True)])
    _add_message(m, pkg, "ExtensionNumberResponse", [
        field("base_type_name", 1, "string"), field("extension_number", 2, "int32", repeated=True)])
    _add_message(m, pkg, "ListServiceResponse", [field("service", 1, p + "ServiceResponse", repeated=True)])
    _add_message(m, pkg, "ServiceResponse", [field("name", 1, "string")])
    _add_message(m, pkg, "ErrorResponse", [field("error_code", 1, "int32"), field("error_message", 2, "string")])
    _add_service(fdp, "ServerReflection", [
        ("ServerReflectionInfo", p + "ServerReflectionRequest", p + "ServerReflectionResponse", True, True),
    ])
    return fdp


POOL = descriptor_pool.Default()
FILES: Dict[str, descriptor_pb2.FileDescriptorProto] = {}


def _register(fdp: descriptor_pb2.FileDescriptorProto) -> None:
    try:
        POOL.FindFileByName(fdp.name)
    except KeyError:
        POOL.AddSerializedFile(fdp.SerializeToString())
    FILES[fdp.name] = fdp


for _fdp in (_build_common(), _build_polykey(), _build_health(),
             _build_reflection("v1alpha"), _build_reflection("v1")):
    _register(_fdp)


def message_class(full_name: str):
    return message_factory.GetMessageClass(POOL.FindMessageTypeByName(full_name))


def serialized_file(name: str) -> bytes:
    """Serialized FileDescriptorProto for `name` (ours or a well-known type)."""
    if name in FILES:
        return FILES[name].SerializeToString()
    fd = POOL.FindFileByName(name)
    out = descriptor_pb2.FileDescriptorProto()
    fd.CopyToProto(out)
    return out.SerializeToString()


def file_dependencies(name: str) -> List[str]:
    return list(POOL.FindFileByName(name).dependencies and
                [d.name for d in POOL.FindFileByName(name).dependencies])


def file_containing_symbol(symbol: str) -> Optional[str]:
    for finder in (POOL.FindServiceByName, POOL.FindMessageTypeByName, POOL.FindEnumTypeByName):
        try:
            return finder(symbol).file.name
        except KeyError:
            pass
    # method symbol: pkg.Service.Method
    if "." in symbol:
        svc, _, _meth = symbol.rpartition(".")
        try:
            return POOL.FindServiceByName(svc).file.name
        except KeyError:
            return None
    return None
