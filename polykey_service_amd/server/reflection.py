"""gRPC server reflection (``grpc.reflection.v1alpha`` and ``v1``), hand-built.

Reference: ``reflection.Register(srv)`` (``cmd/polykey/main.go:80``) so ``grpcurl`` can list
and describe the service.  Descriptors come from :mod:`polykey_service_amd.proto.schema`,
the same ones the message classes are built from.
"""
from __future__ import annotations

from typing import Iterable, List, Set

import grpc

from ..proto import schema


class ReflectionServicer:
    def __init__(self, service_names: Iterable[str], version: str = "v1alpha"):
        self.service_names = sorted(set(service_names))
        self.version = version
        pkg = f"grpc.reflection.{version}"
        self.Req = schema.message_class(pkg + ".ServerReflectionRequest")
        self.Resp = schema.message_class(pkg + ".ServerReflectionResponse")
        self.full_name = pkg + ".ServerReflection"

    def _files_with_deps(self, name: str) -> List[bytes]:
        out: List[bytes] = []
        seen: Set[str] = set()

        def visit(fname: str):
            if fname in seen:
                return
            seen.add(fname)
            out.append(schema.serialized_file(fname))
            fd = schema.POOL.FindFileByName(fname)
            for dep in fd.dependencies:
                visit(dep.name)

        visit(name)
        return out

    def _answer(self, req):
        resp = self.Resp(valid_host=req.host)
        resp.original_request.CopyFrom(req)
        kind = req.WhichOneof("message_request")
        try:
            if kind == "list_services":
                for n in self.service_names:
                    resp.list_services_response.service.add(name=n)
            elif kind == "file_by_filename":
                resp.file_descriptor_response.file_descriptor_proto.extend(
                    self._files_with_deps(req.file_by_filename))
            elif kind == "file_containing_symbol":
                fname = schema.file_containing_symbol(req.file_containing_symbol)
                if fname is None:
                    raise KeyError(req.file_containing_symbol)
                resp.file_descriptor_response.file_descriptor_proto.extend(self._files_with_deps(fname))
            elif kind == "all_extension_numbers_of_type":
                schema.POOL.FindMessageTypeByName(req.all_extension_numbers_of_type)
                resp.all_extension_numbers_response.base_type_name = req.all_extension_numbers_of_type
            else:  # file_containing_extension or unset: we register no extensions
                resp.error_response.error_code = grpc.StatusCode.NOT_FOUND.value[0]
                resp.error_response.error_message = "extensions are not supported"
        except KeyError:
            resp.ClearField("file_descriptor_response")
            resp.error_response.error_code = grpc.StatusCode.NOT_FOUND.value[0]
            resp.error_response.error_message = "not found"
        return resp

    async def ServerReflectionInfo(self, request_iterator, context):
        async for req in request_iterator:
            yield self._answer(req)

    def handler(self) -> grpc.GenericRpcHandler:
        return grpc.method_handlers_generic_handler(self.full_name, {
            "ServerReflectionInfo": grpc.stream_stream_rpc_method_handler(
                self.ServerReflectionInfo, request_deserializer=self.Req.FromString,
                response_serializer=self.Resp.SerializeToString),
        })
