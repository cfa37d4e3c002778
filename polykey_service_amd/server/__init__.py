from .app import SERVER_OPTIONS, PolykeyServer, amain, build_service, grpc_bind_address, main
from .health import NOT_SERVING, SERVICE_UNKNOWN, SERVING, HealthServicer
from .interceptors import GO_CODE, LoggingInterceptor
from .reflection import ReflectionServicer
from .rpc import SERVICE_METHODS, PolykeyServicer

__all__ = ["SERVER_OPTIONS", "PolykeyServer", "amain", "build_service", "grpc_bind_address", "main",
           "NOT_SERVING", "SERVICE_UNKNOWN", "SERVING", "HealthServicer", "GO_CODE", "LoggingInterceptor",
           "ReflectionServicer", "SERVICE_METHODS", "PolykeyServicer"]
