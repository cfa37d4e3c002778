"""``grpc_health_probe`` equivalent (the reference's image ships that Go binary for its
Docker / compose health checks: ``/root/reference/compose.yml:17-23``,
``/root/reference/.github/workflows/ci.yml:108-113``).

    python3 -m polykey_service_amd.client.health_probe -addr=:50051 [-service=NAME] [-connect-timeout=5s]

Exit status as grpc_health_probe's: 0 SERVING, 1 invalid flags, 2 connection failure, 3 RPC
failure (e.g. unknown service), 4 not SERVING.
"""
from __future__ import annotations

import sys
from typing import List, Optional

import grpc

from .. import proto
from ..utils.slog import parse_go_duration as parse_duration


def probe(addr: str, service: str = "", timeout_s: float = 5.0) -> int:
    if addr.startswith(":"):
        addr = "127.0.0.1" + addr
    with grpc.insecure_channel(addr) as ch:
        try:
            grpc.channel_ready_future(ch).result(timeout=timeout_s)
        except grpc.FutureTimeoutError:
            print(f"error: failed to connect service at {addr!r}", file=sys.stderr)
            return 2
        check = ch.unary_unary(proto.HEALTH_CHECK, request_serializer=proto.HealthCheckRequest.SerializeToString,
                               response_deserializer=proto.HealthCheckResponse.FromString)
        try:
            r = check(proto.HealthCheckRequest(service=service), timeout=timeout_s)
        except grpc.RpcError as e:
            print(f"error: health rpc failed: {e.code().name}: {e.details()}", file=sys.stderr)
            return 3
    if r.status != 1:  # SERVING
        print(f"service unhealthy (responded with {proto.HealthCheckResponse.ServingStatus.Name(r.status)})",
              file=sys.stderr)
        return 4
    print("status: SERVING")
    return 0


def main(argv: Optional[List[str]] = None) -> int:
    addr, service, timeout_s = "", "", 5.0
    for a in (sys.argv[1:] if argv is None else argv):
        k, _, v = a.lstrip("-").partition("=")
        if k == "addr":
            addr = v
        elif k == "service":
            service = v
        elif k in ("connect-timeout", "rpc-timeout"):
            timeout_s = parse_duration(v)
        else:
            print(f"unknown flag {a}", file=sys.stderr)
            return 1
    if not addr:
        print("-addr is required", file=sys.stderr)
        return 1
    return probe(addr, service, timeout_s)


if __name__ == "__main__":
    sys.exit(main())
