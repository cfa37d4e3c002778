"""Development client (reference ``cmd/dev_client/main.go``).

Flow (``main.go:107-165``): DEBUG JSON logs into an in-memory buffer → load config
(flags/env/auto-detect) → ``"Configuration loaded" {runtime, server}`` → TCP pre-flight
(3 s) → gRPC channel (insecure; keepalive 10 s / 5 s, permit without stream; 4 MiB
messages) → wait for READY, failing fast on TRANSIENT_FAILURE/SHUTDOWN, bounded by the
config timeout → one ``ExecuteTool`` of ``example_tool`` with the reference's parameters,
secret id and metadata under a 30 s deadline → Jest-style report of the buffered log.

Differences: the process exits 1 when the run failed (the reference always exits 0, SURVEY.md
§2.5 #11), and extra flags select another tool / streaming / an LLM prompt:
``-tool NAME -stream -prompt TEXT -max-tokens N``.
"""
from __future__ import annotations

import os
import signal
import sys
import threading
import time
from typing import Optional

import grpc

from .. import proto
from ..config import ConfigLoader, NetworkTester
from ..report.jest import print_jest_report
from ..server.interceptors import GO_CODE
from ..utils import slog

MIB = 1024 * 1024
CHANNEL_OPTIONS = [
    ("grpc.keepalive_time_ms", 10_000),
    ("grpc.keepalive_timeout_ms", 5_000),
    ("grpc.keepalive_permit_without_calls", 1),
    ("grpc.max_receive_message_length", 4 * MIB),
    ("grpc.max_send_message_length", 4 * MIB),
]


def truncate(s: str, n: int) -> str:
    return s if len(s) <= n else s[:n] + "..."


class Client:
    def __init__(self, channel: grpc.Channel, logger: slog.Logger):
        self.channel = channel
        self.logger = logger
        self._unary = channel.unary_unary(proto.EXECUTE_TOOL,
                                          request_serializer=proto.ExecuteToolRequest.SerializeToString,
                                          response_deserializer=proto.ExecuteToolResponse.FromString)
        self._stream = channel.unary_stream(proto.EXECUTE_TOOL_STREAM,
                                            request_serializer=proto.ExecuteToolRequest.SerializeToString,
                                            response_deserializer=proto.ExecuteToolResponse.FromString)

    def close(self) -> None:
        self.channel.close()

    def _log_call(self, req) -> None:
        self.logger.info("Executing tool", tool_name=req.tool_name,
                         secret_id=req.secret_id if req.HasField("secret_id") else None,
                         has_metadata=req.HasField("metadata"))

    def _log_rpc_error(self, e: grpc.RpcError) -> None:
        code = e.code() if hasattr(e, "code") else None
        self.logger.error("gRPC call failed", code=GO_CODE.get(code.name, "Unknown") if code else "Unknown",
                          message=e.details() if hasattr(e, "details") else str(e), details=[])

    def execute_tool(self, req, timeout: Optional[float] = None):
        self._log_call(req)
        try:
            resp = self._unary(req, timeout=timeout)
        except grpc.RpcError as e:
            self._log_rpc_error(e)
            raise RuntimeError(f"ExecuteTool failed: {e.details() if hasattr(e, 'details') else e}") from e
        self.log_response(resp)
        return resp

    def execute_tool_stream(self, req, timeout: Optional[float] = None):
        self._log_call(req)
        last = None
        try:
            for chunk in self._stream(req, timeout=timeout):
                last = chunk
                yield chunk
        except grpc.RpcError as e:
            self._log_rpc_error(e)
            raise RuntimeError(f"ExecuteToolStream failed: {e.details() if hasattr(e, 'details') else e}") from e
        if last is not None:
            self.log_response(last)

    def log_response(self, resp) -> None:
        if resp.HasField("status"):
            self.logger.info("Tool execution completed", status_code=resp.status.code,
                             status_message=resp.status.message)
        kind = resp.WhichOneof("output")
        if kind == "string_output":
            self.logger.info("Received string output", output_length=len(resp.string_output),
                             output_preview=truncate(resp.string_output, 100))
        elif kind == "struct_output":
            self.logger.info("Received struct output", field_count=len(resp.struct_output.fields))
        elif kind == "file_output":
            f = resp.file_output
            self.logger.info("Received file output", file_name=f.file_name, mime_type=f.mime_type,
                             size_bytes=len(f.content))
        else:
            self.logger.warn("No output returned")


def wait_for_connection(channel: grpc.Channel, timeout: float, logger: slog.Logger) -> None:
    """``waitForConnection`` (``main.go:214-236``): READY or fail."""
    C = grpc.ChannelConnectivity
    cond = threading.Condition()
    states = []

    def cb(state):
        with cond:
            states.append(state)
            cond.notify_all()

    channel.subscribe(cb, try_to_connect=True)
    try:
        deadline = time.monotonic() + timeout
        seen = 0
        with cond:
            while True:
                while seen < len(states):
                    st = states[seen]
                    seen += 1
                    if seen == 1:
                        logger.debug("Initial connection state", state=_state_name(st))
                    else:
                        logger.debug("Connection state changed", state=_state_name(st))
                    if st == C.READY:
                        return
                    if seen > 1 and st in (C.TRANSIENT_FAILURE, C.SHUTDOWN):
                        raise ConnectionError(f"connection failed with state: {_state_name(st)}")
                remaining = deadline - time.monotonic()
                if remaining <= 0:
                    raise TimeoutError("connection timeout")
                cond.wait(remaining)
    finally:
        channel.unsubscribe(cb)


def _state_name(st) -> str:
    return st.name if hasattr(st, "name") else str(st)


def create_connection(address: str, timeout: float, logger: slog.Logger, tls_ca: str = "") -> grpc.Channel:
    """Insecure channel as in the reference; ``tls_ca`` (or env ``POLYKEY_TLS_CA``): a PEM root
    certificate to verify a TLS server with instead."""
    logger.info("Creating gRPC connection", server=address)
    tls_ca = tls_ca or os.environ.get("POLYKEY_TLS_CA", "")
    if tls_ca:
        with open(tls_ca, "rb") as f:
            creds = grpc.ssl_channel_credentials(root_certificates=f.read())
        ch = grpc.secure_channel(address, creds, options=CHANNEL_OPTIONS)
    else:
        ch = grpc.insecure_channel(address, options=CHANNEL_OPTIONS)
    try:
        wait_for_connection(ch, timeout, logger)
    except Exception as e:
        ch.close()
        raise ConnectionError(f"connection failed: {e}") from e
    logger.info("gRPC connection established successfully")
    return ch


def build_request(tool_name: str = "example_tool", extra_params: Optional[dict] = None):
    """The reference's test request (``main.go:238-258``)."""
    params = {"example_param": "value", "timestamp": int(time.time())}
    if extra_params:
        params.update(extra_params)
    req = proto.ExecuteToolRequest(tool_name=tool_name, secret_id="secret-123")
    req.parameters.update(params)
    req.metadata.fields.update({
        "client_version": "1.0.0",
        "request_source": "dev_client",
        "request_id": f"req-{time.time_ns()}",
    })
    return req


def _extra_flags(fs) -> None:
    fs.string("tool", "example_tool", "tool to execute")
    fs.bool("stream", False, "use ExecuteToolStream")
    fs.string("prompt", "", "prompt for llm.* tools")
    fs.int("max-tokens", 32, "max new tokens for llm.* tools")


def run(logger: slog.Logger, argv=None, cancel: Optional[threading.Event] = None) -> None:
    logger.info("Starting polykey client...")
    loader = ConfigLoader()
    cfg = loader.load(argv, define_extra=_extra_flags)
    logger.info("Configuration loaded", runtime=str(loader.detector.detect_runtime()), server=cfg.server_address)

    logger.info("Testing network connectivity...")
    try:
        NetworkTester().test_connection(cfg.server_address)
    except ConnectionError as e:
        raise RuntimeError(f"network test failed: {e}") from e
    logger.info("Network connectivity test passed")

    try:
        channel = create_connection(cfg.server_address, cfg.timeout, logger)
    except ConnectionError as e:
        raise RuntimeError(f"failed to create client: failed to create gRPC connection: {e}") from e
    client = Client(channel, logger)
    try:
        ex = cfg.extras
        extra = {}
        if ex.get("prompt"):
            extra = {"prompt": ex["prompt"], "max_tokens": ex.get("max-tokens", 32)}
        req = build_request(ex.get("tool", "example_tool"), extra)
        if ex.get("stream"):
            resp = None
            for resp in client.execute_tool_stream(req, timeout=30.0):
                if cancel is not None and cancel.is_set():
                    break
        else:
            resp = client.execute_tool(req, timeout=30.0)
        if resp is not None and not resp.HasField("status"):
            logger.warn("Response missing status field")
    except RuntimeError as e:
        raise RuntimeError(f"test request failed: {e}") from e
    finally:
        client.close()


def main(argv=None, out=None) -> int:
    logger = slog.BufferLogger(level=slog.DEBUG)
    cancel = threading.Event()

    def on_signal(signum, frame):
        logger.info("Received shutdown signal")
        cancel.set()

    try:
        signal.signal(signal.SIGINT, on_signal)
        signal.signal(signal.SIGTERM, on_signal)
    except ValueError:
        pass  # not main thread
    failed = False
    try:
        run(logger, argv, cancel)
    except Exception as e:  # noqa: BLE001
        logger.error("Application failed", error=str(e))
        failed = True
    fails = print_jest_report(logger.lines(), out=out)
    return 1 if (failed or fails) else 0


if __name__ == "__main__":
    sys.exit(main())
