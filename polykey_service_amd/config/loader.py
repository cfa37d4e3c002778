"""Client configuration loader (reference ``internal/config/config.go:14-240``).

Precedence (``config.go:156-175``): defaults < flags < environment < auto-detect (the
last only when the address is still empty).

* defaults: ``Timeout=5s, LogLevel="info", Environment="development"`` (``config.go:157-161``)
* flags: ``-server -timeout -log-level -env`` (``config.go:177-183``)
* env: ``POLYKEY_SERVER_ADDR``, ``POLYKEY_TIMEOUT`` (Go duration; silently ignored when
  invalid), ``POLYKEY_LOG_LEVEL``, ``POLYKEY_ENV`` (``config.go:185-203``)
* auto-detect (``config.go:134-154``): Kubernetes → ``polykey-service:50051``;
  Docker/containerd/Podman → ``polykey-server:50051``; local → ``localhost:50051``.

Deliberate differences: the flag set is local, not global (#12), and the
local branch skips the reference's ``isDockerHostReachable`` probe by default because both
of its outcomes return ``localhost:50051`` (#15); ``probe_docker_host=True`` restores it.
"""
from __future__ import annotations

import dataclasses
import os
import socket
import sys
from typing import Mapping, Optional, Sequence

from ..utils.slog import parse_go_duration
from .goflag import FlagSet
from .runtime import RuntimeDetector, RuntimeEnvironment

DEFAULT_PORT = 50051


@dataclasses.dataclass
class Config:
    server_address: str = ""
    timeout: float = 5.0  # seconds
    log_level: str = "info"
    environment: str = "development"
    extras: dict = dataclasses.field(default_factory=dict)


class ConfigLoader:
    def __init__(self, detector: Optional[RuntimeDetector] = None,
                 environ: Optional[Mapping[str, str]] = None, probe_docker_host: bool = False):
        self.environ = os.environ if environ is None else environ
        self.detector = detector or RuntimeDetector(environ=self.environ)
        self.probe_docker_host = probe_docker_host

    def load(self, argv: Optional[Sequence[str]] = None, define_extra=None) -> Config:
        """``define_extra(flagset)`` may register additional flags (e.g. the dev client's
        ``-tool``); their parsed values land in ``Config.extras``."""
        cfg = Config()
        self._load_from_flags(cfg, sys.argv[1:] if argv is None else argv, define_extra)
        self._load_from_env(cfg)
        if cfg.server_address == "":
            cfg.server_address = self.detect_server_address()
        return cfg

    def _load_from_flags(self, cfg: Config, argv: Sequence[str], define_extra=None) -> FlagSet:
        fs = FlagSet("dev_client")
        fs.string("server", "", "gRPC server address")
        fs.duration("timeout", cfg.timeout, "Connection timeout")
        fs.string("log-level", cfg.log_level, "Log level")
        fs.string("env", cfg.environment, "Environment")
        base = set(fs.values)
        if define_extra is not None:
            define_extra(fs)
        fs.parse(argv)
        cfg.extras = {k: v for k, v in fs.values.items() if k not in base}
        cfg.server_address = fs["server"]
        cfg.timeout = fs["timeout"]
        cfg.log_level = fs["log-level"]
        cfg.environment = fs["env"]
        return fs

    def _load_from_env(self, cfg: Config) -> None:
        env = self.environ
        if env.get("POLYKEY_SERVER_ADDR", ""):
            cfg.server_address = env["POLYKEY_SERVER_ADDR"]
        if env.get("POLYKEY_TIMEOUT", ""):
            try:
                cfg.timeout = parse_go_duration(env["POLYKEY_TIMEOUT"])
            except ValueError:
                pass  # config.go:191-195: invalid durations are ignored
        if env.get("POLYKEY_LOG_LEVEL", ""):
            cfg.log_level = env["POLYKEY_LOG_LEVEL"]
        if env.get("POLYKEY_ENV", ""):
            cfg.environment = env["POLYKEY_ENV"]

    def detect_server_address(self) -> str:
        rt = self.detector.detect_runtime()
        if rt == RuntimeEnvironment.KUBERNETES:
            return f"polykey-service:{DEFAULT_PORT}"
        if rt in (RuntimeEnvironment.DOCKER, RuntimeEnvironment.CONTAINERD, RuntimeEnvironment.PODMAN):
            return f"polykey-server:{DEFAULT_PORT}"
        if self.probe_docker_host:
            self.is_docker_host_reachable()
        return f"localhost:{DEFAULT_PORT}"

    def is_docker_host_reachable(self, timeout: float = 2.0) -> bool:
        for addr in (f"host.docker.internal:{DEFAULT_PORT}", f"localhost:{DEFAULT_PORT}"):
            host, port = addr.rsplit(":", 1)
            try:
                with socket.create_connection((host, int(port)), timeout=timeout):
                    return True
            except OSError:
                continue
        return False


class NetworkTester:
    """TCP pre-flight dial, 3 s timeout (``config.go:221-240``)."""

    def __init__(self, timeout: float = 3.0):
        self.timeout = timeout

    def test_connection(self, address: str) -> None:
        host, port = split_host_port(address)
        try:
            with socket.create_connection((host, port), timeout=self.timeout):
                pass
        except OSError as e:
            raise ConnectionError(f"failed to connect to {address}: {e}") from e


def split_host_port(address: str):
    if address.startswith("["):
        host, _, rest = address[1:].partition("]")
        return host, int(rest.lstrip(":"))
    host, _, port = address.rpartition(":")
    return (host or "localhost"), int(port)
