"""Container-runtime detection (reference ``internal/config/config.go:22-120``).

Priority order is Kubernetes → Podman → containerd → Docker → local
(``config.go:57-77``).  The cgroup probe is a substring match on ``/proc/1/cgroup``
(``config.go:111-120``).  ``root`` and ``environ`` are injectable so tests can fake the
filesystem and the environment.
"""
from __future__ import annotations

import enum
import os
from typing import Mapping, Optional


class RuntimeEnvironment(enum.IntEnum):
    LOCAL = 0
    DOCKER = 1
    KUBERNETES = 2
    CONTAINERD = 3
    PODMAN = 4

    def __str__(self) -> str:  # config.go:33-48
        return {0: "local", 1: "docker", 2: "kubernetes", 3: "containerd", 4: "podman"}.get(int(self), "unknown")


class RuntimeDetector:
    K8S_SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"

    def __init__(self, root: str = "/", environ: Optional[Mapping[str, str]] = None):
        self.root = root
        self.environ = os.environ if environ is None else environ

    def _p(self, path: str) -> str:
        return os.path.join(self.root, path.lstrip("/"))

    def detect_runtime(self) -> RuntimeEnvironment:
        if self.is_kubernetes():
            return RuntimeEnvironment.KUBERNETES
        if self.is_podman():
            return RuntimeEnvironment.PODMAN
        if self.is_containerd():
            return RuntimeEnvironment.CONTAINERD
        if self.is_docker():
            return RuntimeEnvironment.DOCKER
        return RuntimeEnvironment.LOCAL

    def is_kubernetes(self) -> bool:
        if os.path.exists(self._p(self.K8S_SA_DIR)):
            return True
        return self.environ.get("KUBERNETES_SERVICE_HOST", "") != ""

    def is_docker(self) -> bool:
        if os.path.exists(self._p("/.dockerenv")):
            return True
        return self.check_cgroup("docker")

    def is_containerd(self) -> bool:
        return self.check_cgroup("containerd")

    def is_podman(self) -> bool:
        if self.environ.get("container", "") == "podman":
            return True
        return self.check_cgroup("podman")

    def check_cgroup(self, runtime: str) -> bool:
        try:
            with open(self._p("/proc/1/cgroup"), "r", errors="replace") as f:
                content = f.read()
        except OSError:
            return False
        return runtime in content or f"/{runtime}/" in content
