"""ConfigLoader precedence matrix + RuntimeDetector (reference internal/config/config.go)."""
import os

import pytest

from polykey_service_amd.config import (ConfigLoader, FlagError, FlagSet, RuntimeDetector,
                                        RuntimeEnvironment, load_server_config)
from polykey_service_amd.utils.slog import go_duration, parse_go_duration


def fake_root(tmp_path, dockerenv=False, k8s=False, cgroup=None):
    if dockerenv:
        (tmp_path / ".dockerenv").write_text("")
    if k8s:
        (tmp_path / "var/run/secrets/kubernetes.io/serviceaccount").mkdir(parents=True)
    if cgroup is not None:
        (tmp_path / "proc/1").mkdir(parents=True)
        (tmp_path / "proc/1/cgroup").write_text(cgroup)
    return str(tmp_path)


@pytest.mark.parametrize("kw,env,expected", [
    ({}, {}, RuntimeEnvironment.LOCAL),
    ({"dockerenv": True}, {}, RuntimeEnvironment.DOCKER),
    ({"cgroup": "12:pids:/docker/abc\n"}, {}, RuntimeEnvironment.DOCKER),
    ({"cgroup": "0::/system.slice/containerd.service\n"}, {}, RuntimeEnvironment.CONTAINERD),
    ({"cgroup": "0::/machine.slice/libpod-podman-123.scope\n"}, {}, RuntimeEnvironment.PODMAN),
    ({}, {"container": "podman"}, RuntimeEnvironment.PODMAN),
    ({"k8s": True, "dockerenv": True}, {}, RuntimeEnvironment.KUBERNETES),
    ({}, {"KUBERNETES_SERVICE_HOST": "10.0.0.1"}, RuntimeEnvironment.KUBERNETES),
    # priority: podman beats containerd beats docker
    ({"dockerenv": True, "cgroup": "containerd"}, {}, RuntimeEnvironment.CONTAINERD),
    ({"dockerenv": True, "cgroup": "containerd podman"}, {}, RuntimeEnvironment.PODMAN),
])
def test_runtime_detection(tmp_path, kw, env, expected):
    det = RuntimeDetector(root=fake_root(tmp_path, **kw), environ=env)
    assert det.detect_runtime() == expected


def test_runtime_strings():
    assert [str(r) for r in RuntimeEnvironment] == ["local", "docker", "kubernetes", "containerd", "podman"]


def loader(tmp_path, env=None, **kw):
    env = env or {}
    return ConfigLoader(RuntimeDetector(root=fake_root(tmp_path, **kw), environ=env), environ=env)


def test_defaults_local(tmp_path):
    cfg = loader(tmp_path).load([])
    assert (cfg.server_address, cfg.timeout, cfg.log_level, cfg.environment) == \
        ("localhost:50051", 5.0, "info", "development")


@pytest.mark.parametrize("kw,addr", [({"k8s": True}, "polykey-service:50051"),
                                     ({"dockerenv": True}, "polykey-server:50051"),
                                     ({"cgroup": "containerd"}, "polykey-server:50051")])
def test_autodetect(tmp_path, kw, addr):
    assert loader(tmp_path, **kw).load([]).server_address == addr


def test_flags_then_env_precedence(tmp_path):
    argv = ["-server", "flag:1", "--timeout=7s", "-log-level", "debug", "-env", "staging"]
    cfg = loader(tmp_path).load(argv)
    assert (cfg.server_address, cfg.timeout, cfg.log_level, cfg.environment) == ("flag:1", 7.0, "debug", "staging")
    env = {"POLYKEY_SERVER_ADDR": "env:2", "POLYKEY_TIMEOUT": "1m30s", "POLYKEY_LOG_LEVEL": "warn",
           "POLYKEY_ENV": "prod"}
    cfg = loader(tmp_path, env).load(argv)
    assert (cfg.server_address, cfg.timeout, cfg.log_level, cfg.environment) == ("env:2", 90.0, "warn", "prod")


def test_invalid_env_timeout_ignored(tmp_path):
    cfg = loader(tmp_path, {"POLYKEY_TIMEOUT": "banana"}).load(["-timeout", "3s"])
    assert cfg.timeout == 3.0


def test_flag_address_prevents_autodetect(tmp_path):
    assert loader(tmp_path, dockerenv=True).load(["-server=x:9"]).server_address == "x:9"


def test_load_twice_does_not_panic(tmp_path):
    l = loader(tmp_path)
    l.load([])
    l.load([])  # the Go version panics with "flag redefined" 


def test_unknown_flag_and_missing_arg():
    fs = FlagSet()
    fs.string("server")
    with pytest.raises(FlagError):
        fs.parse(["-nope"])
    with pytest.raises(FlagError):
        FlagSet().parse(["-server"])
    fs2 = FlagSet()
    fs2.bool("v")
    fs2.string("s")
    fs2.parse(["-v", "-s", "x", "rest", "-s", "y"])
    assert fs2["v"] is True and fs2["s"] == "x" and fs2.args == ["rest", "-s", "y"]


@pytest.mark.parametrize("text,secs", [("5s", 5), ("1m30s", 90), ("250ms", .25), ("1.5h", 5400),
                                       ("2us", 2e-6), ("-3s", -3), ("0", 0), ("1h2m3s", 3723)])
def test_parse_duration(text, secs):
    assert parse_go_duration(text) == pytest.approx(secs)


@pytest.mark.parametrize("bad", ["", "5", "s", "1x", "1.s.2"])
def test_parse_duration_bad(bad):
    with pytest.raises(ValueError):
        parse_go_duration(bad)


@pytest.mark.parametrize("secs,text", [(0, "0s"), (1.5e-3, "1.5ms"), (2.5e-6, "2.5µs"), (5e-9, "5ns"),
                                       (90, "1m30s"), (3723.5, "1h2m3.5s"), (1.0, "1s"), (0.1234567, "123.4567ms")])
def test_go_duration(secs, text):
    assert go_duration(secs) == text


def test_server_config_precedence():
    cfg = load_server_config(["-tp", "8", "-backend", "local", "-hip-graphs=false"],
                             {"LISTEN_ADDR": ":6000", "POLYKEY_MAX_NUM_SEQS": "64"})
    assert cfg.tp == 8 and cfg.backend == "local" and cfg.hip_graphs is False
    assert cfg.listen_addr == ":6000" and cfg.max_num_seqs == 64 and cfg.random_init
