"""Harness for the dead-rank tests (reference contract:
health + exit + ``restart: unless-stopped``, /root/reference/compose.yml:17-33).

Two real server processes form one TP=2 group (``python -m polykey_service_amd.server``, started
directly -- not through torchrun, whose agent would kill the survivor itself and hide what is
under test).  A streaming generation runs; one rank is SIGKILLed mid-decode; the survivor must
exit non-zero within the bound, and when the survivor is the front end (rank 0) its health
must read NOT_SERVING before it goes."""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import threading
import time

import grpc

from polykey_service_amd import proto

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def start_group(tmp, model: str, gpu: bool, timeout_s: float = 5.0):
    master, grpc_port = _port(), _port()
    procs = []
    for r in range(2):
        env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(master), RANK=str(r), WORLD_SIZE="2",
                   LOCAL_RANK="0" if gpu else str(r), LOCAL_WORLD_SIZE="2",
                   POLYKEY_CUSTOM_AR_TIMEOUT_S=str(timeout_s), POLYKEY_WATCHDOG_S=str(3 * timeout_s))
        if gpu:
            env.update(POLYKEY_CUSTOM_AR="force", POLYKEY_DIST_BACKEND="gloo")
        else:
            env["CUDA_VISIBLE_DEVICES"] = ""
        cmd = [sys.executable, "-m", "polykey_service_amd.server", "--backend=local", f"--model={model}", "--tp=2",
               f"--listen-addr=127.0.0.1:{grpc_port}", "--max-num-seqs=4", "--max-model-len=2048",
               "--num-kv-blocks=256", f"--hip-graphs={'true' if gpu else 'false'}", "--shutdown-grace=1"]
        log = open(os.path.join(str(tmp), f"rank{r}.log"), "w")
        procs.append((subprocess.Popen(cmd, env=env, stdout=log, stderr=subprocess.STDOUT, cwd=ROOT), log))
    return procs, f"127.0.0.1:{grpc_port}"


def health(ch) -> int:
    hc = ch.unary_unary(proto.HEALTH_CHECK, request_serializer=proto.HealthCheckRequest.SerializeToString,
                        response_deserializer=proto.HealthCheckResponse.FromString)
    try:
        return hc(proto.HealthCheckRequest(service=""), timeout=2).status
    except grpc.RpcError:
        return -1


def run_kill(tmp, model: str, gpu: bool, victim: int, bound_s: float):
    """Returns (survivor exit code, seconds from kill to exit, health statuses seen after the kill).
    A group whose gRPC port was taken between the free-port probe and the bind (an ephemeral port
    handed to another socket meanwhile) is started once more on new ports."""
    for attempt in range(2):
        try:
            return _run_kill(tmp, model, gpu, victim, bound_s)
        except AssertionError as e:
            if attempt or "Failed to bind to address" not in str(e):
                raise


def _run_kill(tmp, model: str, gpu: bool, victim: int, bound_s: float):
    procs, addr = start_group(tmp, model, gpu)
    try:
        ch = grpc.insecure_channel(addr)
        deadline = time.monotonic() + (600 if gpu else 240)
        while health(ch) != 1:
            if any(p.poll() is not None for p, _ in procs) or time.monotonic() > deadline:
                raise AssertionError("group did not come up:\n" + _logs(tmp))
            time.sleep(0.5)
        stream = ch.unary_stream(proto.EXECUTE_TOOL_STREAM,
                                 request_serializer=proto.ExecuteToolRequest.SerializeToString,
                                 response_deserializer=proto.ExecuteToolResponse.FromString)
        req = proto.ExecuteToolRequest(tool_name=f"llm.generate:{model}")
        req.parameters.update({"prompt_token_ids": list(range(3, 40)), "max_tokens": 1900, "ignore_eos": True})
        got = {"chunks": 0, "error": None}

        def consume():
            try:
                for _ in stream(req, timeout=120):
                    got["chunks"] += 1
            except grpc.RpcError as e:
                got["error"] = e.code().name
        th = threading.Thread(target=consume, daemon=True)
        th.start()
        t_wait = time.monotonic() + 60
        while got["chunks"] < 3 and time.monotonic() < t_wait:
            time.sleep(0.05)
        assert got["chunks"] >= 3, "decode never started:\n" + _logs(tmp)
        os.kill(procs[victim][0].pid, signal.SIGKILL)
        t_kill = time.monotonic()
        survivor = procs[1 - victim][0]
        seen = []
        while survivor.poll() is None and time.monotonic() - t_kill < bound_s:
            if victim == 1:
                seen.append(health(ch))
            time.sleep(0.1)
        rc = survivor.poll()
        dt = time.monotonic() - t_kill
        th.join(10)
        return rc, dt, seen, got, _logs(tmp)
    finally:
        for p, log in procs:
            if p.poll() is None:
                p.kill()
            p.wait(30)
            log.close()


def _logs(tmp) -> str:
    out = []
    for r in range(2):
        path = os.path.join(str(tmp), f"rank{r}.log")
        if os.path.exists(path):
            out.append(f"--- rank {r}\n" + open(path).read()[-3000:])
    return "\n".join(out)
