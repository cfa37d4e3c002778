"""Serve a TP group through the REAL entry point under torchrun, with every rank on one MI355X, and
make one OpenAI ``/v1/chat/completions`` call and one streaming ``ExecuteToolStream`` call against
it (BASELINE.json config 4: "70B TP=8 over xGMI, OpenAI-compatible chat route").

    python tools/tp_serve_rehearsal.py --world 8 --model llama3-70b [--layers 80] --out DIR

Starts ``python -m torch.distributed.run --nproc-per-node W -m polykey_service_amd.server
--backend=local --tp=W ...`` as a child process (rank 0 serves gRPC + HTTP, ranks 1.. run the
worker loop), waits for grpc.health SERVING, makes the two calls, sends SIGTERM and requires
every rank to exit 0 (graceful shutdown: the leader stops its workers through the step channel).
Writes <out>/serve.json."""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank0(torchrun_pid: int):
    import psutil
    for c in psutil.Process(torchrun_pid).children(recursive=True):
        try:
            if c.environ().get("RANK") == "0" and "polykey_service_amd.server" in " ".join(c.cmdline()):
                return c.pid
        except (psutil.Error, OSError):
            continue
    return None


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--layers", type=int, default=0)
    ap.add_argument("--max-tokens", type=int, default=24)
    ap.add_argument("--timeout", type=float, default=900.0)
    ap.add_argument("--hw-queues", type=int, default=1)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "tp_serve"))
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    import grpc

    from polykey_service_amd import proto
    grpc_port, http_port = _port(), _port()
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""),
               POLYKEY_CUSTOM_AR="force", POLYKEY_CUSTOM_AR_TIMEOUT_S="120", POLYKEY_WATCHDOG_S="300")
    if a.hw_queues:
        env["GPU_MAX_HW_QUEUES"] = str(a.hw_queues)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "-m", "polykey_service_amd.server",
           "--backend=local", f"--model={a.model}", f"--tp={a.world}", f"--num-layers={a.layers}",
           f"--listen-addr=127.0.0.1:{grpc_port}", f"--http-addr=127.0.0.1:{http_port}", "--max-num-seqs=8",
           "--max-model-len=2048", "--num-kv-blocks=512", "--shutdown-grace=5"]
    log = open(os.path.join(a.out, "server.log"), "w")
    proc = subprocess.Popen(cmd, env=env, stdout=log, stderr=subprocess.STDOUT, cwd=ROOT, start_new_session=True)
    res = {"model": a.model, "layers": a.layers or "preset", "tp": a.world, "gpus": 1, "entry": "torchrun -m polykey_service_amd.server"}
    t0 = time.monotonic()
    try:
        ch = grpc.insecure_channel(f"127.0.0.1:{grpc_port}")
        hc = ch.unary_unary(proto.HEALTH_CHECK, request_serializer=proto.HealthCheckRequest.SerializeToString,
                            response_deserializer=proto.HealthCheckResponse.FromString)
        while True:
            if proc.poll() is not None:
                raise RuntimeError(f"server exited early ({proc.returncode})")
            if time.monotonic() - t0 > a.timeout:
                raise RuntimeError("server did not become healthy")
            try:
                if hc(proto.HealthCheckRequest(service=""), timeout=2).status == 1:
                    break
            except grpc.RpcError:
                pass
            time.sleep(1.0)
            if int(time.monotonic() - t0) % 30 == 0:  # heartbeat while the ranks build 80 layers
                print(f"[serve] waiting for SERVING: {time.monotonic() - t0:.0f} s", flush=True)
        res["startup_s"] = round(time.monotonic() - t0, 1)
        # 1. OpenAI-compatible chat route (HTTP, non-streaming)
        body = json.dumps({"model": a.model, "messages": [{"role": "user", "content": "Say hello to the MI355X."}],
                           "max_tokens": a.max_tokens, "temperature": 0.0, "ignore_eos": True}).encode()
        req = urllib.request.Request(f"http://127.0.0.1:{http_port}/v1/chat/completions", data=body,
                                     headers={"Content-Type": "application/json"})
        t1 = time.monotonic()
        with urllib.request.urlopen(req, timeout=600) as r:
            chat = json.loads(r.read())
        res["openai_chat"] = {"status": 200, "latency_s": round(time.monotonic() - t1, 2),
                              "finish_reason": chat["choices"][0]["finish_reason"], "usage": chat["usage"],
                              "object": chat["object"]}
        # 2. streaming gRPC ExecuteToolStream
        stream = ch.unary_stream(proto.EXECUTE_TOOL_STREAM,
                                 request_serializer=proto.ExecuteToolRequest.SerializeToString,
                                 response_deserializer=proto.ExecuteToolResponse.FromString)
        treq = proto.ExecuteToolRequest(tool_name=f"llm.generate:{a.model}")
        treq.parameters.update({"prompt_token_ids": list(range(10, 74)), "max_tokens": a.max_tokens,
                                "ignore_eos": True})
        t2 = time.monotonic()
        chunks, last = 0, None
        for last in stream(treq, timeout=600):
            chunks += 1
        usage = proto.struct_to_dict(last.struct_output).get("usage", {}) if last is not None else {}
        res["grpc_stream"] = {"chunks": chunks, "latency_s": round(time.monotonic() - t2, 2), "usage": usage,
                              "status": int(last.status.code) if last is not None else None}
        ok = (res["openai_chat"]["usage"]["completion_tokens"] == a.max_tokens
              and usage.get("completion_tokens") == a.max_tokens and chunks > 1)
    except Exception as e:  # noqa: BLE001
        res["error"] = repr(e)
        ok = False
    finally:
        if proc.poll() is None:
            # graceful stop = SIGTERM to rank 0 only: its server drains, stops the TP workers through
            # the step channel, and every rank exits 0 (a SIGTERM to torchrun would make its agent
            # kill the workers and report failure)
            r0 = _rank0(proc.pid)
            os.kill(r0 if r0 else proc.pid, signal.SIGTERM)
        try:
            res["exit_code"] = proc.wait(timeout=120)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, signal.SIGKILL)
            res["exit_code"] = proc.wait(timeout=30)
        log.close()
    res["ok"] = bool(ok and res.get("exit_code") == 0)
    print(json.dumps(res), flush=True)
    with open(os.path.join(a.out, "serve.json"), "w") as f:
        json.dump(res, f, indent=1)
    return 0 if res["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
