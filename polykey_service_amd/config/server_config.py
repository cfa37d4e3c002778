"""Server configuration.

The reference server reads only ``LISTEN_ADDR`` (``cmd/polykey/main.go:57-60``) even though
``POLYKEY_ENV`` / ``POLYKEY_LOG_LEVEL`` are set for it.  Here the server
uses the same mechanism as the client loader (defaults < flags < env) and also consumes
the engine options that the on-node backend needs.
"""
from __future__ import annotations

import dataclasses
import os
import sys
from typing import Mapping, Optional, Sequence

from .goflag import FlagSet


@dataclasses.dataclass
class ServerConfig:
    listen_addr: str = ":50051"
    http_addr: str = ""            # OpenAI-compatible route; "" disables
    metrics_addr: str = ""         # Prometheus exporter; "" disables
    log_level: str = "info"
    environment: str = "development"
    backend: str = "mock"          # mock | local
    model: str = "llama3-8b"
    # several models behind this one front end, each on its own GPU(s) of the node:
    # "<model>[@<gpu>|@<first>-<last>][,...]", e.g. "llama3-8b@0-3,mixtral-8x7b@4" (a device range
    # = replicas of that model); "llm.chat:<model>" / OpenAI "model" pick one.  "" -> ``model``
    serve_models: str = ""
    model_path: str = ""           # directory of safetensors shards; "" → random init
    tokenizer: str = ""            # tokenizer.json path; "" → byte-level tokenizer
    dtype: str = "bfloat16"
    tp: int = 1
    ep: int = 1
    replicas: int = 1
    max_num_seqs: int = 256
    max_num_batched_tokens: int = 8192
    max_model_len: int = 8192
    num_layers: int = 0            # > 0: truncate the preset's depth (rehearsals)
    kv_block_size: int = 32
    gpu_mem_fraction: float = 0.90
    num_kv_blocks: int = 0         # 0 → size from free HBM
    hip_graphs: bool = True
    device: str = "cuda"
    seed: int = 0
    shutdown_grace: float = 10.0
    tls_cert: str = ""             # PEM certificate chain; with tls_key: TLS instead of insecure
    tls_key: str = ""              # PEM private key

    @property
    def random_init(self) -> bool:
        return self.model_path == ""


_ENV = {
    "listen_addr": "LISTEN_ADDR",
    "http_addr": "POLYKEY_HTTP_ADDR",
    "metrics_addr": "POLYKEY_METRICS_ADDR",
    "log_level": "POLYKEY_LOG_LEVEL",
    "environment": "POLYKEY_ENV",
    "backend": "POLYKEY_BACKEND",
    "model": "POLYKEY_MODEL",
    "serve_models": "POLYKEY_SERVE_MODELS",
    "model_path": "POLYKEY_MODEL_PATH",
    "tokenizer": "POLYKEY_TOKENIZER",
    "dtype": "POLYKEY_DTYPE",
    "tp": "POLYKEY_TP",
    "ep": "POLYKEY_EP",
    "replicas": "POLYKEY_REPLICAS",
    "max_num_seqs": "POLYKEY_MAX_NUM_SEQS",
    "max_num_batched_tokens": "POLYKEY_MAX_BATCHED_TOKENS",
    "max_model_len": "POLYKEY_MAX_MODEL_LEN",
    "num_layers": "POLYKEY_NUM_LAYERS",
    "kv_block_size": "POLYKEY_KV_BLOCK_SIZE",
    "gpu_mem_fraction": "POLYKEY_GPU_MEM_FRACTION",
    "num_kv_blocks": "POLYKEY_NUM_KV_BLOCKS",
    "hip_graphs": "POLYKEY_HIP_GRAPHS",
    "device": "POLYKEY_DEVICE",
    "seed": "POLYKEY_SEED",
    "shutdown_grace": "POLYKEY_SHUTDOWN_GRACE",
    "tls_cert": "POLYKEY_TLS_CERT",
    "tls_key": "POLYKEY_TLS_KEY",
}


def _flag_name(field: str) -> str:
    return field.replace("_", "-")


def load_server_config(argv: Optional[Sequence[str]] = None,
                       environ: Optional[Mapping[str, str]] = None) -> ServerConfig:
    environ = os.environ if environ is None else environ
    cfg = ServerConfig()
    fs = FlagSet("polykey")
    for f in dataclasses.fields(ServerConfig):
        d = getattr(cfg, f.name)
        name = _flag_name(f.name)
        if isinstance(d, bool):
            fs.bool(name, d, f.name)
        elif isinstance(d, int):
            fs.int(name, d, f.name)
        elif isinstance(d, float):
            fs.float(name, d, f.name)
        else:
            fs.string(name, d, f.name)
    fs.parse(sys.argv[1:] if argv is None else argv)
    for f in dataclasses.fields(ServerConfig):
        setattr(cfg, f.name, fs[_flag_name(f.name)])
    for fname, env in _ENV.items():
        raw = environ.get(env, "")
        if raw == "":
            continue
        cur = getattr(cfg, fname)
        try:
            if isinstance(cur, bool):
                val = raw.lower() in ("1", "true", "t", "yes", "on")
            elif isinstance(cur, int):
                val = int(raw, 0)
            elif isinstance(cur, float):
                val = float(raw)
            else:
                val = raw
        except ValueError:
            continue
        setattr(cfg, fname, val)
    return cfg
