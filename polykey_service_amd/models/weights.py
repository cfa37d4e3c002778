"""Weight materialisation: deterministic random init or HF safetensors, sharded for TP/EP.

Random init (the north-star benchmarks use random weights, ``BASELINE.json:5``): each full
parameter is drawn from its own generator seeded by ``hash(seed, name)`` on the target device
and then sliced for this rank, so a TP=N model holds exactly the shards of the TP=1 model
(the TP tests rely on it).  Norm weights are ones.

Safetensors (``safetensors.safe_open``, never pickle): HF Llama / Mixtral tensor names are
mapped onto the fused layout used here (q|k|v → ``qkv``, gate|up → ``gate_up``,
Mixtral w1|w3 → ``w13``) and sliced per rank on load.
"""
from __future__ import annotations

import glob
import hashlib
import os
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch

Slicer = Callable[[torch.Tensor], torch.Tensor]


def _seed_for(seed: int, name: str) -> int:
    h = hashlib.sha256(f"{seed}:{name}".encode()).digest()
    return int.from_bytes(h[:8], "little") & ((1 << 63) - 1)


def random_full(name: str, shape: Sequence[int], std: float, seed: int, device, dtype) -> torch.Tensor:
    g = torch.Generator(device=device)
    g.manual_seed(_seed_for(seed, name))
    t = torch.empty(tuple(shape), dtype=torch.float32 if device.type == "cpu" else dtype, device=device)
    t.normal_(0.0, std, generator=g)
    return t.to(dtype)


RANDOM_BLOCK = 128


def random_slice(name: str, shape: Sequence[int], std: float, seed: int, device, dtype, dim: int = 0,
                 lo: int = 0, hi: Optional[int] = None, block: int = RANDOM_BLOCK) -> torch.Tensor:
    """Indices [lo, hi) along ``dim`` of the logical random tensor ``shape`` without drawing the
    rest: the tensor is cut into ``block``-wide slabs along ``dim``, each drawn from its own
    seeded generator, so every rank of any TP degree materialises exactly its own shard and the
    shards of TP = 8 concatenate to the TP = 1 tensor (a 70B rank draws 17.6 GB, not 141 GB)."""
    n = shape[dim]
    hi = n if hi is None else min(hi, n)
    shp = list(shape)
    shp[dim] = max(hi - lo, 0)
    out = torch.empty(shp, dtype=dtype, device=device)
    b = lo // block
    while b * block < hi:
        bl, bh = b * block, min(n, (b + 1) * block)
        sub = list(shape)
        sub[dim] = bh - bl
        t = random_full(f"{name}#{b}", sub, std, seed, device, dtype)
        a, z = max(lo, bl), min(hi, bh)
        out.narrow(dim, a - lo, z - a).copy_(t.narrow(dim, a - bl, z - a))
        b += 1
    return out


def random_shard(name: str, shape: Sequence[int], std: float, seed: int, device, dtype, rank: int, world: int,
                 dim: int = 0, pad_to: Optional[int] = None) -> torch.Tensor:
    """Rank ``rank``'s 1/``world`` shard along ``dim`` (``pad_to``: shard size after zero-padding
    the logical dimension, e.g. vocab shards rounded up to 128 rows)."""
    n = shape[dim]
    k = pad_to if pad_to is not None else n // world
    assert pad_to is not None or n % world == 0, (shape, world)
    t = random_slice(name, shape, std, seed, device, dtype, dim, rank * k, (rank + 1) * k)
    if t.shape[dim] < k:
        pad = list(t.shape)
        pad[dim] = k - t.shape[dim]
        t = torch.cat([t, t.new_zeros(pad)], dim)
    return t


def shard_rows(t: torch.Tensor, rank: int, world: int) -> torch.Tensor:
    n = t.shape[0]
    assert n % world == 0, (t.shape, world)
    k = n // world
    return t[rank * k:(rank + 1) * k]


def shard_cols(t: torch.Tensor, rank: int, world: int) -> torch.Tensor:
    n = t.shape[-1]
    assert n % world == 0, (t.shape, world)
    k = n // world
    return t[..., rank * k:(rank + 1) * k]


class SafetensorsIndex:
    """Lazy name → file map over a directory of ``*.safetensors`` shards."""

    def __init__(self, path: str):
        from safetensors import safe_open
        self._safe_open = safe_open
        files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
        if not files:
            raise FileNotFoundError(f"no .safetensors files under {path}")
        self.where: Dict[str, str] = {}
        for f in files:
            with safe_open(f, framework="pt") as h:
                for k in h.keys():
                    self.where[k] = f
        self._open: Dict[str, object] = {}

    def has(self, name: str) -> bool:
        return name in self.where

    def get(self, name: str) -> torch.Tensor:
        f = self.where[name]
        if f not in self._open:
            self._open[f] = self._safe_open(f, framework="pt")
        return self._open[f].get_tensor(name)
