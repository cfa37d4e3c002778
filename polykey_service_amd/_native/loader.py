"""Locate (and if needed build) the in-tree native artifacts.

Policy: a missing artifact is built on first use when a toolchain is present; if that is
impossible the import fails loudly — there is no silent pure-Python substitute for a
native component.
"""
from __future__ import annotations

import ctypes
import importlib.util
import os
import sys
import threading

from . import build as _build

_lock = threading.Lock()
_cache = {}


def _target(name: str) -> "_build.Target":
    for t in _build.targets():
        if t.name == name:
            return t
    raise KeyError(name)


def artifact_path(name: str, build_if_missing: bool = True) -> str:
    t = _target(name)
    path = t.out_path()
    if build_if_missing and (not os.path.exists(path) or os.environ.get("POLYKEY_REBUILD") == "1"):
        _build.build_target(t)
    if not os.path.exists(path):
        raise ImportError(f"native artifact {name} not built (expected {path}); "
                          f"run `python -m polykey_service_amd._native.build`")
    return path


def load_extension(name: str):
    """Import a pybind11 module from ``_lib``."""
    with _lock:
        if name in _cache:
            return _cache[name]
        path = artifact_path(name)
        spec = importlib.util.spec_from_file_location(name, path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        sys.modules.setdefault(name, mod)
        _cache[name] = mod
        return mod


def load_cdll(name: str) -> ctypes.CDLL:
    """dlopen a HIP launcher library.  torch must be imported first so the HIP runtime
    (soname ``libamdhip64.so.7``) resolves to the copy torch already loaded."""
    with _lock:
        if name in _cache:
            return _cache[name]
        import torch  # noqa: F401
        # A/B runs of kernel-library builds (tools/ab_decode.py): POLYKEY_LIB_<NAME> = path of a
        # variant build of the same sources
        path = os.environ.get("POLYKEY_LIB_" + name.upper()) or artifact_path(name)
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        _cache[name] = lib
        return lib
