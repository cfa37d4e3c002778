"""In-tree build of every native component (HIP kernels for gfx950 + C++ runtime pieces).

Artifacts land in ``polykey_service_amd/_lib/`` so they travel with a ``gpurun`` snapshot
(a JIT cache under ``~/.cache`` would not).  Each target is rebuilt only when the hash of
its sources, headers and flags changes.  No torch headers are involved: HIP kernels are
plain ``extern "C"`` launchers loaded through ctypes (they launch on the caller's HIP
stream, so they are captured by HIP graphs like any other launch), and the CPU-side
C++ modules use pybind11.

Usage: ``python -m polykey_service_amd._native.build [--force] [--only NAME] [-j N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
import json
import os
import shutil
import subprocess
import sys
import sysconfig
from dataclasses import dataclass, field
from typing import List, Optional

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO = os.path.dirname(PKG_DIR)
LIB_DIR = os.path.join(PKG_DIR, "_lib")
OBJ_DIR = os.path.join(REPO, "build", "obj")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


@dataclass
class Target:
    name: str                 # output file stem
    kind: str                 # "hip" (ctypes .so) | "pybind" (python extension)
    sources: List[str]
    headers: List[str] = field(default_factory=list)
    libs: List[str] = field(default_factory=list)
    extra_flags: List[str] = field(default_factory=list)

    def out_path(self) -> str:
        if self.kind == "pybind":
            suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
            return os.path.join(LIB_DIR, self.name + suffix)
        return os.path.join(LIB_DIR, self.name + ".so")


def _g(pattern: str) -> List[str]:
    return sorted(glob.glob(os.path.join(REPO, pattern)))


def targets() -> List[Target]:
    return [
        Target("libpk_kernels", "hip", _g("csrc/kernels/*.hip"), _g("csrc/kernels/*.h") + _g("csrc/kernels/*.cuh")
               + _g("csrc/comm/signals.h")),
        Target("libpk_comm", "hip", _g("csrc/comm/*.hip"), _g("csrc/comm/*.h")),
        Target("_pk_aesgcm", "pybind", _g("csrc/security/*.cpp"), _g("csrc/security/*.h"), ["crypto"]),
        Target("_pk_runtime", "pybind", _g("csrc/runtime/*.cpp"), _g("csrc/runtime/*.h")),
    ]


HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
             "-Wno-unused-variable", "-Wno-unused-result", "-ffp-contract=fast", "-munsafe-fp-atomics"]
CXX_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-fvisibility=hidden"]
if os.environ.get("POLYKEY_DEBUG_KERNELS", "0") == "1":  # device bounds asserts (PK_DEVICE_ASSERT)
    HIP_FLAGS = HIP_FLAGS + ["-DPK_DEBUG", "-g"]


def _hash(t: Target, flags: List[str]) -> str:
    h = hashlib.sha256()
    for p in t.sources + t.headers:
        h.update(p.encode())
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(json.dumps([flags, t.libs, t.extra_flags, ARCH]).encode())
    return h.hexdigest()


def _run(cmd: List[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n  " + " ".join(cmd) + "\n" + r.stdout)


def _pybind_includes() -> List[str]:
    import pybind11
    return ["-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"]]


def build_target(t: Target, force: bool = False, jobs: int = 8, verbose: bool = False) -> Optional[str]:
    if not t.sources:
        return None
    flags = HIP_FLAGS if t.kind == "hip" else CXX_FLAGS + _pybind_includes()
    digest = _hash(t, flags)
    out = t.out_path()
    stamp = out + ".stamp"
    if not force and os.path.exists(out) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == digest:
                return out
    os.makedirs(LIB_DIR, exist_ok=True)
    odir = os.path.join(OBJ_DIR, t.name)
    os.makedirs(odir, exist_ok=True)
    compiler = HIPCC if t.kind == "hip" else "g++"
    inc = ["-I" + os.path.join(REPO, "csrc")]
    objs = []

    def compile_one(src: str) -> str:
        obj = os.path.join(odir, os.path.basename(src) + ".o")
        lang = ["-x", "hip"] if t.kind == "hip" else []
        cmd = [compiler, *lang, *flags, *inc, *t.extra_flags, "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        _run(cmd)
        return obj

    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(compile_one, t.sources))
    tmp = out + ".tmp"
    if t.kind == "hip":
        link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp]
    else:
        link = ["g++", "-shared", "-fPIC", *objs, "-o", tmp] + [f"-l{l}" for l in t.libs]
    _run(link)
    os.replace(tmp, out)
    with open(stamp, "w") as f:
        f.write(digest)
    return out


def build_all(force: bool = False, only: Optional[str] = None, jobs: int = 8, verbose: bool = False) -> List[str]:
    outs = []
    for t in targets():
        if only and t.name != only:
            continue
        o = build_target(t, force=force, jobs=jobs, verbose=verbose)
        if o:
            outs.append(o)
    return outs


def clean() -> None:
    shutil.rmtree(OBJ_DIR, ignore_errors=True)
    for p in glob.glob(os.path.join(LIB_DIR, "*")):
        os.remove(p)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only")
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    if a.clean:
        clean()
        return 0
    for o in build_all(a.force, a.only, a.jobs, a.verbose):
        print(o)
    return 0


if __name__ == "__main__":
    sys.exit(main())
