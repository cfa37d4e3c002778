"""Every in-tree native library dlopens with all symbols resolved (RTLD_NOW) on the CPU: hipcc's
host pass can silently drop a kernel template's launch stub (e.g. a buffer / LDS-DMA builtin called
directly inside the template), which otherwise surfaces only on the GPU box as an undefined
symbol at first use."""
import ctypes
import glob
import os

import pytest

LIB = os.path.join(os.path.dirname(__file__), "..", "..", "polykey_service_amd", "_lib")


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(LIB, "*.so"))), ids=os.path.basename)
def test_library_resolves_all_symbols(path):
    ctypes.CDLL(path, mode=os.RTLD_NOW | os.RTLD_LOCAL)
