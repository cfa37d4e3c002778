"""Build sanity of the HIP kernel library: every kernel launch stub is defined.

hipcc's host pass can silently drop a kernel's launch stub (seen with an LDS-DMA builtin
called directly inside a kernel template, csrc/kernels/gemm_prefill.hip glds16): the library
links, and only dlopen on the GPU box fails with an undefined ``__device_stub__`` symbol."""
import shutil
import subprocess

import pytest

from polykey_service_amd._native.loader import artifact_path


@pytest.mark.skipif(shutil.which("nm") is None, reason="binutils nm not installed")
def test_no_undefined_kernel_stubs():
    path = artifact_path("libpk_kernels", build_if_missing=False)
    out = subprocess.run(["nm", "-D", "--undefined-only", path], capture_output=True, text=True, check=True).stdout
    missing = [l.split()[-1] for l in out.splitlines() if "__device_stub__" in l]
    assert not missing, f"undefined kernel launch stubs in {path}: {missing}"


def test_grouped_reference_matches_dense_reference():
    import torch
    from polykey_service_amd.ops import gemm_prefill
    x, w = torch.randn(40, 64).bfloat16(), (torch.randn(3, 256, 64) * 0.1).bfloat16()
    offs = torch.tensor([0, 10, 10, 33], dtype=torch.int32)
    y = gemm_prefill.grouped_linear(x, w, offs, silu=True)
    assert y.shape == (40, 128) and torch.count_nonzero(y[33:]) == 0
    torch.testing.assert_close(y[10:33], gemm_prefill.linear(x[10:33], w[2], silu=True))


def test_gemm_args_mirror_matches_the_native_struct():
    """ops/gemm.py GemmArgs (ctypes) has the size of csrc/kernels/skinny_tile.h GemmArgs, including
    the push fields of the TP decode GEMM epilogue; the comm library exports the push entry points."""
    import ctypes

    from polykey_service_amd.ops import gemm, native
    from polykey_service_amd.parallel import custom_ar
    assert native.lib().pk_gemm_args_size() == ctypes.sizeof(gemm.GemmArgs)
    lib = custom_ar._lib()
    assert lib.pk_car_push_target and lib.pk_car_reduce_residual_pushed
