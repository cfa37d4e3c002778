"""Direct RCCL binding (csrc/comm/rccl_comm.hip, parallel/rccl.py) on the CPU: the library
resolves the RCCL copy PyTorch already loaded (no second RCCL in the process), reports its
version, draws distinct 128-byte unique ids and names its errors.  Communicators themselves
need a GPU: tests/parallel/test_rccl_gpu.py."""
import ctypes

from polykey_service_amd.parallel import rccl


def test_binding_resolves_the_resident_rccl():
    assert rccl.load()
    assert rccl.version() > 20000  # e.g. 22606 = RCCL 2.26.6
    assert "resident" in rccl.library()


def test_unique_ids_are_fresh():
    a, b = rccl.unique_id(), rccl.unique_id()
    assert len(a) == len(b) == 128 and a != b


def test_error_paths_report_instead_of_crashing():
    lib = rccl._lib()
    assert lib.pk_rccl_all_reduce(None, None, None, 0, 0, 0, None) == -1  # null communicator
    assert lib.pk_rccl_init(ctypes.byref(ctypes.c_void_p()), None, 1, 0) == -1  # no unique id
    assert b"bad argument" in lib.pk_rccl_error_string(-1)
    assert rccl.DTYPES and set(rccl.OPS) == {"sum", "max", "min"}
