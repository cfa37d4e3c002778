"""Probe: torch.as_tensor over __cuda_array_interface__ of native device memory on ROCm."""
import ctypes
import torch
x = torch.arange(16, dtype=torch.int32, device="cuda")
ptr = x.data_ptr()


class H:
    __cuda_array_interface__ = {"shape": (64,), "typestr": "|u1", "data": (ptr, False), "version": 3}


t = torch.as_tensor(H(), device="cuda").view(torch.int32)
print("ok", t.device, t[:4].tolist(), t.data_ptr() == ptr)
