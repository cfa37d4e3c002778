"""The fused TP decode collective at the 70B TP=8 per-rank shapes, one process on one GPU: a
loopback group (CustomAllReduce.loopback: the 7 peers are local stand-in buffers whose flags never
block), so each call does all of its own work -- slab sum, publishes, slot stores and reads,
fences -- without the xGMI latency or rank skew.  Graph of 80 calls per form, us per call:

  rr       reduce_residual after the plain split-K o GEMM's slabs (the serving chain)
  gemm_rr  the o GEMM + reduce_residual
  push_rr  the push o GEMM + reduce_residual_pushed (POLYKEY_TP_PUSH)

    python tools/car_probe.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from polykey_service_amd.ops import gemm  # noqa: E402
from polykey_service_amd.parallel.custom_ar import CustomAllReduce  # noqa: E402
from tools.push_probe import timed  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    W, M, N, K = 8, 64, 8192, 1024
    car = CustomAllReduce.loopback(0, W, dev)
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    wp = gemm.pack_weight((torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16))
    ws = torch.empty(8 * M * N, dtype=torch.float32, device=dev)
    res = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
    parts = torch.zeros((N // 256) * M, dtype=torch.float32, device=dev)
    ctr = torch.zeros(N // 64, dtype=torch.int32, device=dev)
    pend = gemm.linear_partial(x, wp, ws, packed=wp, half=True)
    torch.cuda.synchronize()
    r = {"W": W, "M": M, "N": N, "K": K, "lib": os.environ.get("POLYKEY_LIB_LIBPK_COMM", "in-tree"),
         "rr_us": timed(lambda: car.reduce_residual(pend, res, parts)),
         "gemm_rr_us": timed(lambda: car.reduce_residual(gemm.linear_partial(x, wp, ws, packed=wp, half=True),
                                                           res, parts)),
         "push_rr_us": timed(lambda: car.reduce_residual_pushed(
             res, parts, gemm.push_projection(x, wp, ws, wp, ctr, car.push_target())))}
    assert car.error() == 0
    car.close()
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
