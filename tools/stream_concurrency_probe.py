"""Do kernels on two HIP streams of one process run concurrently on MI355X?  A GEMM (hipBLASLt)
on the current stream and an elementwise stream on a side stream, timed alone and together
(events; best of 5).  Under ``rocprofv3 --kernel-trace`` the trace shows whether they overlap
there too (tools/overlap_report.py).  One JSON line.

    python tools/stream_concurrency_probe.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def timed(fn, reps=5):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return round(best * 1000, 1)


def main():
    a = torch.randn(8192, 8192, device="cuda").to(torch.bfloat16)
    b = torch.randn(8192, 8192, device="cuda").to(torch.bfloat16)
    c = torch.empty(8192, 8192, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(128 << 20, device="cuda")  # 512 MB
    side = torch.cuda.Stream()
    main_s = torch.cuda.current_stream()

    def gemm():
        for _ in range(4):
            torch.mm(a, b, out=c)

    def ew():
        with torch.cuda.stream(side):
            for _ in range(8):
                x.mul_(1.0001)
        main_s.wait_stream(side)

    def both():
        side.wait_stream(main_s)
        with torch.cuda.stream(side):
            for _ in range(8):
                x.mul_(1.0001)
        gemm()
        main_s.wait_stream(side)

    for f in (gemm, ew, both):
        f()
    r = {"gemm_us": timed(gemm), "side_us": timed(ew), "both_us": timed(both),
         "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "default")}
    r["overlap_fraction"] = round((r["gemm_us"] + r["side_us"] - r["both_us"]) / min(r["gemm_us"], r["side_us"]), 2)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
