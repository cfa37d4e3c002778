"""Per-rank GPU busy fraction over time from rocprofv3 kernel traces of ranks sharing one GPU
(same clock): one row per time bin, one column per rank, plus the union -- shows whether a slow
stretch of a multi-process run is GPU-bound (busy) or host-starved (idle).

    python tools/busy_timeline.py <trace dir rank 0> <rank 1> ... [--bin-ms 500] [--out f.md]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tp_gaps import load  # noqa: E402


def _merge(iv):
    out = []
    for s, e, _ in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def _bins(merged, t0, step, nb):
    busy = [0] * nb
    for s, e in merged:
        b = (s - t0) // step
        while s < e and b < nb:
            be = t0 + (b + 1) * step
            busy[b] += min(e, be) - s
            s = be
            b += 1
    return busy


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--bin-ms", type=float, default=500.0)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    ranks = [load(d) for d in a.dirs]
    t0 = min(tr[0][0] for tr in ranks if tr)
    t1 = max(tr[-1][1] for tr in ranks if tr)
    step = int(a.bin_ms * 1e6)
    nb = (t1 - t0) // step + 1
    per = [_bins(_merge(tr), t0, step, nb) for tr in ranks]
    uni = _bins(_merge(sorted(k for tr in ranks for k in tr)), t0, step, nb)
    cnt = [0] * nb
    for s, _, _ in ranks[0]:
        cnt[(s - t0) // step] += 1
    lines = ["| t (s) | " + " | ".join(f"r{i} busy %" for i in range(len(ranks))) + " | union % | r0 kernels |",
             "|---" * (len(ranks) + 3) + "|"]
    for b in range(nb):
        lines.append(f"| {b * step / 1e9:.1f} | " + " | ".join(f"{100 * p[b] / step:.0f}" for p in per)
                     + f" | {100 * uni[b] / step:.0f} | {cnt[b]} |")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
