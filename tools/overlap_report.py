"""Did the comm-stream kernels run concurrently with the compute stream?  Reads one rank's
rocprofv3 ``--kernel-trace --output-format csv`` directory (tools/tp_rehearsal.py --prof writes one
per rank) and reports, per kernel name on the non-dominant stream(s), how much of its duration
overlaps kernels of the rank's main (busiest) stream -- the evidence for the prefill TP overlap
(parallel/comm.py tp_row_parallel_overlapped: the collective of row chunk i on the comm stream
while the GEMM of chunk i + 1 runs).

    python tools/overlap_report.py <trace dir> [out.md]
"""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402


def _stream(r):
    for k in ("Stream_Id", "Queue_Id"):
        if r.get(k) not in (None, ""):
            return r[k]
    return "?"


def overlap(a0, a1, spans):
    """Length of [a0, a1) covered by the sorted, merged intervals ``spans``."""
    tot = 0
    for s0, s1 in spans:
        if s1 <= a0:
            continue
        if s0 >= a1:
            break
        tot += min(a1, s1) - max(a0, s0)
    return tot


def merged(iv):
    out = []
    for s0, s1 in sorted(iv):
        if out and s0 <= out[-1][1]:
            out[-1][1] = max(out[-1][1], s1)
        else:
            out.append([s0, s1])
    return out


def main(argv):
    f = glob.glob(os.path.join(argv[0], "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    by_stream = collections.defaultdict(list)
    for r in rows:
        by_stream[_stream(r)].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    main_s = max(by_stream, key=lambda s: sum(e - b for b, e, _ in by_stream[s]))
    main_spans = merged([(b, e) for b, e, _ in by_stream[main_s]])
    lines = [f"trace {f}", f"streams: " + ", ".join(f"{s}: {len(v)} kernels" for s, v in by_stream.items()),
             f"main stream {main_s}", "",
             "| stream | kernel | calls | total us | overlapped with main stream us | % | calls overlapping a main-stream GEMM |",
             "|---|---|---|---|---|---|---|"]
    gemm_spans = merged([(b, e) for b, e, n in by_stream[main_s] if "Cijk" in n or "gemm" in n.lower()])
    for s, ks in by_stream.items():
        if s == main_s:
            continue
        agg = collections.defaultdict(lambda: [0, 0, 0, 0])
        for b, e, n in ks:
            a = agg[n]
            a[0] += 1
            a[1] += e - b
            a[2] += overlap(b, e, main_spans)
            a[3] += overlap(b, e, gemm_spans) > 0
        for n, (c, tot, ov, g) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            lines.append(f"| {s} | `{n}` | {c} | {tot / 1e3:.1f} | {ov / 1e3:.1f} | {100 * ov / max(tot, 1):.0f} | {g} |")
    # timeline around the first kernel of the busiest side stream: what the main stream was doing
    side = [s for s in by_stream if s != main_s]
    if side:
        s = max(side, key=lambda q: sum(e - b for b, e, _ in by_stream[q]))
        t0 = by_stream[s][0][0] if by_stream[s] else 0
        allk = sorted((b, e, st, n) for st, v in by_stream.items() for b, e, n in v)
        i0 = max(0, next((i for i, k in enumerate(allk) if k[0] >= t0), 0) - 12)
        lines += ["", f"timeline from 12 kernels before the first stream-{s} kernel (us from there)", "",
                  "| start | end | stream | kernel |", "|---|---|---|---|"]
        for b, e, st, n in allk[i0:i0 + 48]:
            lines.append(f"| {(b - t0) / 1e3:.1f} | {(e - t0) / 1e3:.1f} | {st} | `{n}` |")
    text = "\n".join(lines) + "\n"
    if len(argv) > 1:
        open(argv[1], "w").write(text)
    print(text)


if __name__ == "__main__":
    main(sys.argv[1:])
