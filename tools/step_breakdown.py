"""Per-phase kernel breakdown of one timed bench wave from a rocprofv3 kernel trace
(``rocprofv3 --kernel-trace --output-format csv -- python3 bench.py --steps 1 --warmup 1``).

The last wave is located after the longest idle gap in the second half of the trace; steps are
delimited by the sampler kernel.  Prints wall/busy time of the prefill steps and the decode
steps and the per-kernel time of an average decode step (us), as markdown.
Usage: step_breakdown.py <rocprof dir> [out.md]"""
import collections
import csv
import glob
import os
import re
import sys


def short(n: str) -> str:
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"\(.*", "", n).replace("void ", "")
    return n[:70]


def main(argv):
    f = glob.glob(os.path.join(argv[0], "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    t = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    half = len(t) // 2
    gaps = [(t[i + 1][0] - t[i][1], i) for i in range(half, len(t) - 1)]
    start = max(gaps)[1] + 1 if gaps else 0
    # the wave starts at the first embedding after the longest gap of the second half
    w = t[start:]
    idx = [i for i, x in enumerate(w) if "sample_kernel" in x[2]]
    steps, prev = [], 0
    for i in idx:
        steps.append(w[prev:i + 1])
        prev = i + 1
    pre = [s for s in steps if any("Cijk" in k[2] and "MT256x256" in k[2] for k in s) or len(s) > 400]
    dec = [s for s in steps if s not in pre]
    out = []
    span = lambda seg: (seg[-1][1] - seg[0][0]) / 1e6
    busy = lambda seg: sum(b - a for a, b, _ in seg) / 1e6
    out.append(f"wave: {len(steps)} steps, wall {span(w):.1f} ms, kernel busy {busy(w):.1f} ms")
    out.append(f"prefill steps: {len(pre)}, wall {sum(span(s) for s in pre):.1f} ms, busy {sum(busy(s) for s in pre):.1f} ms")
    if dec:
        out.append(f"decode steps: {len(dec)}, wall {sum(span(s) for s in dec):.1f} ms, busy "
                   f"{sum(busy(s) for s in dec):.1f} ms, {1e3 * sum(span(s) for s in dec) / len(dec):.0f} us/step")
        d = collections.defaultdict(lambda: [0, 0])
        for s in dec:
            for a, b, n in s:
                d[short(n)][0] += 1
                d[short(n)][1] += b - a
        out += ["", "| kernel (decode step average) | calls/step | us/step | us/call |", "|---|---|---|---|"]
        for k, (c, tt) in sorted(d.items(), key=lambda x: -x[1][1]):
            out.append(f"| `{k}` | {c / len(dec):.0f} | {tt / len(dec) / 1e3:.1f} | {tt / c / 1e3:.1f} |")
    if pre:
        d = collections.defaultdict(lambda: [0, 0])
        for s in pre:
            for a, b, n in s:
                d[short(n)][0] += 1
                d[short(n)][1] += b - a
        out += ["", "| kernel (all prefill steps of the wave) | calls | ms | us/call |", "|---|---|---|---|"]
        for k, (c, tt) in sorted(d.items(), key=lambda x: -x[1][1])[:12]:
            out.append(f"| `{k}` | {c} | {tt / 1e6:.2f} | {tt / c / 1e3:.1f} |")
    text = "\n".join(out) + "\n"
    if len(argv) > 1:
        open(argv[1], "w").write(text)
    print(text)


if __name__ == "__main__":
    main(sys.argv[1:])
