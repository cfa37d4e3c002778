"""Where the GPU idles inside one timed bench wave (rocprofv3 kernel trace of
``bench.py --steps 1 --warmup 1``): every inter-kernel gap above a threshold in the last wave,
with the step it falls in (steps delimited by the sampler kernel), the kernels on both sides and
a histogram by (before, after) pair -- host stalls show up as gaps in front of a step's first
kernel, in-graph dependencies as gaps inside a step.

    python tools/wave_gaps.py <rocprof dir> [threshold_us=10] [out.md]
"""
import collections
import csv
import glob
import os
import re
import sys


def short(n: str) -> str:
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"\(.*", "", n).replace("void ", "")
    return n[:60]


def main(argv):
    f = glob.glob(os.path.join(argv[0], "**", "*kernel_trace.csv"), recursive=True)[0]
    thr = float(argv[1]) if len(argv) > 1 else 10.0
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    t = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows]
    half = len(t) // 2
    gaps = [(t[i + 1][0] - t[i][1], i) for i in range(half, len(t) - 1)]
    start = max(gaps)[1] + 1 if gaps else 0  # the last wave starts after the longest idle of the second half
    w = t[start:]
    step = 0
    found = []
    end_seen = 0
    for i in range(len(w) - 1):
        if "sample_kernel" in w[i][2]:
            step += 1
        end_seen = max(end_seen, w[i][1])
        g = (w[i + 1][0] - end_seen) / 1e3
        if g > thr:
            found.append((step, g, w[i][2], w[i + 1][2]))
    span = (w[-1][1] - w[0][0]) / 1e6
    busy = sum(b - a for a, b, _ in w) / 1e6
    out = [f"wave: {step} steps, wall {span:.1f} ms, kernel busy {busy:.1f} ms, "
           f"{len(found)} gaps > {thr:g} us summing {sum(g for _, g, _, _ in found) / 1e3:.2f} ms", ""]
    pairs = collections.defaultdict(list)
    for s, g, a, b in found:
        pairs[(a, b)].append(g)
    out += ["| before | after | gaps | total ms | mean us | max us |", "|---|---|---|---|---|---|"]
    for (a, b), gs in sorted(pairs.items(), key=lambda kv: -sum(kv[1])):
        out.append(f"| `{a}` | `{b}` | {len(gs)} | {sum(gs) / 1e3:.2f} | {sum(gs) / len(gs):.1f} | {max(gs):.1f} |")
    out += ["", "largest gaps (step, us, before -> after):", ""]
    for s, g, a, b in sorted(found, key=lambda x: -x[1])[:25]:
        out.append(f"- step {s}: {g:.1f} us, `{a}` -> `{b}`")
    text = "\n".join(out)
    print(text)
    if len(argv) > 2:
        open(argv[2], "w").write(text + "\n")


if __name__ == "__main__":
    main(sys.argv[1:])
