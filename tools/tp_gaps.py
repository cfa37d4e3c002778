"""Merge the kernel traces of a one-GPU TP rehearsal's ranks (same GPU, same clock) and report,
for the steady-state decode window: GPU idle time per decode step, each rank's kernels per step
and host gaps, and rank 0's per-kernel table (calls / step, us / call) -- the collective kernels'
cost per call among them.

    python tools/tp_gaps.py <trace dir of rank 0> <rank 1> ... [--out report.md]

Decode steps are delimited by rank 0's sampler kernel; the window is the last 3/4 of the longest
run of sampler launches spaced < 50 ms apart (the timed decode run of tools/tp_rehearsal.py)."""
import argparse
import collections
import csv
import glob
import os


def load(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    return sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f)))


def union_busy(iv, t0, t1):
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in iv:
        s, e = max(s, t0), min(e, t1)
        if e <= s:
            continue
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    return busy


def short(name, n=70):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "", 1)
    depth, cut = 0, len(name)
    for i, ch in enumerate(name):  # the name up to its argument list (template args may hold '(')
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            cut = i
            break
    name = name[:cut]
    return name if len(name) <= n else name[:n]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    ranks = [load(d) for d in a.dirs]
    r0 = ranks[0]
    samp = [k for k in r0 if "sample_kernel" in k[2]]
    runs, cur = [], [samp[0]]
    for x, y in zip(samp, samp[1:]):
        if y[0] - x[0] < 50_000_000:
            cur.append(y)
        else:
            runs.append(cur)
            cur = [y]
    runs.append(cur)
    best = max(runs, key=len)
    best = best[len(best) // 4:]
    t0, t1 = best[0][1], best[-1][1]
    n = max(len(best) - 1, 1)
    allk = sorted(k for tr in ranks for k in tr)
    busy = union_busy(allk, t0, t1)
    lines = [f"# TP rehearsal trace: {len(ranks)} ranks on one GPU", "",
             f"decode window: {n} steps, wall {(t1 - t0) / 1e6:.2f} ms ({(t1 - t0) / n / 1e3:.1f} us/step)",
             f"GPU busy (union of all ranks' kernels): {100 * busy / (t1 - t0):.1f} %, "
             f"idle {(t1 - t0 - busy) / n / 1e3:.2f} us/step", ""]
    for i, tr in enumerate(ranks):
        w = [k for k in tr if t0 <= k[0] < t1]
        gaps = sorted(y[0] - x[1] for x, y in zip(w, w[1:]))
        big = [g for g in gaps if g > 20_000]
        lines.append(f"rank {i}: {len(w)} kernels ({len(w) / n:.0f}/step), own busy "
                     f"{100 * sum(e - s for s, e, _ in w) / (t1 - t0):.1f} %, host gaps > 20 us: {len(big)} "
                     f"({len(big) / n:.2f}/step, max {max(gaps) / 1e3 if gaps else 0:.1f} us)")
    lines += ["", "rank 0 kernels in the window (all ranks share the CUs: times include co-runners)", "",
              "| kernel | calls/step | us/call | us/step |", "|---|---|---|---|"]
    agg = collections.defaultdict(lambda: [0, 0])
    for s, e, name in r0:
        if t0 <= s < t1:
            agg[short(name)][0] += 1
            agg[short(name)][1] += e - s
    for name, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        lines.append(f"| `{name}` | {c / n:.1f} | {t / c / 1e3:.1f} | {t / n / 1e3:.1f} |")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
