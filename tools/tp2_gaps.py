"""Merge the kernel traces of the two TP=2 rehearsal ranks (same GPU, same clock) and report, for
the decode window, the GPU idle time per decode step and each rank's inter-step gaps.

    python tools/tp2_gaps.py <rank0 rocprof dir> <rank1 rocprof dir> [out.md]

Decode steps are delimited by rank 0's sampler kernel.  The window is the last ``--frac`` of
rank 0's sampler launches (steady-state decode of the timed run)."""
import csv
import glob
import os
import sys


def load(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    return sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f))))


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


def main(argv):
    r0, r1 = load(argv[0]), load(argv[1])
    samp = [k for k in r0 if "sample_kernel" in k[2]]
    # the timed decode run: the longest run of sampler launches spaced < 50 ms apart, last 3/4 of it
    runs, cur = [], [samp[0]]
    for a, b in zip(samp, samp[1:]):
        if b[0] - a[0] < 50_000_000:
            cur.append(b)
        else:
            runs.append(cur)
            cur = [b]
    runs.append(cur)
    best = max(runs, key=len)
    best = best[len(best) // 4:]
    t0, t1 = best[0][1], best[-1][1]
    n = len(best) - 1
    both = sorted(r0 + r1)
    busy = union_busy(both, t0, t1)
    lines = [f"decode window: {n} steps, wall {(t1 - t0) / 1e6:.2f} ms ({(t1 - t0) / n / 1e3:.1f} us/step)",
             f"GPU busy (union of both ranks' kernels): {100 * busy / (t1 - t0):.1f} %, "
             f"idle {(t1 - t0 - busy) / n / 1e3:.2f} us/step"]
    for name, tr in (("rank 0 (driver)", r0), ("rank 1 (worker)", r1)):
        w = [k for k in tr if t0 <= k[0] < t1]
        gaps = sorted(b[0] - a[1] for a, b in zip(w, w[1:]))
        big = [x for x in gaps if x > 20_000]
        lines.append(f"{name}: {len(w)} kernels ({len(w) / n:.0f}/step), own busy "
                     f"{100 * sum(e - s for s, e, _ in w) / (t1 - t0):.1f} %, gaps > 20 us: {len(big)} "
                     f"({len(big) / n:.2f}/step, max {max(gaps) / 1e3 if gaps else 0:.1f} us)")
    txt = "\n".join(lines)
    print(txt)
    if len(argv) > 2:
        with open(argv[2], "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main(sys.argv[1:])
