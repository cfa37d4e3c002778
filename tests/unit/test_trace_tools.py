"""The rocprofv3 trace readers behind the round-6 evidence (tools/wave_gaps.py, idle gaps inside a
bench wave; tools/overlap_report.py, comm-stream kernels concurrent with the compute stream) on
synthetic kernel traces with known answers."""
import csv
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _load(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "tools", f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _trace(tmp_path, rows):
    d = tmp_path / "trace" / "run"
    d.mkdir(parents=True)
    with open(d / "1_kernel_trace.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Stream_Id"])
        w.writeheader()
        for name, b, e, s in rows:
            w.writerow({"Kernel_Name": name, "Start_Timestamp": b, "End_Timestamp": e, "Stream_Id": s})
    return str(tmp_path / "trace")


def test_wave_gaps_finds_the_gaps_of_the_last_wave(tmp_path, capsys):
    us = 1000  # timestamps in ns
    rows, t = [], 0
    # a warm-up wave of three steps, a long idle gap (in the trace's second half, where the tool
    # looks for it), then the measured wave: two steps (sample_kernel ends a step)
    for name, dur, gap in [("embedding_kernel", 5, 1), ("gemm", 50, 1), ("sample_kernel<float>", 5, 1)] * 3:
        rows.append((name, t, t + dur * us, 0))
        t += (dur + gap) * us
    t += 100000 * us
    for name, dur, gap in [("copy_from_host_kernel", 5, 40), ("embedding_kernel", 5, 2), ("gemm", 50, 1),
                           ("sample_kernel<float>", 5, 25), ("embedding_kernel", 5, 1), ("gemm", 50, 1),
                           ("sample_kernel<float>", 5, 0)]:
        rows.append((name, t, t + dur * us, 0))
        t += (dur + gap) * us
    wg = _load("wave_gaps")
    out = tmp_path / "gaps.md"
    wg.main([_trace(tmp_path, rows), "10", str(out)])
    text = out.read_text()
    assert "2 gaps > 10 us summing 0.07 ms" in text, text
    assert "step 0: 40.0 us, `copy_from_host_kernel` -> `embedding_kernel`" in text
    assert "step 1: 25.0 us, `sample_kernel<float>` -> `embedding_kernel`" in text


def test_overlap_report_measures_comm_stream_concurrency(tmp_path):
    us = 1000
    rows = [("Cijk_gemm_a", 0, 100 * us, 0), ("rmsnorm", 100 * us, 110 * us, 0), ("Cijk_gemm_b", 110 * us, 210 * us, 0),
            # on the comm stream: 20 us inside gemm_a, then 20 us half inside gemm_b, half after it
            ("allreduce_2shot<2>", 40 * us, 60 * us, 4), ("allreduce_2shot<2>", 200 * us, 220 * us, 4)]
    ov = _load("overlap_report")
    out = tmp_path / "ov.md"
    ov.main([_trace(tmp_path, rows), str(out)])
    text = out.read_text()
    line = next(l for l in text.splitlines() if l.startswith("| 4 | `allreduce_2shot<2>`"))
    cells = [c.strip() for c in line.strip("|").split("|")]
    # calls, total us, overlapped us, %, calls overlapping a main-stream GEMM
    assert cells[2:] == ["2", "40.0", "30.0", "75", "2"], cells
