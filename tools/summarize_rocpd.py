#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace run stored as its SQLite database (rocprofv3's default output on ROCm 7.2)
into the committed profile artefacts.

  python tools/summarize_rocpd.py gpurun_out/prof_r3/run_results.db profiles/r3 [bench_line.json]
  python tools/summarize_rocpd.py gpurun_out/prof/run_kernel_trace.csv profiles/r3/... [bench_line.json]

Writes <dst>/kernel_stats.csv (per kernel: calls, total / average / min / max duration in ns, the columns of
rocprofv3 --stats) and <dst>/trace_roofline.json: for the headline transform kernels (ntt_tw_body_kernel at the
8192-polynomial grid) the trace's average launch duration, the HBM roofline fraction it implies
(268,435,456 algorithmic bytes per launch / 8 TB/s), and, when the bench line of the same command is given, that
line's roofline.frac and the relative difference.
"""
import csv
import json
import os
import sqlite3
import sys
from collections import defaultdict

ALG_BYTES = 8192 * 2048 * 8 * 2  # one N = 2048, batch-8192 pass: read + write in place
PEAK = 8.0e12
HEAD_GRID = 8192 * 64  # lanes of the headline launches (both directions)


def is_fwd(name):
    """ntt_tw_body_kernel<true> / <true, false> (r5: the PERSIST parameter) or its mangled form."""
    return "<true" in name or "ILb1E" in name


def main():
    db, dst = sys.argv[1], sys.argv[2]
    line = json.load(open(sys.argv[3])) if len(sys.argv) > 3 else None
    os.makedirs(dst, exist_ok=True)
    if db.endswith(".csv"):  # rocprofv3 --output-format csv: <prefix>_kernel_trace.csv
        with open(db, newline="") as f:
            rows = sorted(((r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), int(r["Grid_Size_X"]),
                            int(r["Start_Timestamp"])) for r in csv.DictReader(f)), key=lambda t: t[3])
    else:
        c = sqlite3.connect(db)
        rows = c.execute("select name, duration, grid_x, start from kernels order by start").fetchall()
    stats = defaultdict(list)
    for name, dur, grid, _ in rows:
        stats[name].append((int(dur), int(grid)))
    total_all = sum(d for v in stats.values() for d, _ in v)
    with open(os.path.join(dst, "kernel_stats.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, v in sorted(stats.items(), key=lambda kv: -sum(d for d, _ in kv[1])):
            ds = [d for d, _ in v]
            w.writerow([name, len(ds), sum(ds), sum(ds) / len(ds), 100.0 * sum(ds) / total_all, min(ds), max(ds)])
    head = {}
    for name, v in stats.items():
        if "ntt_tw_body_kernel" not in name:
            continue
        ds = [d for d, g in v if g == HEAD_GRID]  # the headline batch: 8192 one-wave / 2048 four-wave workgroups
        if not ds:
            continue
        avg = sum(ds) / len(ds)
        head["fwd" if is_fwd(name) else "inv"] = {
            "kernel": name, "launches": len(ds), "average_ns": avg, "min_ns": min(ds),
            "achieved_GBps": ALG_BYTES / (avg * 1e-9) / 1e9, "frac": ALG_BYTES / (avg * 1e-9) / PEAK}
    out = {"source": os.path.basename(db), "headline_kernels": head}
    if line:
        # bench.py's launch order for the transform at the headline grid: cold start (W warmup + K timed steps),
        # the legs (other kernels), the headline (W warmup + K timed steps), steady state, the direction split
        W, K = line["warmup"], line["steps"]
        # runs of consecutive dispatches alternating forward / inverse body at the headline grid (the split-transform
        # and large-PBS launches of the legs use the same kernels, never in that alternation): the first run of
        # >= 2 (W + K) launches is the cold start, the second the headline (then the steady-state loop)
        runs, cur = [], []
        for name, d, g, _ in rows:
            kind = ("fwd" if is_fwd(name) else "inv") if "ntt_tw_body_kernel" in name and g == HEAD_GRID else None
            if kind and (not cur or cur[-1][0] != kind):
                cur.append((kind, d))
                continue
            if len(cur) >= 2 * (W + K):
                runs.append(cur)
            cur = [(kind, d)] if kind else []
        if len(cur) >= 2 * (W + K):
            runs.append(cur)
        timed = [d for _, d in runs[1][2 * W: 2 * W + 2 * K]]
        avg_t = sum(timed) / len(timed)
        out["headline_timed_launches"] = {
            "launches": len(timed), "average_ns": avg_t, "frac": ALG_BYTES / (avg_t * 1e-9) / PEAK,
            "note": "the 2 K launches of the headline's timed region, picked by dispatch order; kernel durations "
                    "only (the bench line's event interval also holds the gaps between launches)"}
        out["bench_line_frac"] = line["roofline"]["frac"]
        out["timed_relative_difference"] = out["headline_timed_launches"]["frac"] / line["roofline"]["frac"] - 1.0
    if len(head) == 2:
        avg2 = (head["fwd"]["average_ns"] * head["fwd"]["launches"] + head["inv"]["average_ns"] * head["inv"]["launches"]) / (
            head["fwd"]["launches"] + head["inv"]["launches"])
        out["both_directions"] = {"average_ns": avg2, "frac": ALG_BYTES / (avg2 * 1e-9) / PEAK}
        out["both_directions"]["note"] = "every launch at the headline grid: cold start, headline, the >= 1 s steady-state loop"
    with open(os.path.join(dst, "trace_roofline.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
