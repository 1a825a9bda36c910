"""Attribute a rocprofv3 kernel trace of tools/placement_ab.py to its blocks (round 6).

The tool's JSON lines give each block's kernel (trace_name), warm-up and timed launch counts, in launch order; the
blocks of one kernel never interleave with other launches of that kernel, so the trace's launches of each kernel
name, in start order, split into consecutive blocks. For every block: the mean duration of its timed launches
(the warm-up ones dropped) and the fraction of 8 TB/s next to the in-process event figure. Prints JSON lines, then
a summary per (kernel, mode).

  python tools/placement_ab_trace.py gpurun_out/ab.jsonl gpurun_out/ab_trace   (a directory holding *kernel_trace.csv)
"""
import csv
import glob
import json
import os
import statistics
import sys

PEAK = 8e12
BYTES = {"pair": 3 * 256 << 20, "scan": 16 * 64 << 20, "tree": 9 * 1024 << 20, "copy": 2 * 256 << 20}


def main(lines_path: str, trace_dir: str) -> None:
    blocks = [json.loads(x) for x in open(lines_path) if x.startswith("{")]
    traces = glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True)
    if len(traces) != 1:
        raise SystemExit(f"expected one kernel trace under {trace_dir}, found {traces}")
    rows = sorted(csv.DictReader(open(traces[0])), key=lambda r: int(r["Start_Timestamp"]))
    by_name = {}
    for r in rows:
        by_name.setdefault(r["Kernel_Name"], []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    cursor = {}
    summary = {}
    for b in blocks:
        names = [k for k in by_name if b["trace_name"] in k]
        if len(names) != 1:
            raise SystemExit(f"kernel {b['trace_name']!r} matches {names}")
        durs = by_name[names[0]]
        i = cursor.get(names[0], 0)
        take = durs[i:i + b["warmup"] + b["steps"]][b["warmup"]:]
        cursor[names[0]] = i + b["warmup"] + b["steps"]
        if len(take) != b["steps"]:
            raise SystemExit(f"trace ran out of {names[0]} launches at block {b}")
        us = statistics.mean(take) / 1e3
        frac = BYTES[b["kernel"]] / (us * 1e-6) / PEAK
        row = {"kernel": b["kernel"], "mode": b["mode"], "rep": b["rep"], "trace_us": round(us, 2),
               "trace_frac": round(frac, 4), "events_us": b["us"], "events_frac": b["frac"]}
        print(json.dumps(row))
        summary.setdefault((b["kernel"], b["mode"]), []).append(row)
    for name, durs in by_name.items():
        for k, (n0, c) in enumerate(cursor.items()):
            if n0 == name and c != len(durs):
                print(json.dumps({"warning": f"{len(durs) - c} launches of {name} not attributed"}))
    for (k, m), rs in summary.items():
        print(json.dumps({"summary": k, "mode": m, "reps": len(rs),
                          "trace_frac_mean": round(statistics.mean(r["trace_frac"] for r in rs), 4),
                          "events_frac_mean": round(statistics.mean(r["events_frac"] for r in rs), 4),
                          "trace_frac_each": [r["trace_frac"] for r in rs]}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
