"""Per-kernel launch statistics from a rocprofv3 `--kernel-trace --output-format csv` run: calls, median, mean
and min duration (us) per kernel name, as JSON lines sorted by name.

    python tools/trace_medians.py gpurun_out/tp [name-substring]
"""
import csv
import glob
import json
import os
import statistics
import sys


def main(path: str, sub: str = "") -> None:
    if os.path.isdir(path):  # the rocprofv3 output directory: its (one) kernel-trace CSV
        path = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))[0]
    groups = {}
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            if sub and sub not in name:
                continue
            dur = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3
            groups.setdefault(name.replace("fmi::dev::", "").split("(")[0], []).append(dur)
    for name in sorted(groups):
        d = groups[name]
        print(json.dumps({"kernel": name, "calls": len(d), "median_us": round(statistics.median(d), 2),
                          "mean_us": round(statistics.fmean(d), 2), "min_us": round(min(d), 2)}))


if __name__ == "__main__":
    main(*sys.argv[1:])
