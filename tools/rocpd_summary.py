"""Summarise a rocprofv3 --kernel-trace database (rocpd SQLite, `*_results.db`) per (kernel, launch shape):
calls, mean / median / min duration (us), VGPRs and scratch bytes. One launch shape = one configuration of
tools/bench_configs.py, so the rows line up with its JSON lines (the time per launch there comes from HIP
events; here from the profiler's own dispatch timestamps).

    python tools/rocpd_summary.py gpurun_out/cfgprof/run_results.db > profiles/archive/r01_configs_kernel_stats.csv
"""
import csv
import sqlite3
import statistics
import sys


def short(name: str) -> str:
    return name.replace("fmi::dev::", "").replace("void ", "").split("(")[0]


def main(path: str) -> None:
    db = sqlite3.connect(path)
    rows = db.execute("select name, grid_x, workgroup_x, duration, vgpr_count, scratch_size from kernels").fetchall()
    groups = {}
    for name, grid, wg, dur, vgpr, scratch in rows:
        groups.setdefault((short(name), grid, wg, vgpr, scratch), []).append(dur / 1e3)
    out = csv.writer(sys.stdout)
    out.writerow(["kernel", "grid_threads", "workgroup", "vgprs", "scratch_bytes", "calls", "mean_us", "median_us",
                  "min_us"])
    for (name, grid, wg, vgpr, scratch), d in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        out.writerow([name, grid, wg, vgpr, scratch, len(d), round(statistics.fmean(d), 2),
                      round(statistics.median(d), 2), round(min(d), 2)])


if __name__ == "__main__":
    main(sys.argv[1])
