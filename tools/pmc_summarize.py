"""Summarise rocprofv3 runs of bench.py into profiles/ (committed evidence).

Inputs (from a gpurun call):
  <trace_dir>/*_kernel_stats.csv        rocprofv3 --kernel-trace --stats
  <fetch_dir>/*_counter_collection.csv  rocprofv3 --pmc FETCH_SIZE --kernel-trace   (own pass)
  <write_dir>/*_counter_collection.csv  rocprofv3 --pmc WRITE_SIZE --kernel-trace   (own pass)

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports exactly half the bytes of a wide (16 B/lane) coalesced streaming read, so it is
doubled; WRITE_SIZE is exact for 16 B/lane streaming stores.
"""
import argparse
import csv
import glob
import json
import os
import shutil
import re
import statistics


def algorithmic_bytes(kernel: str, write_bytes: float):
    """Algorithmic HBM bytes of one launch, from the launch's output bytes, which every
    kernel here writes exactly once: pair a = a (+) b reads 2 and writes 1 bucket (3 x out); the fused P-way
    tree reads P buckets and writes one (P + 1 x out); the peer-axis scan reads P and writes P (2 x out); the
    synthetic-input generator only writes (1 x out); a buffer copy (the runtime's, or the library's copy_tile)
    reads and writes (2 x out). The output is
    rounded to whole 4 KiB pages first (a WRITE_SIZE median carries a few hundred stray bytes). None for a
    kernel of another shape."""
    out = round(write_bytes / 4096) * 4096
    m = re.search(r"tree_kernel<[^,]+, [^,]+, \d+, (\d+),", kernel)
    if m:
        return (int(m.group(1)) + 1) * out
    if "pair_tile<" in kernel or "pair_stride<" in kernel:
        return 3 * out
    if "scan_kernel<" in kernel:
        return 2 * out
    if "synth_kernel<" in kernel:
        return out
    if "copyBuffer" in kernel or "copy_tile<" in kernel:
        return 2 * out
    return None


def same_launch(a: dict, b: dict) -> bool:
    """Two PMC entries describe the same launch: the same instantiation (name up to the parameter list) AND
    the same algorithmic bytes — the N = 8 shard tree (32 MiB shards) and C3's 8-peer tree (64 MiB buckets)
    are one instantiation at two shapes and must both stay."""
    return (a["kernel"].split("(")[0] == b["kernel"].split("(")[0]
            and a.get("algorithmic_bytes_per_launch") == b.get("algorithmic_bytes_per_launch"))


def _rows(path_glob):
    out = []
    for p in glob.glob(path_glob):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--tag", required=True, help="e.g. r01_c2")
    ap.add_argument("--command", required=True)
    ap.add_argument("--no-default", action="store_true",
                    help="do not overwrite profiles/pmc_summary.json (the file bench.py reads for C2)")
    ap.add_argument("--merge", action="store_true",
                    help="add these kernels to profiles/pmc_summary.json (replacing entries of the same instantiation "
                         "and shape) instead of "
                         "overwriting it: e.g. the N > 1 shard kernels beside C2's pair kernel")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "profiles"))
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    stats = glob.glob(os.path.join(args.trace, "*_kernel_stats.csv"))
    if stats:
        shutil.copy(stats[0], os.path.join(args.out, f"{args.tag}_kernel_stats.csv"))
    # Launches are grouped by (kernel, grid size): one instantiation launched at several shapes in one run
    # (copy_tile at 256 MiB and at the 64 MiB host-pipeline chunks) gives one entry per shape, never a median
    # across shapes.
    def grid_of(r):
        if "Grid_Size" in r:
            return int(float(r["Grid_Size"]))
        return int(float(r["Grid_Size_X"])) * int(float(r["Grid_Size_Y"])) * int(float(r["Grid_Size_Z"]))

    fetch, write = {}, {}
    for r in _rows(os.path.join(args.fetch, "*_counter_collection.csv")):
        if r["Counter_Name"] == "FETCH_SIZE":
            fetch.setdefault((r["Kernel_Name"], grid_of(r)), []).append(float(r["Counter_Value"]))
    for r in _rows(os.path.join(args.write, "*_counter_collection.csv")):
        if r["Counter_Name"] == "WRITE_SIZE":
            write.setdefault((r["Kernel_Name"], grid_of(r)), []).append(float(r["Counter_Value"]))
    durations = {}
    traces = glob.glob(os.path.join(args.trace, "*_kernel_trace.csv"))
    if traces:
        per = {}
        for r in _rows(traces[0]):
            per.setdefault((r["Kernel_Name"], grid_of(r)), []).append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
        for key, ns in per.items():
            durations[key] = dict(calls=len(ns), avg_ns=statistics.fmean(ns), median_ns=statistics.median(ns),
                                  min_ns=min(ns), max_ns=max(ns), source="kernel_trace.csv, this shape")
    elif stats:
        for r in _rows(stats[0]):
            durations[(r["Name"], None)] = dict(calls=int(r["Calls"]), avg_ns=float(r["AverageNs"]),
                                                min_ns=float(r["MinNs"]), max_ns=float(r["MaxNs"]),
                                                source="kernel_stats.csv, every shape of this kernel")
    kernels = []
    for name, grid in sorted(set(fetch) | set(write)):
        f_kib = statistics.median(fetch.get((name, grid), [0.0]))
        w_kib = statistics.median(write.get((name, grid), [0.0]))
        kernels.append({
            "kernel": name,
            "grid_size": grid,
            "launches_profiled": max(len(fetch.get((name, grid), [])), len(write.get((name, grid), []))),
            "fetch_size_kib_median": f_kib,
            "write_size_kib_median": w_kib,
            "hbm_read_bytes_per_launch": int(round(2 * f_kib * 1024)),
            "hbm_write_bytes_per_launch": int(round(w_kib * 1024)),
            "hbm_bytes_per_launch": int(round(2 * f_kib * 1024 + w_kib * 1024)),
            "algorithmic_bytes_per_launch": algorithmic_bytes(name, w_kib * 1024),
            "trace": durations.get((name, grid)) or durations.get((name, None)),
        })
    summary = {
        "source": f"profiles/{args.tag}: rocprofv3 separate --pmc FETCH_SIZE / --pmc WRITE_SIZE passes, "
                  "FETCH_SIZE x2 (gfx950 wide-read correction, MI355X_MICROARCH.md §HBM)",
        "command": args.command,
        "kernels": kernels,
    }
    for k in kernels:  # each entry names its own source once summaries are merged
        k["source"] = summary["source"]
    default = os.path.join(args.out, "pmc_summary.json")
    if args.merge and os.path.exists(default):
        merged = json.load(open(default))
        # an entry is replaced only by a profile of the same launch (instantiation AND shape, same_launch);
        # the same instantiation at another shape stands beside it
        merged["kernels"] = [k for k in merged["kernels"] if not any(same_launch(k, n) for n in kernels)] + kernels
        merged.setdefault("merged", []).append({"source": summary["source"], "command": args.command})
        with open(default, "w") as f:
            json.dump(merged, f, indent=1)
    elif not args.no_default:
        with open(default, "w") as f:
            json.dump(summary, f, indent=1)
    with open(os.path.join(args.out, f"{args.tag}_pmc_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
