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
import statistics


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
                    help="add these kernels to profiles/pmc_summary.json (replacing same-name entries) instead of "
                         "overwriting it: e.g. the N > 1 shard kernels beside C2's pair kernel")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "profiles"))
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    stats = glob.glob(os.path.join(args.trace, "*_kernel_stats.csv"))
    if stats:
        shutil.copy(stats[0], os.path.join(args.out, f"{args.tag}_kernel_stats.csv"))
    fetch = {}
    for r in _rows(os.path.join(args.fetch, "*_counter_collection.csv")):
        if r["Counter_Name"] == "FETCH_SIZE":
            fetch.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    write = {}
    for r in _rows(os.path.join(args.write, "*_counter_collection.csv")):
        if r["Counter_Name"] == "WRITE_SIZE":
            write.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    durations = {}
    if stats:
        for r in _rows(stats[0]):
            durations[r["Name"]] = dict(calls=int(r["Calls"]), avg_ns=float(r["AverageNs"]),
                                        min_ns=float(r["MinNs"]), max_ns=float(r["MaxNs"]))
    kernels = []
    for name in sorted(set(fetch) | set(write)):
        f_kib = statistics.median(fetch.get(name, [0.0]))
        w_kib = statistics.median(write.get(name, [0.0]))
        kernels.append({
            "kernel": name,
            "launches_profiled": max(len(fetch.get(name, [])), len(write.get(name, []))),
            "fetch_size_kib_median": f_kib,
            "write_size_kib_median": w_kib,
            "hbm_read_bytes_per_launch": int(round(2 * f_kib * 1024)),
            "hbm_write_bytes_per_launch": int(round(w_kib * 1024)),
            "hbm_bytes_per_launch": int(round(2 * f_kib * 1024 + w_kib * 1024)),
            "trace": durations.get(name),
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
        # same instantiation = same name up to the parameter list (a kernel whose arguments changed replaces
        # its old entry instead of standing beside it)
        names = {k["kernel"].split("(")[0] for k in kernels}
        merged["kernels"] = [k for k in merged["kernels"] if k["kernel"].split("(")[0] not in names] + kernels
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
