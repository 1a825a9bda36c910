"""Summarise the --pmc passes of `bash tools/gpu_round5.sh b` (tools/tree8_shapes.py under rocprofv3, one pass per
counter group) into one JSON: per tree_kernel launch shape (MiB per peer), the mean of every counter over its
launches, and the ratios that could separate the shapes — average read / write latency at the L2's memory side
(TCC_EA0_RDREQ_LEVEL / TCC_EA0_RDREQ, cycles), DRAM credit and tag stalls per request, UTCL1 translation misses
and UTCL2 busy per byte, TA stalls and GUI-active cycles per byte, and HBM traffic against the algorithmic bytes
(FETCH_SIZE x 2 on gfx950, WRITE_SIZE; MI355X_MICROARCH.md).

  python tools/tree8_pmc_summary.py gpurun_out/r05_tree8_pmc > profiles/r05_tree8_pmc_summary.json
"""
import collections
import csv
import glob
import json
import sys


def main(prefix: str) -> None:
    mean = collections.defaultdict(dict)
    for f in sorted(glob.glob(prefix + "*/run_counter_collection.csv")):
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if "tree_kernel" in r["Kernel_Name"]:
                acc[(int(r["Grid_Size"]) * 16 >> 20, r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (mib, name), v in acc.items():
            key = name if name != "GRBM_GUI_ACTIVE" else f"GRBM_GUI_ACTIVE[{f.split('/')[-2]}]"
            mean[mib][key] = sum(v) / len(v)
    out = {"source": prefix + "*/run_counter_collection.csv", "kernel": "tree_kernel<OpSum, float, 0, 8, false>",
           "shapes": {}}
    for mib, c in sorted(mean.items()):
        gib = mib / 1024
        algo = 9 * mib * (1 << 20)
        gui = [v for k, v in c.items() if k.startswith("GRBM_GUI_ACTIVE")]
        row = {"counters": {k: round(v) for k, v in sorted(c.items())},
               "read_latency_cycles": round(c["TCC_EA0_RDREQ_LEVEL_sum"] / c["TCC_EA0_RDREQ_sum"], 1),
               "write_latency_cycles": round(c["TCC_EA0_WRREQ_LEVEL_sum"] / c["TCC_EA0_WRREQ_sum"], 1),
               "dram_read_credit_stall_per_req": round(c["TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"] / c["TCC_EA0_RDREQ_sum"], 4),
               "tag_stall_per_req": round(c["TCC_TAG_STALL_sum"] / c["TCC_EA0_RDREQ_sum"], 4),
               "utcl1_misses_per_gib": round(c["TCP_UTCL1_TRANSLATION_MISS_sum"] / gib),
               "ta_data_stalled_per_gib": round(c["TA_DATA_STALLED_BY_TC_CYCLES_sum"] / gib),
               "tcc_busy_per_gib": round(c["TCC_BUSY_sum"] / gib),
               "gui_active_per_gib_mean_over_passes": round(sum(gui) / len(gui) / gib),
               "hbm_bytes_over_algorithmic": round((c["FETCH_SIZE"] * 2 + c["WRITE_SIZE"]) * 1024 / algo, 6)}
        out["shapes"][str(mib)] = row
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
