"""The LOCAL transport's exchange, host-synchronised against ordered on the streams (FMI_TUNE_COMM_LOCAL_ASYNC 0 / 1),
on C5's co-resident block (bench.py c5_local_peers: 8 LOCAL ranks x 1 GiB page-locked host buckets through
fmi_comm_allreduce_host), interleaved `--reps` times in one process, each run self-checked. One JSON line per run.

  python tools/local_async_ab.py [--reps 3] [--mib 1024]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
import fmi_amd  # noqa: E402
from fmi_amd import Tune  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--mib", type=int, default=1024)
    a = ap.parse_args()
    fmi_amd.init(0)
    old = fmi_amd.tune_get(Tune.COMM_LOCAL_ASYNC)
    bad = 0
    try:
        for rep in range(a.reps):
            for mode in ((1, 0) if rep % 2 == 0 else (0, 1)):
                fmi_amd.tune_set(Tune.COMM_LOCAL_ASYNC, mode)
                bench.quiet_device()
                r = bench.c5_local_peers(8, a.mib)
                ok = r["self_check"]["ok"]
                bad += not ok
                print(json.dumps({"rep": rep, "local_async": mode, "ms": r["ms"],
                                  "pcie_GB_s": r["pcie_GB_s_both_directions"], "ok": ok}), flush=True)
    finally:
        fmi_amd.tune_set(Tune.COMM_LOCAL_ASYNC, old)
    if bad:
        raise SystemExit(f"{bad} runs failed their self-check")


if __name__ == "__main__":
    main()
