"""A/B of the pairwise kernel's sc1 tiles through the library (FMI_TUNE_PAIR_SC1_OF_8), in bench.py's own
configuration: in-place combines a = a + b of separately allocated buckets, K back-to-back launches over
rotating sets between two events on the library stream, budgets interleaved over rounds; for several
bucket sizes and rotating-set counts. Also checks that every budget gives identical bits.

    python tools/ab_pair_sc1.py [--rounds 5] [--mib 64,256] [--sets 2,4] [--budgets 0,1,2,4]

Rotating sets: the sc1 tiles' lines stay in the 256 MB MALL (nontemporal reads do not displace them), so a
set re-read within ~256 MB of sc1 writes partly hits the MALL — use enough sets that it cannot (sets x
sc1 bytes per launch >> 256 MB) to measure the combine itself (profiles/archive/r02_ab_pair_sc1_*).
"""
import argparse
import json
import os
import statistics
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
MIB = 1 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--mib", default="64,256")
    ap.add_argument("--sets", default="4")
    ap.add_argument("--dtype", default="f32", choices=["f32", "i64"])
    ap.add_argument("--budgets", default="0,1,2,4", help="FMI_TUNE_PAIR_SC1_OF_8 values")
    ap.add_argument("--launches", type=int, default=20)
    args = ap.parse_args()
    import fmi_amd
    from fmi_amd import Bucket, Event, Op
    from fmi_amd.device import Tune, tune_get, tune_set

    fmi_amd.init(0)
    dtype, op = (np.float32, Op.SUM) if args.dtype == "f32" else (np.int64, Op.MAX)
    budgets = [int(b) for b in args.budgets.split(",")]
    default = tune_get(Tune.PAIR_SC1_OF_8)
    for mib in [int(m) for m in args.mib.split(",")]:
        n = mib * MIB // np.dtype(dtype).itemsize
        for nsets in [int(s) for s in args.sets.split(",")]:
            sets = [(Bucket(n, dtype).fill_synthetic(42 + s, 0), Bucket(n, dtype).fill_synthetic(42 + s, 1))
                    for s in range(nsets)]
            # identical bits for every budget (on a fresh copy of set 0's first bucket)
            ref = None
            for b in budgets:
                tune_set(Tune.PAIR_SC1_OF_8, b)
                a = Bucket(n, dtype).fill_synthetic(42, 0)
                fmi_amd.reduce_pair(op, a, sets[0][1])
                got = a.numpy().tobytes()
                a.free()
                assert ref is None or got == ref, f"budget {b} changed the result"
                ref = got
            times = {b: [] for b in budgets}
            pos = 0  # one running position over the sets: every set is re-used exactly nsets launches later

            def launch():
                nonlocal pos
                fmi_amd.reduce_pair(op, *sets[pos % nsets])
                pos += 1

            for _ in range(args.rounds):
                for b in budgets:
                    tune_set(Tune.PAIR_SC1_OF_8, b)
                    for k in range(3):
                        launch()
                    e0, e1 = Event(), Event()
                    e0.record()
                    for k in range(args.launches):
                        launch()
                    e1.record()
                    e1.sync()
                    times[b].append(e0.elapsed_ms(e1) * 1e3 / args.launches)
                    e0.destroy()
                    e1.destroy()
            for b in budgets:
                us = statistics.median(times[b])
                frac = 3 * mib * MIB / (us * 1e-6) / 8e12
                print(json.dumps({"dtype": args.dtype, "mib": mib, "sets": nsets, "sc1_of_8": b, "median_us": round(us, 2),
                                  "min_us": round(min(times[b]), 2), "frac": round(frac, 4), "bit_identical": True}),
                      flush=True)
            for a, b in sets:
                a.free()
                b.free()
    tune_set(Tune.PAIR_SC1_OF_8, default)


if __name__ == "__main__":
    main()
