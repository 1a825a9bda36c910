"""How the production pairwise kernel's time scales with bucket size (is config C3's
64 MiB i64 max bound by streaming rate or by a fixed per-launch cost?).

For i64 max and f32 sum at 8 … 512 MiB per bucket, times fmi_dev_reduce_pair launch by launch (an event pair
around each launch on the library stream) over rotating buffer sets whose footprint exceeds the 256 MB
MALL, sizes interleaved over several rounds; reports the median per size and a least-squares fit
t = t0 + bytes / R over the sizes (t0: fixed cost per launch, R: asymptotic streaming rate).

    python tools/pair_size_scaling.py [--rounds 3] [--launches 60]
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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--launches", type=int, default=60)
    ap.add_argument("--sizes", default="8,16,32,64,128,256,512")
    args = ap.parse_args()
    import fmi_amd
    from fmi_amd import Bucket, Op
    from fmi_amd.device import Event, reduce_pair

    fmi_amd.init(0)
    sizes = [int(s) for s in args.sizes.split(",")]
    cases = [("i64_max", np.int64, Op.MAX), ("f32_sum", np.float32, Op.SUM)]
    times = {(c[0], m): [] for c in cases for m in sizes}
    for rnd in range(args.rounds):
        for name, dtype, op in cases:
            for mib in sizes:
                n = mib * MIB // np.dtype(dtype).itemsize
                sets = max(2, -(-1536 // (2 * mib)))  # >= 1.5 GiB of buckets
                bufs = [(Bucket(n, dtype).fill_synthetic(s, 0), Bucket(n, dtype).fill_synthetic(s, 1)) for s in range(sets)]
                for s in range(sets):  # warm
                    reduce_pair(op, *bufs[s])
                ev = [(Event(), Event()) for _ in range(args.launches)]
                for k in range(args.launches):
                    a, b = bufs[k % sets]
                    ev[k][0].record()
                    reduce_pair(op, a, b)
                    ev[k][1].record()
                fmi_amd.sync()
                times[(name, mib)].extend(e0.elapsed_ms(e1) * 1e3 for e0, e1 in ev)
                for e0, e1 in ev:
                    e0.destroy()
                    e1.destroy()
                for a, b in bufs:
                    a.free()
                    b.free()
    for name, _, _ in cases:
        xs, ys = [], []
        for mib in sizes:
            med = statistics.median(times[(name, mib)])
            algo = 3 * mib * MIB
            xs.append(algo)
            ys.append(med)
            print(json.dumps({"case": name, "mib_per_bucket": mib, "median_us": round(med, 2),
                              "algorithmic_bytes": algo, "TB_s": round(algo / med / 1e6, 3),
                              "frac_of_8TBs": round(algo / med / 1e6 / 8.0, 4), "launches": len(times[(name, mib)])}),
                  flush=True)
        slope, t0 = np.polyfit(np.array(xs, dtype=np.float64), np.array(ys), 1)
        print(json.dumps({"case": name, "fit": "t = t0 + bytes / R", "t0_us": round(float(t0), 3),
                          "R_TB_s": round(1.0 / float(slope) / 1e6, 3),
                          "c3_predicted_us": round(float(t0 + slope * 3 * 64 * MIB), 2)}), flush=True)


if __name__ == "__main__":
    main()
