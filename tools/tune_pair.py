"""Sweep the pairwise kernel's launch variants on C2 (256 MiB f32 sum), interleaved in one process
(cdna_hip_programming.md §5.4 rule 24). Prints one JSON line per variant: median/min µs and GB/s of
algorithmic traffic (3 · 256 MiB per launch)."""
import argparse
import itertools
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import fmi_amd  # noqa: E402
from fmi_amd import Bucket, Event, Op, Tune  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dtype", default="f32")
    args = ap.parse_args()
    dt = {"f32": np.float32, "f64": np.float64, "i32": np.int32, "i64": np.int64}[args.dtype]
    fmi_amd.init(0)
    n = args.mib * (1 << 20) // np.dtype(dt).itemsize
    sets = [(Bucket(n, dt).fill_synthetic(42 + s, 0), Bucket(n, dt).fill_synthetic(42 + s, 1)) for s in range(4)]
    variants = []
    for v, u, b in itertools.product((0, 2, 3, 4), (1, 2, 4, 8), (256, 512, 1024)):
        variants.append(dict(variant=v, unroll=u, block=b, grid_per_cu=0))
    for u, b, g in itertools.product((2, 4, 8), (256, 512), (2, 4, 8, 16)):
        variants.append(dict(variant=1, unroll=u, block=b, grid_per_cu=g))
    times = {i: [] for i in range(len(variants))}
    ev = [Event() for _ in range(2 * args.iters)]
    for _ in range(args.rounds):
        for i, cfg in enumerate(variants):
            fmi_amd.tune_set(Tune.PAIR_VARIANT, cfg["variant"])
            fmi_amd.tune_set(Tune.PAIR_UNROLL, cfg["unroll"])
            fmi_amd.tune_set(Tune.BLOCK, cfg["block"])
            if cfg["grid_per_cu"]:
                fmi_amd.tune_set(Tune.GRID_PER_CU, cfg["grid_per_cu"])
            for k in range(3):
                a, b = sets[k % 4]
                fmi_amd.reduce_pair(Op.SUM, a, b)
            for k in range(args.iters):
                a, b = sets[k % 4]
                ev[2 * k].record()
                fmi_amd.reduce_pair(Op.SUM, a, b)
                ev[2 * k + 1].record()
            fmi_amd.sync()
            times[i] += [ev[2 * k].elapsed_ms(ev[2 * k + 1]) for k in range(args.iters)]
    nbytes = 3 * n * np.dtype(dt).itemsize
    rows = []
    for i, cfg in enumerate(variants):
        med = statistics.median(times[i])
        rows.append(dict(cfg, median_us=round(med * 1e3, 2), min_us=round(min(times[i]) * 1e3, 2),
                         gbs=round(nbytes / (med * 1e-3) / 1e9, 1)))
    rows.sort(key=lambda r: r["median_us"])
    for r in rows:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
