"""A/B of FMI_TUNE_FUSED_INFLIGHT_KIB on the fused P-way kernels through the library (C3 shapes: P = 8 × 64 MiB
f32 scan / tree; tree P = 2, 4, 16 over 1 GiB), interleaved in one process over several rounds. Prints one
JSON object per (round, budget, kernel): median µs over the iterations and the fraction of the 8 TB/s peak."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import fmi_amd  # noqa: E402
from fmi_amd import Alg, Bucket, Event, Op, Tune  # noqa: E402

MIB = 1 << 20


def timed(fn, iters, rotate):
    ev = [(Event(), Event()) for _ in range(iters)]
    for k in range(3):
        fn(k % rotate)
    fmi_amd.sync()
    for k in range(iters):
        ev[k][0].record()
        fn(k % rotate)
        ev[k][1].record()
    fmi_amd.sync()
    return statistics.median(a.elapsed_ms(b) for a, b in ev)


def main():
    caps = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "0,96,64,128").split(",")]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    fmi_amd.init(0)
    P, n = 8, 64 * MIB // 4
    ins = [[Bucket(n, np.float32).fill_synthetic(42 + s, p) for p in range(P)] for s in range(2)]
    outs = [Bucket(n, np.float32) for _ in range(P)]
    out = Bucket(n, np.float32)
    wide = {P2: ([Bucket(1024 * MIB // 4 // P2, np.float32).fill_synthetic(7, p) for p in range(P2)],
                 Bucket(1024 * MIB // 4 // P2, np.float32)) for P2 in (2, 4, 16)}
    cases = [
        ("scan f32 P=8 x 64MiB", 2 * P * 64 * MIB, lambda k: fmi_amd.scan_peers(Op.SUM, Alg.SCAN, outs, ins[k]), 2),
        ("scan_ltr f32 P=8 x 64MiB", 2 * P * 64 * MIB,
         lambda k: fmi_amd.scan_peers(Op.SUM, Alg.SCAN_LTR, outs, ins[k]), 2),
        ("tree allreduce f32 P=8 x 64MiB", (P + 1) * 64 * MIB,
         lambda k: fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, out, ins[k]), 2),
        ("tree reduce_ltr f32 P=8 x 64MiB", (P + 1) * 64 * MIB,
         lambda k: fmi_amd.reduce_tree(Op.SUM, Alg.REDUCE_LTR, out, ins[k]), 2),
    ]
    for P2, (ins2, out2) in wide.items():
        cases.append((f"tree allreduce f32 P={P2} x {1024 // P2}MiB", (P2 + 1) * (1024 // P2) * MIB,
                      lambda k, i=ins2, o=out2: fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, o, i), 1))
    for r in range(rounds):
        for cap in caps:
            fmi_amd.tune_set(Tune.FUSED_INFLIGHT_KIB, cap)
            for name, nbytes, fn, rot in cases:
                ms = timed(fn, 20, rot)
                gbs = nbytes / (ms * 1e-3) / 1e9
                print(json.dumps({"round": r, "inflight_kib": cap, "kernel": name, "us": round(ms * 1e3, 2),
                                  "GB_s": round(gbs, 1), "frac": round(gbs / 8000.0, 4)}), flush=True)


if __name__ == "__main__":
    main()
