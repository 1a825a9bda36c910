"""A/B of the one-pass blocked scans (scan P = 32, 48, 64, 128, scan_ltr P = 64, 128 over 1 GiB of f32 input): against the blocked launches
(FMI_TUNE_BLOCKS_ONE_PASS = 0) and over the residency cap FMI_TUNE_FUSED_INFLIGHT_KIB (64 -> 2 workgroups per CU,
192 -> 3, 0 -> register-limited), interleaved in one process over several rounds. One JSON object per
(round, form, cap, P): median µs and fraction of the 8 TB/s peak (on the one-pass bytes, 2P buckets).
Usage: ab_scan_one_pass.py [caps, default 64] [rounds, default 3]"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import fmi_amd  # noqa: E402
from fmi_amd import Alg, Bucket, Event, Op, Tune  # noqa: E402

MIB = 1 << 20


def timed(fn, iters):
    ev = [(Event(), Event()) for _ in range(iters)]
    for _ in range(3):
        fn()
    fmi_amd.sync()
    for k in range(iters):
        ev[k][0].record()
        fn()
        ev[k][1].record()
    fmi_amd.sync()
    return statistics.median(a.elapsed_ms(b) for a, b in ev)


def main():
    caps = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "64").split(",")]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    fmi_amd.init(0)
    sets = {}
    for alg, P in ((Alg.SCAN, 32), (Alg.SCAN, 48), (Alg.SCAN, 64), (Alg.SCAN, 128), (Alg.SCAN_LTR, 64),
                   (Alg.SCAN_LTR, 128)):
        n = 1024 * MIB // 4 // P
        sets[(alg, P)] = ([Bucket(n, np.float32).fill_synthetic(7, p) for p in range(P)],
                          [Bucket(n, np.float32) for _ in range(P)], n)
    old = fmi_amd.tune_get(Tune.FUSED_INFLIGHT_KIB)
    for r in range(rounds):
        for cap in caps:
            fmi_amd.tune_set(Tune.FUSED_INFLIGHT_KIB, cap)
            for (alg, P), (ins, outs, n) in sets.items():
                for one_pass in (1, 0):
                    fmi_amd.tune_set(Tune.BLOCKS_ONE_PASS, one_pass)
                    ms = timed(lambda: fmi_amd.scan_peers(Op.SUM, alg, outs, ins), 10)
                    frac = 2 * P * n * 4 / (ms * 1e-3) / 8e12
                    print(json.dumps({"round": r, "alg": alg.name.lower(),
                                      "form": "one-pass" if one_pass else "blocked launches",
                                      "cap_kib": cap, "P": P, "median_us": round(ms * 1e3, 2),
                                      "frac_of_peak": round(frac, 4)}), flush=True)
    fmi_amd.tune_set(Tune.FUSED_INFLIGHT_KIB, old)
    fmi_amd.tune_set(Tune.BLOCKS_ONE_PASS, 1)


if __name__ == "__main__":
    main()
