"""Small-message combines (FMI's C1 shape: 1 MiB f32 buckets) launched one by one, replayed from a HIP graph
(fmi_graph_*), batched into one launch per 64 (fmi_dev_reduce_pair_batch), and the batch replayed from a
graph: K = 256 pairwise combines over distinct bucket pairs per submission, median of rounds.

    python tools/graph_bench.py [--kib 1024] [--k 256] [--rounds 7]
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kib", type=int, default=1024)
    ap.add_argument("--k", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=7)
    args = ap.parse_args()
    import fmi_amd
    from fmi_amd import Bucket, Event, Graph, Op, Stream

    fmi_amd.init(0)
    n = args.kib * 1024 // 4
    s = Stream()
    pairs = [(Bucket(n, np.float32).fill_synthetic(1, 2 * k), Bucket(n, np.float32).fill_synthetic(1, 2 * k + 1))
             for k in range(args.k)]

    def launches():
        for a, b in pairs:
            fmi_amd.reduce_pair(Op.SUM, a, b, stream=s)

    g = Graph.capture(s, launches)
    from fmi_amd import reduce_pair_batch

    def batch():
        reduce_pair_batch(Op.SUM, pairs, stream=s)

    gb = Graph.capture(s, batch)
    res = {}
    for name, fn in (("launches", launches), ("graph", lambda: g.launch(s)), ("batch", batch),
                     ("batch_graph", lambda: gb.launch(s))):
        dev_us, wall_us = [], []
        for _ in range(args.rounds):
            fn()
            s.sync()
            e0, e1 = Event(), Event()
            t0 = time.perf_counter()
            e0.record(s)
            fn()
            e1.record(s)
            e1.sync()
            wall_us.append((time.perf_counter() - t0) * 1e6 / args.k)
            dev_us.append(e0.elapsed_ms(e1) * 1e3 / args.k)
            e0.destroy()
            e1.destroy()
        res[name] = {"us_per_combine_device": round(statistics.median(dev_us), 3),
                     "us_per_combine_wall": round(statistics.median(wall_us), 3)}
    algo = 3 * n * 4
    for v in res.values():
        v["frac_of_8TBs"] = round(algo / (v["us_per_combine_device"] * 1e-6) / 8e12, 4)
    print(json.dumps({"bucket_kib": args.kib, "combines_per_submission": args.k, **res}), flush=True)
    g.destroy()
    gb.destroy()
    s.destroy()


if __name__ == "__main__":
    main()
