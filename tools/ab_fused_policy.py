"""A/B of the fused P-way kernels' access policy through the library (FMI_TUNE_FUSED_POLICY): 0 = global
loads / stores nt, 2 = buffer loads nt with sc1 (tree) / nt sc1 (scan) stores (1, the default, picks one of
the two per kernel from this tool's results). Same buffers, same launch,
policies interleaved over rounds; K back-to-back launches over rotating buffer sets (>= 1.5 GiB, so nothing is
re-read from the MALL) between two events.
Also checks that both policies give identical bits.

    python tools/ab_fused_policy.py [--rounds 5] [--mib 64]
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
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--launches", type=int, default=24)
    ap.add_argument("--footprint-gib", type=float, default=1.5,
                    help="rotating buckets per shape; the sc1-stored outputs stay in the 256 MB MALL, so the sets "
                         "must hold well over 256 MB of outputs for no launch to re-read one from there")
    args = ap.parse_args()
    import fmi_amd
    from fmi_amd import Alg, Bucket, Op
    from fmi_amd.device import Event, Tune, reduce_tree, scan_peers, tune_set

    fmi_amd.init(0)
    shapes = []  # (name, dtype, op, alg, P, kind, mib per bucket)
    for P in (2, 4, 8, 16):
        shapes.append((f"tree allreduce f32 sum P={P}", np.float32, Op.SUM, Alg.ALLREDUCE, P, "tree", args.mib))
        shapes.append((f"scan f32 sum P={P}", np.float32, Op.SUM, Alg.SCAN, P, "scan", args.mib))
    shapes += [("tree reduce i64 max P=8", np.int64, Op.MAX, Alg.REDUCE, 8, "tree", args.mib),
               ("scan_ltr f32 sum P=8", np.float32, Op.SUM, Alg.SCAN_LTR, 8, "scan", args.mib),
               ("tree allreduce f32 max P=8 (all ranks)", np.float32, Op.MAX, Alg.ALLREDUCE, 8, "tree", args.mib),
               ("tree allreduce f32 sum P=8, 32 MiB shard (N=8 bench)", np.float32, Op.SUM, Alg.ALLREDUCE, 8, "tree", 32),
               ("tree allreduce f32 sum P=2, 128 MiB shard (N=2 bench)", np.float32, Op.SUM, Alg.ALLREDUCE, 2, "tree", 128)]
    for name, dtype, op, alg, P, kind, mib in shapes:
        n = mib * MIB // np.dtype(dtype).itemsize
        per_set = (P + (P if kind == "scan" else 1)) * mib
        nsets = max(2, -(-int(args.footprint_gib * 1024) // per_set))
        sets = [[Bucket(n, dtype).fill_synthetic(7 + s, p) for p in range(P)] for s in range(nsets)]
        outs = [[Bucket(n, dtype) for _ in range(P if kind == "scan" else 1)] for _ in range(nsets)]

        def launch(s):
            if kind == "scan":
                scan_peers(op, alg, outs[s], sets[s])
            else:
                reduce_tree(op, alg, outs[s][0], sets[s])

        pos = 0  # one running position over the sets: every set is re-used exactly nsets launches later

        def next_launch():
            nonlocal pos
            launch(pos % nsets)
            pos += 1

        bits = {}
        for pol in (0, 2):
            tune_set(Tune.FUSED_POLICY, pol)
            launch(0)
            fmi_amd.sync()
            bits[pol] = [o.numpy().tobytes() for o in outs[0]]
        same = bits[0] == bits[2]
        times = {0: [], 2: []}
        for r in range(args.rounds):
            for pol in ((0, 2) if r % 2 == 0 else (2, 0)):
                tune_set(Tune.FUSED_POLICY, pol)
                next_launch()
                next_launch()
                e0, e1 = Event(), Event()
                e0.record()
                for k in range(args.launches):
                    next_launch()
                e1.record()
                e1.sync()
                times[pol].append(e0.elapsed_ms(e1) * 1e3 / args.launches)
                e0.destroy()
                e1.destroy()
        tune_set(Tune.FUSED_POLICY, 1)
        algo = (P + (P if kind == "scan" else 1)) * n * np.dtype(dtype).itemsize
        m0, m1 = statistics.median(times[0]), statistics.median(times[2])
        print(json.dumps({"shape": name, "global_nt_us": round(m0, 2), "buffer_sc1_us": round(m1, 2),
                          "speedup": round(m0 / m1, 4), "frac_global": round(algo / m0 / 8e6, 4),
                          "frac_buffer": round(algo / m1 / 8e6, 4), "bit_identical": same, "rotating_sets": nsets}), flush=True)
        for grp in sets + outs:
            for b in grp:
                b.free()


if __name__ == "__main__":
    main()
