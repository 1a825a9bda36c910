"""A/B of the programs beyond 128 peers: superblocks of 128 (fmi_dev.hip chain_superblocks /
tree_superblocks, FMI_TUNE_BLOCKS_ONE_PASS = 1) against the fused 16-peer block launches (= 0), over 1 GiB of
input in total, under bench_configs' no-re-use protocol (outputs rotating, set index running on), the two
forms interleaved. Fraction of 8 TB/s on the one-pass ideal (P reads + 1 write; scans P + P).

    python tools/ab_superblocks.py [--rounds 3]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
MIB = 1 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=8)
    args = ap.parse_args()
    import fmi_amd
    from fmi_amd import Alg, Bucket, Op
    from fmi_amd.device import Tune, tune_set

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from bench_configs import out_sets, timed_fresh

    fmi_amd.init(0)
    cases = [(Alg.ALLREDUCE, 256), (Alg.ALLREDUCE, 512), (Alg.REDUCE, 256), (Alg.REDUCE, 300),
             (Alg.REDUCE_LTR, 256), (Alg.SCAN_LTR, 256)]
    for alg, P in cases:
        scan = alg == Alg.SCAN_LTR
        n = 1024 * MIB // 4 // P // 64 * 64
        ins = [Bucket(n, np.float32).fill_synthetic(7, p) for p in range(P)]
        k_out = out_sets((P if scan else 1) * n * 4)
        outs = [[Bucket(n, np.float32) for _ in range(P if scan else 1)] for _ in range(k_out)]

        def launch(k):
            if scan:
                fmi_amd.scan_peers(Op.SUM, alg, outs[k], ins)
            else:
                fmi_amd.reduce_tree(Op.SUM, alg, outs[k][0], ins, rank=0)

        res = {1: [], 0: []}
        for r in range(args.rounds):
            for one_pass in ((1, 0) if r % 2 == 0 else (0, 1)):
                tune_set(Tune.BLOCKS_ONE_PASS, one_pass)
                med, _ = timed_fresh(launch, args.iters, k_out, reps=3)
                res[one_pass].append(med)
        tune_set(Tune.BLOCKS_ONE_PASS, 1)
        algo = (2 * P if scan else P + 1) * n * 4
        row = {"alg": alg.name.lower(), "P": P, "bucket_mib": round(n * 4 / MIB, 2), "output_sets": k_out}
        for one_pass, name in ((1, "superblocks"), (0, "block_launches")):
            ms = sorted(res[one_pass])[len(res[one_pass]) // 2]
            row[name + "_us"] = round(ms * 1e3, 2)
            row[name + "_frac"] = round(algo / (ms * 1e-3) / 1e9 / 8000, 4)
        print(json.dumps(row), flush=True)
        for grp in [ins] + outs:
            for b in grp:
                b.free()


if __name__ == "__main__":
    main()
