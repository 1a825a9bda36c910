"""A/B of allreduce_no_order over P = 2^k > 128 peers: superblocks of 64 (one-pass 64-peer allreduces, then
the allreduce over the superblock values; the default) against the 16-peer block launches
(FMI_TUNE_BLOCKS_ONE_PASS = 0), 1 GiB of input in total, no-re-use protocol, interleaved; bit identity of the
two forms.

    python tools/ab_allreduce_super.py [--rounds 3]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
MIB = 1 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    import fmi_amd
    from fmi_amd import Alg, Bucket, Op
    from bench_configs import out_sets, timed_fresh

    fmi_amd.init(0)
    for P in (256, 512, 1024):
        n = 1024 * MIB // 4 // P
        ins = [Bucket(n, np.float32).fill_synthetic(7, p) for p in range(P)]
        k_out = out_sets(n * 4)
        outs = [Bucket(n, np.float32) for _ in range(k_out)]
        bits = {}
        for form in (0, 1):
            fmi_amd.tune_set(fmi_amd.Tune.BLOCKS_ONE_PASS, form)
            fmi_amd.reduce_tree(Op.MAX, Alg.ALLREDUCE, outs[0], ins, rank=P - 3)
            bits[form] = outs[0].numpy().tobytes()
        res = {0: [], 1: []}
        for r in range(args.rounds):
            for form in ((0, 1) if r % 2 == 0 else (1, 0)):
                fmi_amd.tune_set(fmi_amd.Tune.BLOCKS_ONE_PASS, form)
                med, _ = timed_fresh(lambda k: fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, outs[k], ins, rank=5), 8, k_out, reps=3)
                res[form].append(med)
        fmi_amd.tune_set(fmi_amd.Tune.BLOCKS_ONE_PASS, 1)
        algo = (P + 1) * n * 4
        row = {"P": P, "bucket_mib": round(n * 4 / MIB, 2), "bit_identical_f32_max_rank_P-3": bits[0] == bits[1]}
        for form, name in ((1, "superblocks64"), (0, "block_launches")):
            ms = sorted(res[form])[len(res[form]) // 2]
            row[name + "_us"] = round(ms * 1e3, 2)
            row[name + "_frac"] = round(algo / (ms * 1e-3) / 1e9 / 8000, 4)
        print(json.dumps(row), flush=True)
        for b in ins + outs:
            b.free()


if __name__ == "__main__":
    main()
