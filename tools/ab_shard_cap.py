"""A/B of the fused kernels' residency budget (FMI_TUNE_FUSED_INFLIGHT_KIB) on the N > 1 shard kernels: the
allreduce_no_order tree over N shards of a 256 MiB bucket (N = 2 / 4 / 8: 128 / 64 / 32 MiB shards), its
inputs carved from one staging allocation as fmi_comm's all-to-all leaves them, outputs rotating under
bench_configs' no-re-use protocol; budgets interleaved over rounds.

    python tools/ab_shard_cap.py [--rounds 3] [--budgets 0,32,64,96,128,256]
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
    ap.add_argument("--budgets", default="0,32,64,96,128,256")
    args = ap.parse_args()
    import fmi_amd
    from fmi_amd import Alg, Bucket, Op
    from fmi_amd.device import Tune, tune_get, tune_set
    from bench_configs import out_sets, timed_fresh

    fmi_amd.init(0)
    budgets = [int(b) for b in args.budgets.split(",")]
    default = tune_get(Tune.FUSED_INFLIGHT_KIB)
    for N in (2, 4, 8):
        shard = 256 * MIB // 4 // N
        stagings = [Bucket(N * shard, np.float32) for _ in range(2)]
        ins = [[st.view(j * shard, shard).fill_synthetic(9 + s, j) for j in range(N)] for s, st in enumerate(stagings)]
        k_out = out_sets(shard * 4)
        outs = [Bucket(shard, np.float32) for _ in range(k_out)]
        res = {b: [] for b in budgets}
        for r in range(args.rounds):
            for b in (budgets if r % 2 == 0 else budgets[::-1]):
                tune_set(Tune.FUSED_INFLIGHT_KIB, b)
                med, _ = timed_fresh(lambda k: fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, outs[k], ins[k % 2]), 12,
                                     k_out, reps=3)
                res[b].append(med)
        algo = (N + 1) * shard * 4
        row = {"N": N, "shard_mib": shard * 4 // MIB}
        for b in budgets:
            ms = sorted(res[b])[len(res[b]) // 2]
            row[f"budget{b}_us"] = round(ms * 1e3, 2)
            row[f"budget{b}_frac"] = round(algo / (ms * 1e-3) / 1e9 / 8000, 4)
        print(json.dumps(row), flush=True)
        for x in stagings + outs:
            x.free()
    tune_set(Tune.FUSED_INFLIGHT_KIB, default)


if __name__ == "__main__":
    main()
