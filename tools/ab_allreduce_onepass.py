"""allreduce_no_order one-pass kernels (full-block programs P = 32 / 64, pre-fold programs P = 48 / 80 / 96 /
112) against the 16-peer block launches (FMI_TUNE_BLOCKS_ONE_PASS = 0), 1 GiB of input in total, no-re-use
protocol, interleaved.

    python tools/ab_allreduce_onepass.py
"""
import json, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__)))); sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import fmi_amd
from fmi_amd import Alg, Bucket, Op
from bench_configs import out_sets, timed_fresh
MIB = 1 << 20
fmi_amd.init(0)
for P in (32, 48, 64, 80, 96, 112):
    n = 1024 * MIB // 4 // P // 64 * 64
    ins = [Bucket(n, np.float32).fill_synthetic(7, p) for p in range(P)]
    k_out = out_sets(n * 4)
    outs = [Bucket(n, np.float32) for _ in range(k_out)]
    res = {0: [], 1: []}
    for r in range(3):
        for f in ((1, 0) if r % 2 == 0 else (0, 1)):
            fmi_amd.tune_set(fmi_amd.Tune.BLOCKS_ONE_PASS, f)
            med, _ = timed_fresh(lambda k: fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, outs[k], ins, rank=5), 8, k_out, reps=3)
            res[f].append(med)
    fmi_amd.tune_set(fmi_amd.Tune.BLOCKS_ONE_PASS, 1)
    algo = (P + 1) * n * 4
    row = {"P": P, "bucket_mib": round(n * 4 / MIB, 2)}
    for f, name in ((1, "one_pass"), (0, "block_launches")):
        ms = sorted(res[f])[1]
        row[name + "_us"] = round(ms * 1e3, 2)
        row[name + "_frac"] = round(algo / (ms * 1e-3) / 1e9 / 8000, 4)
    print(json.dumps(row), flush=True)
    for b in ins + outs:
        b.free()
