"""Reduce superblock size A/B (128 / 64 / 32 peers), through a temporary FMI_RED_SUPER switch that only the
library of this commit reads (removed in the next commit, 128 kept): profiles/r02_ab_reduce_superblock_size.jsonl.
"""
import json, os, sys, numpy as np
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tools"))
import fmi_amd
from fmi_amd import Alg, Bucket, Op
from bench_configs import out_sets, timed_fresh
MIB = 1 << 20
fmi_amd.init(0)
for P in (256, 300, 1000):
    n = 1024 * MIB // 4 // P // 64 * 64
    ins = [Bucket(n, np.float32).fill_synthetic(7, p) for p in range(P)]
    k_out = out_sets(n * 4)
    outs = [Bucket(n, np.float32) for _ in range(k_out)]
    forms = ["128", "64", "32"]
    bits, res = {}, {f: [] for f in forms}
    for f in forms:
        os.environ["FMI_RED_SUPER"] = f
        fmi_amd.reduce_tree(Op.SUM, Alg.REDUCE, outs[0], ins, rank=7)
        bits[f] = outs[0].numpy().tobytes()
    for r in range(3):
        for f in (forms if r % 2 == 0 else forms[::-1]):
            os.environ["FMI_RED_SUPER"] = f
            med, _ = timed_fresh(lambda k: fmi_amd.reduce_tree(Op.SUM, Alg.REDUCE, outs[k], ins, rank=7), 8, k_out, reps=3)
            res[f].append(med)
    row = {"P": P, "same_bits": len(set(bits.values())) == 1}
    for f in forms:
        row["super" + f + "_us"] = round(sorted(res[f])[1] * 1e3, 2)
    print(json.dumps(row), flush=True)
    for b in ins + outs:
        b.free()
