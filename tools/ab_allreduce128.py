"""allreduce_no_order over exactly 128 peers: the one-pass 128-peer kernel against two superblocks of 64 plus
a 2-value allreduce, through a temporary FMI_AR128 switch read only by the library of commit "allreduce P=128
measured with a temporary switch" (the superblocks became the default for P = 128 right after);
no-re-use protocol, interleaved, bit identity checked."""
import json, os, sys, numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__)))); sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import fmi_amd
from fmi_amd import Alg, Bucket, Op
from bench_configs import out_sets, timed_fresh
MIB = 1 << 20
fmi_amd.init(0)
P = 128
for mib in (8, 2):
    n = mib * MIB // 4
    ins = [Bucket(n, np.float32).fill_synthetic(7, p) for p in range(P)]
    k_out = out_sets(n * 4)
    outs = [Bucket(n, np.float32) for _ in range(k_out)]
    bits, res = {}, {0: [], 1: []}
    for f in (0, 1):
        if f: os.environ["FMI_AR128"] = "1"
        else: os.environ.pop("FMI_AR128", None)
        fmi_amd.reduce_tree(Op.MAX, Alg.ALLREDUCE, outs[0], ins, rank=77)
        bits[f] = outs[0].numpy().tobytes()
    for r in range(3):
        for f in ((0, 1) if r % 2 == 0 else (1, 0)):
            if f: os.environ["FMI_AR128"] = "1"
            else: os.environ.pop("FMI_AR128", None)
            med, _ = timed_fresh(lambda k: fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, outs[k], ins, rank=5), 8, k_out, reps=3)
            res[f].append(med)
    os.environ.pop("FMI_AR128", None)
    print(json.dumps({"P": P, "bucket_mib": mib, "same_bits": bits[0] == bits[1],
                      "one_pass_128_us": round(sorted(res[0])[1] * 1e3, 2), "superblocks64_us": round(sorted(res[1])[1] * 1e3, 2)}), flush=True)
    for b in ins + outs:
        b.free()
