"""The fused shard kernel of bench.py's N > 1 headline, alone on one GPU, for rocprofv3 passes (kernel trace,
--pmc FETCH_SIZE, --pmc WRITE_SIZE): at N GPUs every GPU reduces its 256/N MiB shard of N peers' 256 MiB
buckets with tree_kernel<OpSum, float, ALLREDUCE, P = N>. One launch shape per P (N = 2, 4, 8), rotating
over 2 input sets, so the per-kernel PMC medians are the per-launch HBM bytes bench.py reports as
roofline.traffic at that N.

    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d DIR -- python3 tools/shard_kernels.py
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import fmi_amd  # noqa: E402
from fmi_amd import Alg, Bucket, Op  # noqa: E402

MIB = 1 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--bucket-mib", type=int, default=256)
    args = ap.parse_args()
    fmi_amd.init(0)
    for P in (2, 4, 8):
        per = -(-(args.bucket_mib * MIB // 4) // P)
        shard = -(-per // 64) * 64  # fmi_comm's shard_elems
        sets = [[Bucket(shard, np.float32).fill_synthetic(3 + s, p) for p in range(P)] for s in range(2)]
        out = Bucket(shard, np.float32)
        for k in range(args.iters):
            fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, out, sets[k % 2])
        fmi_amd.sync()
        for b in [out] + [x for s in sets for x in s]:
            b.free()


if __name__ == "__main__":
    main()
