"""BASELINE config C3 kernels alone, for rocprofv3 passes (kernel trace, --pmc FETCH_SIZE, --pmc WRITE_SIZE):
the i64 max pairwise combine of 64 MiB buckets, the f32 peer-axis scan over 8 peers x 64 MiB, and the fused
8-peer allreduce tree over the same buckets. Each kernel name appears at one launch shape only, so the
per-kernel PMC medians are per-launch figures. Buffers rotate over sets larger than the 256 MiB Infinity
Cache; the pair kernel's over 64 sets, so no launch re-reads a bucket whose sc1-stored tiles the MALL may
still hold ("store policy across the XCDs"; with 4 sets its trace median read 30.7 us).

    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d DIR -- python3 tools/c3_kernels.py
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
    args = ap.parse_args()
    fmi_amd.init(0)
    n64 = 64 * MIB // 8
    nsets = 64
    pairs = [(Bucket(n64, np.int64).fill_synthetic(42 + s, 0), Bucket(n64, np.int64).fill_synthetic(42 + s, 1))
             for s in range(nsets)]
    for k in range(args.iters):
        a, b = pairs[k % nsets]
        fmi_amd.reduce_pair(Op.MAX, a, b)
    fmi_amd.sync()
    del pairs
    P, n32 = 8, 64 * MIB // 4
    sets = [[Bucket(n32, np.float32).fill_synthetic(7 + s, p) for p in range(P)] for s in range(2)]
    outs = [[Bucket(n32, np.float32) for _ in range(P)] for _ in range(2)]
    for k in range(args.iters):
        fmi_amd.scan_peers(Op.SUM, Alg.SCAN, outs[k % 2], sets[k % 2])
    for k in range(args.iters):
        fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, outs[k % 2][0], sets[k % 2])
    fmi_amd.sync()


if __name__ == "__main__":
    main()
