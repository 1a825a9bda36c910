"""The N > 1 shard kernel's input layout (round 6): one bounded A/B.

fmi_comm_allreduce (path TREE) receives the N shards of a 256 MiB bucket into one plain hipMalloc (Comm::scratch), back
to back at stride `shard` (a multiple of 64 KiB), and its fused kernel (tree_kernel, allreduce_no_order order) streams
all N at the same offset, plus the reduced shard into another plain hipMalloc. This tool runs that kernel on exactly
that layout ("packed") and on the product's skewed layout (fmi_comm.hip shard_stride: shard j at j x (shard + 4 KiB),
the output at N x (shard + 4 KiB) of the same range; round 6's first run, profiles/r06a_shard_layout.jsonl, had the
output in a separate allocation), one kernel at a time as on each GPU of an N-GPU node,
rotating over 8 staging sets (no MALL re-use), interleaved `--reps` times. Every launch's result window is checked
against numpy's evaluation of rank 0's bracketing.

  python tools/shard_layout_ab.py [--ranks 2,4,8] [--reps 3] [--launches 40]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import fmi_amd  # noqa: E402
from bench import eval_bracketing  # noqa: E402
from fmi_amd import Alg, Bucket, Event, Op, Tune  # noqa: E402

MIB = 1 << 20
PEAK = 8e12
SLOT = 4096


def run(N, layout, launches, sets=8):
    shard = 256 * MIB // 4 // N  # elements (a multiple of 64 KiB for N = 2, 4, 8)
    stride = shard
    fmi_amd.tune_set(Tune.ALLOC_SLOTS, 0)  # Comm::scratch is a plain hipMalloc
    st = []
    for s in range(sets):
        if layout == "skewed":  # the product's layout (fmi_comm.hip shard_stride): inputs and output in one range
            stride = (shard * 4 + 65535) // 65536 * 65536 // 4 + SLOT // 4
            staging = Bucket((N + 1) * stride, np.float32)
            red_owner, red = staging, staging.view(N * stride, shard)
        else:
            staging = Bucket(N * stride, np.float32)
            red_owner = Bucket(shard, np.float32)
            red = red_owner
        parts = [staging.view(j * stride, shard) for j in range(N)]
        for j, p in enumerate(parts):
            p.fill_synthetic(100 + s, j)
        st.append((staging, parts, red_owner if red_owner is not staging else None, red))
    fmi_amd.sync()
    time.sleep(1.0)
    for i in range(sets):
        fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, st[i][3], st[i][1])
    e0, e1 = Event(), Event()
    e0.record()
    for i in range(launches):
        _, parts, _, red = st[i % sets]
        fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, red, parts)
    e1.record()
    e1.sync()
    us = e0.elapsed_ms(e1) * 1e3 / launches
    expr = fmi_amd.schedule_expr(Alg.ALLREDUCE, N, 0)
    bad = 0
    for _, parts, _, red in st:
        want = eval_bracketing(expr, [p.view(0, 1 << 14).numpy() for p in parts])
        bad += int(np.count_nonzero(red.view(0, 1 << 14).numpy().view(np.uint32) != want.view(np.uint32)))
    for staging, _, red_owner, _ in st:
        staging.free()
        if red_owner is not None:
            red_owner.free()
    return {"ranks": N, "layout": layout, "shard_mib": shard * 4 // MIB, "us": round(us, 2),
            "frac": round((N + 1) * shard * 4 / (us * 1e-6) / PEAK, 4), "mismatches": bad}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="2,4,8")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--launches", type=int, default=40)
    a = ap.parse_args()
    fmi_amd.init(0)
    old = fmi_amd.tune_get(Tune.ALLOC_SLOTS)
    bad = 0
    try:
        for rep in range(a.reps):
            for N in [int(x) for x in a.ranks.split(",")]:
                for layout in ("packed", "skewed"):
                    r = run(N, layout, a.launches)
                    bad += r["mismatches"]
                    print(json.dumps(dict(rep=rep, **r)), flush=True)
    finally:
        fmi_amd.tune_set(Tune.ALLOC_SLOTS, old)
    if bad:
        raise SystemExit(f"{bad} mismatching elements")


if __name__ == "__main__":
    main()
