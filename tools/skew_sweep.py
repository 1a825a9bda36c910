"""Placement sweep (round 5): how the relative placement of the buckets a kernel streams at the same
offset changes its rate. For each kernel shape, every rotating set's buckets are carved out of ONE allocation at
stride `bucket + skew` (skew = -1: one fmi_dev_alloc per bucket — with --alloc-slots 0 a plain hipMalloc, the
layout every measurement before round 5 used; 1 the library's rotating 4 KiB slots), the sets
rotate so that no bucket is re-read from the 256 MiB MALL, and the mean launch time comes from two HIP events on
the library stream around `launches` launches (after a quiet second and a warm-up pass over the sets).

  kernels: pair   C2's a = a + b, 256 MiB f32 (pair_tile; 3 streams: a, b in, a out), 16 sets
           tree8  the fused 8-way allreduce (tree_kernel; 8 in, 1 out) at --tree-mib per peer
           scan8  C3's peer scan, 8 x 64 MiB (scan_kernel; 8 in, 8 out), 8 sets
           copy   the P = 1 allreduce's device copy, 256 MiB (copy_tile; 1 in, 1 out), 8 sets

  python tools/skew_sweep.py [--kernels pair,tree8,scan8,copy] [--skew-kib=-1,0,4,...] [--tree-mib 32,512]

Every launch's result is checked on one window per set against numpy (pair: a + b repeated; tree8 / scan8: the
reference's bracketing; copy: the source), so a placement can only change the time, never the bits.
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
from fmi_amd import Alg, Bucket, Event, Op  # noqa: E402

MIB = 1 << 20
PEAK = 8e12


def carve(count, n, skew_kib, dtype=np.float32):
    """`count` buckets of n elements: separate allocations (skew < 0) or one allocation at stride n + skew."""
    if skew_kib < 0:
        return [Bucket(n, dtype) for _ in range(count)], []
    item = np.dtype(dtype).itemsize
    stride = n + skew_kib * 1024 // item
    owner = Bucket(stride * count, dtype)
    return [owner.view(j * stride, n) for j in range(count)], [owner]


def timed(launch, sets, launches):
    fmi_amd.sync()
    time.sleep(1.0)
    for i in range(sets):
        launch(i)
    e0, e1 = Event(), Event()
    e0.record()
    for i in range(launches):
        launch(i % sets)
    e1.record()
    e1.sync()
    return e0.elapsed_ms(e1) * 1e3 / launches


def pair(skew, launches):
    n, S = 256 * MIB // 4, 16
    sets, owners = [], []
    for s in range(S):
        (a, b), own = carve(2, n, skew)
        a.fill_synthetic(42 + s, 0)
        b.fill_synthetic(42 + s, 1)
        sets.append((a, b))
        owners += own
    us = timed(lambda i: fmi_amd.reduce_pair(Op.SUM, *sets[i]), S, launches)
    bad = 0
    for s, (a, b) in enumerate(sets):
        k = 1 + sum(1 for i in range(launches) if i % S == s)  # the warm-up pass + its timed rotations
        x = Bucket(1 << 16, np.float32).fill_synthetic(42 + s, 0).numpy()
        y = b.view(0, 1 << 16).numpy()
        for _ in range(k):
            x = x + y
        bad += int(np.count_nonzero(a.view(0, 1 << 16).numpy().view(np.uint32) != x.view(np.uint32)))
    for o in owners or [b for st in sets for b in st]:
        o.free()
    return {"us": round(us, 2), "frac": round(3 * n * 4 / (us * 1e-6) / PEAK, 4), "mismatches": bad}


def tree8(skew, launches, mib):
    n, P = mib * MIB // 4, 8
    S = max(1, min(8, (2048 // mib)))  # >= 2 GiB of inputs per rotation where it fits
    sets, owners = [], []
    for s in range(S):
        bs, own = carve(P + 1, n, skew)
        for p in range(P):
            bs[p].fill_synthetic(11 + s, p)
        sets.append(bs)
        owners += own
    us = timed(lambda i: fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, sets[i][P], sets[i][:P]), S, launches)
    bad = 0
    expr = fmi_amd.schedule_expr(Alg.ALLREDUCE, P, 0)
    for bs in sets:
        want = eval_bracketing(expr, [b.view(0, 1 << 14).numpy() for b in bs[:P]])
        bad += int(np.count_nonzero(bs[P].view(0, 1 << 14).numpy().view(np.uint32) != want.view(np.uint32)))
    for o in owners or [b for st in sets for b in st]:
        o.free()
    return {"mib_per_peer": mib, "sets": S, "us": round(us, 2), "frac": round((P + 1) * n * 4 / (us * 1e-6) / PEAK, 4),
            "mismatches": bad}


def scan8(skew, launches):
    n, P, S = 64 * MIB // 4, 8, 8
    sets, owners = [], []
    for s in range(S):
        bs, own = carve(2 * P, n, skew)
        for p in range(P):
            bs[p].fill_synthetic(7 + s, p)
        sets.append(bs)
        owners += own
    us = timed(lambda i: fmi_amd.scan_peers(Op.SUM, Alg.SCAN, sets[i][P:], sets[i][:P]), S, launches)
    bad = 0
    for bs in sets:
        xs = [b.view(0, 1 << 14).numpy() for b in bs[:P]]
        for r in range(P):
            want = eval_bracketing(fmi_amd.schedule_expr(Alg.SCAN, P, r), xs)
            bad += int(np.count_nonzero(bs[P + r].view(0, 1 << 14).numpy().view(np.uint32) != want.view(np.uint32)))
    for o in owners or [b for st in sets for b in st]:
        o.free()
    return {"us": round(us, 2), "frac": round(2 * P * n * 4 / (us * 1e-6) / PEAK, 4), "mismatches": bad}


def copy(skew, launches):
    n, S = 256 * MIB // 4, 8
    sets, owners = [], []
    for s in range(S):
        (a, b), own = carve(2, n, skew)
        a.fill_synthetic(3 + s, 0)
        sets.append((a, b))
        owners += own
    us = timed(lambda i: sets[i][1].copy_from(sets[i][0]), S, launches)
    bad = sum(int(np.count_nonzero(a.view(0, 1 << 14).numpy() != b.view(0, 1 << 14).numpy())) for a, b in sets)
    for o in owners or [b for st in sets for b in st]:
        o.free()
    return {"us": round(us, 2), "frac": round(2 * n * 4 / (us * 1e-6) / PEAK, 4), "mismatches": bad}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernels", default="pair,tree8,scan8,copy")
    ap.add_argument("--skew-kib", default="-1,0,4")
    ap.add_argument("--tree-mib", default="32,512")
    ap.add_argument("--launches", type=int, default=48)
    ap.add_argument("--alloc-slots", default="1", help="FMI_TUNE_ALLOC_SLOTS for the separate allocations (skew -1): "
                                                        "0 = plain hipMalloc, 1 = the library's rotating 4 KiB slots; "
                                                        "a list runs each")
    a = ap.parse_args()
    fmi_amd.init(0)
    bad = 0
    runs = [(skew, slots) for skew in [int(x) for x in a.skew_kib.split(",")]
            for slots in ([int(v) for v in a.alloc_slots.split(",")] if skew < 0 else [0])]
    for skew, slots in runs:
        fmi_amd.tune_set(fmi_amd.Tune.ALLOC_SLOTS, slots)  # carved layouts: one allocation, its own offsets
        for k in a.kernels.split(","):
            rows = [tree8(skew, a.launches, int(m)) for m in a.tree_mib.split(",")] if k == "tree8" else \
                [{"pair": pair, "scan8": scan8, "copy": copy}[k](skew, a.launches)]
            for r in rows:
                bad += r["mismatches"]
                print(json.dumps(dict(kernel=k, skew_kib=skew, alloc_slots=slots, **r)), flush=True)
    if bad:
        raise SystemExit(f"{bad} mismatching elements")


if __name__ == "__main__":
    main()
