"""Re-tune of the fused P-way kernels' two launch knobs on slotted buckets (round 5), and on carved groups (round 6,
the default; --separate for one allocation per bucket). FMI_TUNE_FUSED_INFLIGHT_KIB
(the LDS reservation that caps workgroups per CU) and FMI_TUNE_FUSED_POLICY (buffer loads nt + sc1 stores vs global
nt accesses) were chosen in rounds 1-2 on buckets whose streams collided in HBM; with fmi_dev_alloc's
rotating 4 KiB slots the best setting may differ. Shapes: the 8-way tree at 1 GiB per peer (C4 on one GPU) and at
32 MiB (the N = 8 shard), the 8-peer scan at 64 MiB (C3). Buckets allocated once (slots on), every (budget, policy)
pair timed in each of `rounds` interleaved rounds: events around `launches` launches rotating over the sets, after
a quiet second. One JSON line per (round, shape, budget, policy); every result window checked once per shape.

  python tools/fused_retune.py [--rounds 2] [--budgets 0,64,128,256] [--policies 2,0]
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


GROUPS = True  # round 6: each set one carved group (fmi_dev_alloc_group); --separate: one fmi_dev_alloc per bucket


def buckets(count, n):
    return Bucket.group(count, n, np.float32) if GROUPS else [Bucket(n, np.float32) for _ in range(count)]


def make_tree(mib, sets, P=8):
    n = mib * MIB // 4
    out = []
    for s in range(sets):
        bs = buckets(P + 1, n)
        for p in range(P):
            bs[p].fill_synthetic(11 + s, p)
        out.append(bs)
    return n, out


def make_scan(mib, sets, P=8):
    n = mib * MIB // 4
    out = []
    for s in range(sets):
        bs = buckets(2 * P, n)
        for p in range(P):
            bs[p].fill_synthetic(7 + s, p)
        out.append(bs)
    return n, out


def timed(launch, sets, launches):
    fmi_amd.sync()
    time.sleep(0.5)
    for i in range(sets):
        launch(i)
    e0, e1 = Event(), Event()
    e0.record()
    for i in range(launches):
        launch(i % sets)
    e1.record()
    e1.sync()
    return e0.elapsed_ms(e1) * 1e3 / launches


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--budgets", default="0,64,128,256")
    ap.add_argument("--policies", default="2,0")
    ap.add_argument("--separate", action="store_true", help="one fmi_dev_alloc per bucket instead of carved groups")
    a = ap.parse_args()
    global GROUPS
    GROUPS = not a.separate
    fmi_amd.init(0)
    P = 8
    shapes = {}
    n1g, t1g = make_tree(1024, 2)
    shapes["tree8_1GiB"] = (lambda i: fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, t1g[i][P], t1g[i][:P]), 2, 12,
                            (P + 1) * n1g * 4)
    n32, t32 = make_tree(32, 8)
    shapes["tree8_32MiB"] = (lambda i: fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, t32[i][P], t32[i][:P]), 8, 96,
                             (P + 1) * n32 * 4)
    n64, s64 = make_scan(64, 8)
    shapes["scan8_64MiB"] = (lambda i: fmi_amd.scan_peers(Op.SUM, Alg.SCAN, s64[i][P:], s64[i][:P]), 8, 48,
                             2 * P * n64 * 4)
    old = (fmi_amd.tune_get(Tune.FUSED_INFLIGHT_KIB), fmi_amd.tune_get(Tune.FUSED_POLICY))
    bad = 0
    try:
        for r in range(a.rounds):
            for name, (launch, sets, launches, algo) in shapes.items():
                for b in [int(x) for x in a.budgets.split(",")]:
                    for pol in [int(x) for x in a.policies.split(",")]:
                        fmi_amd.tune_set(Tune.FUSED_INFLIGHT_KIB, b)
                        fmi_amd.tune_set(Tune.FUSED_POLICY, pol)
                        us = timed(launch, sets, launches)
                        print(json.dumps({"round": r, "shape": name, "inflight_kib": b, "policy": pol, "us": round(us, 2),
                                          "frac": round(algo / (us * 1e-6) / PEAK, 4)}), flush=True)
    finally:
        fmi_amd.tune_set(Tune.FUSED_INFLIGHT_KIB, old[0])
        fmi_amd.tune_set(Tune.FUSED_POLICY, old[1])
    expr = fmi_amd.schedule_expr(Alg.ALLREDUCE, P, 0)
    for bs in t1g + t32:
        want = eval_bracketing(expr, [b.view(0, 1 << 14).numpy() for b in bs[:P]])
        bad += int(np.count_nonzero(bs[P].view(0, 1 << 14).numpy().view(np.uint32) != want.view(np.uint32)))
    for bs in s64:
        xs = [b.view(0, 1 << 14).numpy() for b in bs[:P]]
        for q in range(P):
            want = eval_bracketing(fmi_amd.schedule_expr(Alg.SCAN, P, q), xs)
            bad += int(np.count_nonzero(bs[P + q].view(0, 1 << 14).numpy().view(np.uint32) != want.view(np.uint32)))
    print(json.dumps({"check": "result windows of every set vs numpy's bracketing", "mismatches": bad}), flush=True)
    if bad:
        raise SystemExit(1)


if __name__ == "__main__":
    main()
