"""The fused 8-way allreduce kernel (the N > 1 shard kernel; bench.py `c4_one_gpu` at 1 GiB per peer) at several
bucket sizes per peer, for the counter-led experiment of VERDICT r04 item 2. Run it under rocprofv3
(--kernel-trace --stats, then one --pmc pass per counter group): every shape is a fresh set of 8 input buckets and
one output, allocated in the order given, filled, a quiet second, then `launches` back-to-back launches between two
HIP events on the library stream. Prints one JSON line per shape (events) to stdout.

  python tools/tree8_shapes.py [--mib 256,512,1024] [--launches 8] [--slices S] [--skew-kib K,...]

--slices S launches each allreduce as S consecutive slices of the buckets (same program per element, so the
same bits), the shape change VERDICT r04 item 2 names as the first candidate.
--skew-kib K,...: instead of one hipMalloc per bucket, carve the 8 inputs and the output out of ONE allocation,
bucket j at j x (bucket + K KiB): whether the buckets' relative placement (address aliasing between the streams
read at the same offset) is what separates the shapes. -1 = separate allocations (the default layout).
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


def run(mib: int, launches: int, slices: int, skew_kib: int = -1, peers: int = 8) -> dict:
    n = mib * (1 << 20) // 4
    owner = None
    if skew_kib < 0:
        ins = [Bucket(n, np.float32).fill_synthetic(11, p) for p in range(peers)]
        out = Bucket(n, np.float32)
    else:
        stride = n + skew_kib * 256  # elements
        owner = Bucket(stride * (peers + 1), np.float32)
        ins = [owner.view(p * stride, n).fill_synthetic(11, p) for p in range(peers)]
        out = owner.view(peers * stride, n)
    bases = [b.ptr for b in ins] + [out.ptr]
    step = -(-n // slices)
    step = -(-step // 64) * 64

    def once():
        for o in range(0, n, step):
            k = min(step, n - o)
            fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, out.view(o, k), [b.view(o, k) for b in ins])

    fmi_amd.sync()
    time.sleep(1.0)  # freed VRAM of the previous shape is cleared in the background
    once()
    e0, e1 = Event(), Event()
    e0.record()
    for _ in range(launches):
        once()
    e1.record()
    e1.sync()
    us = e0.elapsed_ms(e1) * 1e3 / launches
    got = out.view(0, 1 << 16).numpy()
    xs = [b.view(0, 1 << 16).numpy() for b in ins]
    want = eval_bracketing(fmi_amd.schedule_expr(Alg.ALLREDUCE, peers, 0), xs)
    ok = bool(np.array_equal(got.view(np.uint32), want.view(np.uint32)))
    for b in [out] + ins + ([owner] if owner is not None else []):
        b.free()
    algo = (peers + 1) * n * 4
    return {"mib_per_peer": mib, "slices": slices, "skew_kib": skew_kib, "launches": launches, "us": round(us, 2),
            "frac": round(algo / (us * 1e-6) / 8e12, 4), "window_bit_exact": ok,
            "bases": [hex(b) for b in bases]}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", default="256,512,1024")
    ap.add_argument("--launches", type=int, default=8)
    ap.add_argument("--slices", default="1")
    ap.add_argument("--skew-kib", default="-1")
    a = ap.parse_args()
    fmi_amd.init(0)
    for k in [int(x) for x in a.skew_kib.split(",")]:
        for s in [int(x) for x in a.slices.split(",")]:
            for mib in [int(x) for x in a.mib.split(",")]:
                print(json.dumps(run(mib, a.launches, s, k)), flush=True)


if __name__ == "__main__":
    main()
