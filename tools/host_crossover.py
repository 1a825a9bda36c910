"""Where does fmi_host_reduce_pair pay? (ChannelPolicy's host-combine
threshold.) One f32 sum combine of two host buckets, one calling thread, at 64 KiB .. 512 MiB per bucket:

  gpu_pageable_us   fmi_host_reduce_pair on pageable numpy arrays (staged H2D, kernel, D2H)
  gpu_pinned_us     fmi_host_reduce_pair on page-locked arrays (the zero-copy kernel over PCIe)
  host_inplace_us   numpy `np.add(a, b, out=a)`: the reference's std::transform in place on one core, the best
                    CPU combine the reference could run (its own vector adapter costs 6 more bucket copies)
  host_adapter_us   the reference's adapter as it executes (Communicator.h:180-189: both buckets copied into
                    vectors, Function called by value, the result copied back), restated with numpy copies

Median of `reps` after two warm-ups, buckets re-filled from the same source each rep (cold in cache as the
recv buffer of a channel is). Every GPU result is checked bit-exact against numpy's a + b. One JSON line per size.

  python tools/host_crossover.py [--reps 41]
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import fmi_amd  # noqa: E402
from fmi_amd import Op, PinnedArray  # noqa: E402

KIB = 1 << 10


def timed(fn, reps, refill):
    ts = []
    for k in range(reps + 2):
        refill()
        t0 = time.perf_counter()
        fn()
        t = time.perf_counter() - t0
        if k >= 2:
            ts.append(t)
    return statistics.median(ts) * 1e6


def adapter(a, b):  # Communicator.h:180-189 as executed: vec copies in, op by value, copy back
    va, vb = a.copy(), b.copy()
    fa, fb = va.copy(), vb.copy()  # Function<T>::operator()(T a, T b) takes both by value
    r = fa + fb
    va[:] = r
    a[:] = va


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=41)
    ap.add_argument("--sizes-kib", default="64,256,1024,4096,16384,32768,65536,131072,262144,524288")
    a = ap.parse_args()
    fmi_amd.init(0)
    rng = np.random.default_rng(5)
    for kib in [int(x) for x in a.sizes_kib.split(",")]:
        n = kib * KIB // 4
        src_a = rng.random(n, dtype=np.float32)
        src_b = rng.random(n, dtype=np.float32)
        want = src_a + src_b
        x, y = np.empty_like(src_a), src_b.copy()
        px, py = PinnedArray(n, np.float32), PinnedArray(n, np.float32)
        py.array[:] = src_b

        def refill():
            x[:] = src_a
            px.array[:] = src_a

        reps = a.reps if kib <= 16384 else 9  # the large buckets' adapter passes take 0.1-0.4 s each
        row = {"bucket_kib": kib, "reps": reps}
        row["gpu_pageable_us"] = round(timed(lambda: fmi_amd.host_reduce_pair(Op.SUM, x, y), reps, refill), 1)
        ok_pageable = bool(np.array_equal(x, want))
        row["gpu_pinned_us"] = round(timed(lambda: fmi_amd.host_reduce_pair(Op.SUM, px.array, py.array), reps, refill), 1)
        ok_pinned = bool(np.array_equal(px.array, want))
        row["host_inplace_us"] = round(timed(lambda: np.add(x, y, out=x), reps, refill), 1)
        row["host_adapter_us"] = round(timed(lambda: adapter(x, y), reps, refill), 1)
        row["bit_exact"] = ok_pageable and ok_pinned
        best_gpu = min(row["gpu_pageable_us"], row["gpu_pinned_us"])
        row["gpu_pinned_over_host_inplace"] = round(row["gpu_pinned_us"] / row["host_inplace_us"], 3)
        row["gpu_pageable_over_host_inplace"] = round(row["gpu_pageable_us"] / row["host_inplace_us"], 3)
        row["gpu_pays_vs_inplace"] = {"pinned": row["gpu_pinned_us"] < row["host_inplace_us"],
                                      "pageable": row["gpu_pageable_us"] < row["host_inplace_us"]}
        row["gpu_pays_vs_adapter"] = best_gpu < row["host_adapter_us"]
        px.free()
        py.free()
        print(json.dumps(row), flush=True)
        if not row["bit_exact"]:
            raise SystemExit(f"GPU combine differs from numpy at {kib} KiB")


if __name__ == "__main__":
    main()
