"""A/B of the host-ingress allreduce's pipeline fill / drain (FMI_TUNE_HOST_RAMP): config C5's 1 GiB f32
page-locked host bucket through fmi_comm_allreduce_host on a one-rank communicator, ramp off / on
interleaved, for a few chunk sizes; median wall time, result checked bit-exact (a one-peer allreduce is a
copy). After a 1 s pause, so no freed VRAM is being cleared on the copy engines.

    python tools/ab_host_ramp.py [--rounds 7] [--mib 1024] [--chunks 32,64,128]

Needs the library of commit 3e69cb5 (FMI_TUNE_HOST_RAMP); the ramp was rejected and removed after this
measurement (profiles/r02_c5_ramp_rejected.jsonl).
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
MIB = 1 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--chunks", default="32,64,128")
    args = ap.parse_args()
    import fmi_amd
    from fmi_amd import Op, PinnedArray
    from fmi_amd.comm import Comm, Transport, unique_id
    from fmi_amd.device import Tune, tune_get, tune_set

    fmi_amd.init(0)
    n = args.mib * MIB // 4
    comm = Comm(unique_id(Transport.LOCAL), 1, 0)
    send, recv = PinnedArray(n, np.float32), PinnedArray(n, np.float32)
    send.array[:] = np.random.default_rng(5).random(n, dtype=np.float32)
    default = tune_get(Tune.HOST_RAMP)
    time.sleep(1.0)
    try:
        for cmib in [int(c) for c in args.chunks.split(",")]:
            chunk = cmib * MIB // 4
            times = {0: [], 1: []}
            for r in range(args.rounds + 1):
                for ramp in ((0, 1) if r % 2 == 0 else (1, 0)):
                    tune_set(Tune.HOST_RAMP, ramp)
                    recv.array[:1] = np.float32(-1.0)
                    t0 = time.perf_counter()
                    comm.allreduce_host(Op.SUM, send.array, recv.array, chunk=chunk)
                    if r:
                        times[ramp].append((time.perf_counter() - t0) * 1e3)
                    assert np.array_equal(send.array.view(np.uint32), recv.array.view(np.uint32)), "result differs"
            for ramp in (0, 1):
                ms = statistics.median(times[ramp])
                print(json.dumps({"mib": args.mib, "chunk_mib": cmib, "ramp": ramp, "median_ms": round(ms, 3),
                                  "min_ms": round(min(times[ramp]), 3), "host_bucket_GiB_s": round(args.mib / 1024 / (ms * 1e-3), 2),
                                  "bit_exact": True}), flush=True)
    finally:
        tune_set(Tune.HOST_RAMP, default)
        send.free()
        recv.free()
        comm.destroy()


if __name__ == "__main__":
    main()
