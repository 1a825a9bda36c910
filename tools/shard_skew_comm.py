"""The shard kernel inside the product's sharded allreduce, skewed shards on / off (round 6).

N LOCAL ranks (threads of this process on the one GPU) run fmi_comm_allreduce (path TREE, f32 sum) of 256 MiB
buckets; fmi_comm_timing times every shard-kernel launch with an event pair on the stream it runs on (the LOCAL
ranks' kernels and device copies share the library stream, so each launch runs alone, as the one shard kernel of
each GPU of an N-GPU node does). FMI_TUNE_COMM_SHARD_SKEW 1 / 0 interleaved `--reps` times; each block builds a fresh
communicator and buckets, runs `--warmup` + `--steps` allreduces and reports the mean shard-kernel time over every
rank's timed launches, with rank 0's result checked bit for bit on three windows against the single-GPU fused
kernel over the same buckets (the reference's allreduce_no_order order).

  python tools/shard_skew_comm.py [--ranks 8] [--reps 3] [--steps 10]
"""
import argparse
import json
import os
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import fmi_amd  # noqa: E402
from fmi_amd import Alg, Bucket, Op, Tune  # noqa: E402
from fmi_amd.comm import Comm, Transport, unique_id  # noqa: E402

MIB = 1 << 20
PEAK = 8e12


def block(N, skew, warmup, steps, mib=256):
    fmi_amd.tune_set(Tune.COMM_SHARD_SKEW, skew)
    n = mib * MIB // 4
    uid = unique_id(Transport.LOCAL)
    res, errors = [None] * N, []

    def rank(r):
        try:
            c = Comm(uid, N, r)
            send, recv = Bucket(n, np.float32).fill_synthetic(500, r), Bucket(n, np.float32)
            for _ in range(warmup):
                c.allreduce(Op.SUM, send, recv)
            c.timing(True)
            for _ in range(steps):
                c.allreduce(Op.SUM, send, recv)
            ms, k = c.timing_read()
            out = [recv.view(o, 4096).numpy() for o in (0, n // 2, n - 4096)] if r == 0 else None
            res[r] = (ms, k, out)
            send.free()
            recv.free()
            c.destroy()
        except BaseException as e:  # noqa: BLE001 - reported below
            errors.append(f"rank {r}: {e!r}")

    ts = [threading.Thread(target=rank, args=(r,)) for r in range(N)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=600)
    if errors:
        raise SystemExit("; ".join(errors))
    # the single-GPU fused kernel over the same buckets, rank 0's order
    ins = [Bucket(4096, np.float32) for _ in range(N)]
    out = Bucket(4096, np.float32)
    bad = 0
    for w, o in enumerate((0, n // 2, n - 4096)):
        for r in range(N):
            ins[r].fill_synthetic(500, r, first=o)
        fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, out, ins)
        bad += int(np.count_nonzero(out.numpy().view(np.uint32) != res[0][2][w].view(np.uint32)))
    for b in ins + [out]:
        b.free()
    total_ms = sum(r[0] for r in res)
    launches = sum(r[1] for r in res)
    us = total_ms * 1e3 / launches
    shard = n // N
    return {"ranks": N, "skew": skew, "launches": launches, "shard_kernel_us": round(us, 2),
            "frac": round((N + 1) * shard * 4 / (us * 1e-6) / PEAK, 4), "mismatches": bad}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    fmi_amd.init(0)
    old = fmi_amd.tune_get(Tune.COMM_SHARD_SKEW)
    bad = 0
    try:
        for rep in range(a.reps):
            for skew in (1, 0) if rep % 2 == 0 else (0, 1):
                r = block(a.ranks, skew, a.warmup, a.steps)
                bad += r["mismatches"]
                print(json.dumps(dict(rep=rep, **r)), flush=True)
    finally:
        fmi_amd.tune_set(Tune.COMM_SHARD_SKEW, old)
    if bad:
        raise SystemExit(f"{bad} mismatching elements")


if __name__ == "__main__":
    main()
