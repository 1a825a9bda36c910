"""Bucket placement A/B on the bench's own allocation orders (round 6).

Each block allocates its buckets EXACTLY as bench.py does (or through the group allocator), fills them, waits a quiet
second (the driver clears freed VRAM in the background), launches `warmup` untimed and `steps` timed kernels
(bench.py's 5 / 20 by default), and frees. Modes, interleaved `--reps` times in one process:

  pair  (C2, bench.py run_single: 16 sets, per set a then b, 256 MiB f32 each)
        plain     FMI_TUNE_ALLOC_SLOTS = 0: every bucket a plain hipMalloc (2 MiB aligned: a, b at the same offset)
        rotating  FMI_TUNE_ALLOC_SLOTS = 1: round 5's rotating 4 KiB slots (a in slot g, b in slot g + 1)
        group     Bucket.group(2): a in slot 0, b in slot 1 of their own hipMallocs (fmi_dev_alloc_group)
        same_slot both operands in slot k = 1 + s % 15 (same relative offset as plain, not 2 MiB aligned)
  any kernel: s:i.j.k...  bucket j (allocation order: pair a, b; scan 8 inputs then 8 outputs; tree 8 inputs then
            the output) at 4 KiB slot list[j] of a plain hipMalloc 64 KiB larger, every set alike;
            s:i.j.k...@K  the same with set s's slots moved by K x s (mod 16)
  pair only: c:K    each set's a and b carved from one allocation at stride bucket + K KiB
             call:K every set's a and b carved from ONE allocation (8 GiB) at stride bucket + K KiB
  scan  (C3 scan, bench.py c3_single: 8 sets of 8 inputs ALL allocated first, then all 8 x 8 outputs, 64 MiB f32)
        plain / rotating as above; group: Bucket.group(16) per set (inputs slots 0-7, outputs 8-15)
  tree  (bench.py c4_single: 8 inputs then the output, 1 GiB f32 each, one set)
        plain / rotating; group: Bucket.group(9)

One JSON line per block: kernel, mode, rep, mean launch time from two HIP events around the timed launches on the
library stream, fraction of 8 TB/s, and a bit-exact check of one window per set. Under
`rocprofv3 --kernel-trace` the blocks' launches are attributed by tools/placement_ab_trace.py (the lines give each
block's launch counts in order).

  python tools/placement_ab.py [--kernels pair,scan,tree] [--reps 3] [--modes ...]
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


def at_slots(slots, n, dtype=np.float32):
    """One plain hipMalloc 64 KiB larger per bucket (as the slotted allocator makes), bucket j viewed at 4 KiB slot
    slots[j]: any placement, from the same allocation calls (owners to free, views to use)."""
    fmi_amd.tune_set(Tune.ALLOC_SLOTS, 0)
    item = np.dtype(dtype).itemsize
    owners = [Bucket(n + 16 * SLOT // item, dtype) for _ in slots]
    return [o.view(k * SLOT // item, n) for o, k in zip(owners, slots)], owners


def slot_mode(mode, s=0):
    """'s:0.1...' -> the slot list; 's:0.1...@K' -> each slot + K x set index (mod 16); else None"""
    if not mode.startswith("s:"):
        return None
    body, _, k = mode[2:].partition("@")
    return [(int(x) + int(k or 0) * s) % 16 for x in body.split(".")]


def alloc(mode, count, n, dtype=np.float32, slot=None):
    """`count` buckets of n elements, one allocation each, placed per `mode` (owners to free, views to use)."""
    if slot_mode(mode):
        return at_slots(slot_mode(mode, slot), n, dtype)
    if mode == "group":
        bs = Bucket.group(count, n, dtype)
        return bs, bs
    if mode == "same_slot":
        fmi_amd.tune_set(Tune.ALLOC_SLOTS, 0)
        item = np.dtype(dtype).itemsize
        owners = [Bucket(n + 16 * SLOT // item, dtype) for _ in range(count)]
        return [o.view(slot * SLOT // item, n) for o in owners], owners
    fmi_amd.tune_set(Tune.ALLOC_SLOTS, 1 if mode == "rotating" else 0)
    bs = [Bucket(n, dtype) for _ in range(count)]
    return bs, bs


def timed(launch, warmup, steps):
    fmi_amd.sync()
    time.sleep(1.0)
    for k in range(warmup):
        launch(k)
    e0, e1 = Event(), Event()
    e0.record()
    for k in range(warmup, warmup + steps):
        launch(k)
    e1.record()
    e1.sync()
    us = e0.elapsed_ms(e1) * 1e3 / steps
    e0.destroy()
    e1.destroy()
    return us


def pair(mode, warmup, steps):
    n, S = 256 * MIB // 4, 16
    sets, owners = [], []
    if mode.startswith("call:"):  # every set's a and b carved from ONE allocation at stride bucket + K KiB
        fmi_amd.tune_set(Tune.ALLOC_SLOTS, 0)
        stride = n + int(mode[5:]) * 1024 // 4
        owner = Bucket(stride * 2 * S, np.float32)
        owners = [owner]
        views = [owner.view(j * stride, n) for j in range(2 * S)]
    for s in range(S):  # bench.py run_single: a then b, set after set
        if mode.startswith("call:"):
            a, b = views[2 * s], views[2 * s + 1]
        elif mode.startswith("c:"):  # the set's a and b carved from one allocation at stride bucket + K KiB
            fmi_amd.tune_set(Tune.ALLOC_SLOTS, 0)
            stride = n + int(mode[2:]) * 1024 // 4
            o = Bucket(stride + n, np.float32)
            a, b = o.view(0, n), o.view(stride, n)
            owners.append(o)
        else:
            (a, b), own = alloc(mode, 2, n, slot=s if slot_mode(mode) else 1 + s % 15)
            owners += own
        a.fill_synthetic(42 + s, 0)
        b.fill_synthetic(42 + s, 1)
        sets.append((a, b))
    slots = sorted({(x.ptr % (64 * 1024)) // SLOT for st in sets for x in st})
    used = [0] * S

    def launch(k):
        used[k % S] += 1
        fmi_amd.reduce_pair(Op.SUM, *sets[k % S])

    us = timed(launch, warmup, steps)
    bad = 0
    for s, (a, b) in enumerate(sets):
        x = Bucket(1 << 16, np.float32).fill_synthetic(42 + s, 0).numpy()
        y = b.view(0, 1 << 16).numpy()
        for _ in range(used[s]):
            x = x + y
        bad += int(np.count_nonzero(a.view(0, 1 << 16).numpy().view(np.uint32) != x.view(np.uint32)))
    for o in owners:
        o.free()
    return {"us": round(us, 2), "frac": round(3 * n * 4 / (us * 1e-6) / PEAK, 4), "mismatches": bad,
            "slots_mod_64k": slots}


def copy(mode, warmup, steps):
    """the P = 1 allreduce's device copy (copy_tile<1>, bench.py allreduce_1peer's shape): 8 sets of (src, dst),
    256 MiB each"""
    n, S = 256 * MIB // 4, 8
    sets, owners = [], []
    for s in range(S):
        if mode.startswith("c:"):
            fmi_amd.tune_set(Tune.ALLOC_SLOTS, 0)
            stride = n + int(mode[2:]) * 1024 // 4
            o = Bucket(stride + n, np.float32)
            a, b = o.view(0, n), o.view(stride, n)
            owners.append(o)
        else:
            (a, b), own = alloc(mode, 2, n, slot=s if slot_mode(mode) else 1 + s % 15)
            owners += own
        a.fill_synthetic(3 + s, 0)
        sets.append((a, b))
    us = timed(lambda k: sets[k % S][1].copy_from(sets[k % S][0]), warmup, steps)
    bad = sum(int(np.count_nonzero(a.view(0, 1 << 14).numpy() != b.view(0, 1 << 14).numpy())) for a, b in sets)
    for o in owners:
        o.free()
    return {"us": round(us, 2), "frac": round(2 * n * 4 / (us * 1e-6) / PEAK, 4), "mismatches": bad}


def scan(mode, warmup, steps):
    n, P, S = 64 * MIB // 4, 8, 8
    owners = []
    if mode == "group" or slot_mode(mode):
        groups, owners = [], []
        for s in range(S):
            g, own = (Bucket.group(2 * P, n, np.float32), None) if mode == "group" else at_slots(slot_mode(mode, s), n)
            groups.append(g)
            owners += own or g
        ins = [g[:P] for g in groups]
        outs = [g[P:] for g in groups]
    else:  # bench.py c3_single: every set's inputs first, then every set's outputs
        fmi_amd.tune_set(Tune.ALLOC_SLOTS, 1 if mode == "rotating" else 0)
        ins = [[Bucket(n, np.float32) for _ in range(P)] for _ in range(S)]
        outs = [[Bucket(n, np.float32) for _ in range(P)] for _ in range(S)]
        owners = [b for s in ins + outs for b in s]
    for s in range(S):
        for p in range(P):
            ins[s][p].fill_synthetic(7 + s, p)
    distinct = [len({(b.ptr % (64 * 1024)) // SLOT for b in ins[s] + outs[s]}) for s in range(S)]
    us = timed(lambda k: fmi_amd.scan_peers(Op.SUM, Alg.SCAN, outs[k % S], ins[k % S]), warmup, steps)
    bad = 0
    for s in range(S):
        xs = [b.view(0, 1 << 14).numpy() for b in ins[s]]
        for r in range(P):
            want = eval_bracketing(fmi_amd.schedule_expr(Alg.SCAN, P, r), xs)
            bad += int(np.count_nonzero(outs[s][r].view(0, 1 << 14).numpy().view(np.uint32) != want.view(np.uint32)))
    for o in owners:
        o.free()
    return {"us": round(us, 2), "frac": round(2 * P * n * 4 / (us * 1e-6) / PEAK, 4), "mismatches": bad,
            "distinct_slots_per_set": distinct}


def tree(mode, warmup, steps):
    n, P = 1024 * MIB // 4, 8
    owners = None
    if mode == "group":
        bs = Bucket.group(P + 1, n, np.float32)
    elif slot_mode(mode):
        bs, owners = at_slots(slot_mode(mode), n)
    else:  # bench.py c4_single: the 8 inputs, then the output
        fmi_amd.tune_set(Tune.ALLOC_SLOTS, 1 if mode == "rotating" else 0)
        bs = [Bucket(n, np.float32) for _ in range(P + 1)]
    for p in range(P):
        bs[p].fill_synthetic(11, p)
    distinct = len({(b.ptr % (64 * 1024)) // SLOT for b in bs})
    us = timed(lambda k: fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, bs[P], bs[:P]), warmup, steps)
    want = eval_bracketing(fmi_amd.schedule_expr(Alg.ALLREDUCE, P, 0), [b.view(0, 1 << 14).numpy() for b in bs[:P]])
    bad = int(np.count_nonzero(bs[P].view(0, 1 << 14).numpy().view(np.uint32) != want.view(np.uint32)))
    slots = [(b.ptr % (64 * 1024)) // SLOT for b in bs]
    for b in owners or bs:
        b.free()
    return {"us": round(us, 2), "frac": round((P + 1) * n * 4 / (us * 1e-6) / PEAK, 4), "mismatches": bad,
            "distinct_slots": distinct, "slots": slots}


KERNELS = {"pair": (pair, "plain,rotating,group,same_slot", "pair_tile<fmi::dev::OpSum, float, 4, 3>"),
           "scan": (scan, "plain,rotating,group", "scan_kernel<fmi::dev::OpSum, float, 3, 8>"),
           "tree": (tree, "plain,rotating,group", "tree_kernel<fmi::dev::OpSum, float, 0, 8, false>"),
           "copy": (copy, "plain,group,c:0", "copy_tile<1>")}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernels", default="pair,scan,tree")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--modes", default="", help="comma list overriding every kernel's default modes")
    for k in KERNELS:
        ap.add_argument(f"--modes-{k}", default="", help=f"{k}'s modes; 's:0.1.2' = bucket j at 4 KiB slot j-th entry")
    ap.add_argument("--rotate-order", action="store_true", help="rotate the mode order by one per rep")
    a = ap.parse_args()
    fmi_amd.init(0)
    default_slots = fmi_amd.tune_get(Tune.ALLOC_SLOTS)
    bad = 0
    for rep in range(a.reps):
        for k in a.kernels.split(","):
            fn, modes, trace_name = KERNELS[k]
            ms = (getattr(a, f"modes_{k}") or a.modes or modes).split(",")
            if a.rotate_order:  # rep r starts at mode r: every mode runs after a different one in each rep
                ms = ms[rep % len(ms):] + ms[:rep % len(ms)]
            for mode in ms:
                r = fn(mode, a.warmup, a.steps)
                fmi_amd.tune_set(Tune.ALLOC_SLOTS, default_slots)
                bad += r["mismatches"]
                print(json.dumps(dict(kernel=k, mode=mode, rep=rep, warmup=a.warmup, steps=a.steps,
                                      trace_name=trace_name, **r)), flush=True)
    if bad:
        raise SystemExit(f"{bad} mismatching elements")


if __name__ == "__main__":
    main()
