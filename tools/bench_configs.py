"""Per-config measurements for DESIGN.md (BASELINE.json configs C2, C3, C5-shaped; tree and scan kernels).

Each row: kernel time from HIP events on the launching stream (median over iterations, rotating buffer
sets so the working set exceeds the 256 MiB Infinity Cache where the config allows), algorithmic HBM
bytes per launch, GB/s and fraction of the 8 TB/s peak. Host-inclusive rows time fmi_host_reduce_pair
on pinned and on pageable host buffers (PCIe-bound). Prints one JSON object per row.
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import fmi_amd  # noqa: E402
from fmi_amd import Alg, Bucket, Event, Op, _lib  # noqa: E402

PEAK = 8000.0
MIB = 1 << 20


def timed(fn, iters, rotate):
    ev = [(Event(), Event()) for _ in range(iters)]
    for k in range(3):
        fn(k % rotate)
    fmi_amd.sync()
    for k in range(iters):
        ev[k][0].record()
        fn(k % rotate)
        ev[k][1].record()
    fmi_amd.sync()
    ms = [a.elapsed_ms(b) for a, b in ev]
    return statistics.median(ms), min(ms)


def timed_fresh(fn, iters, rotate, reps=5):
    """No-re-use protocol ("store policy across the XCDs"): the buffer-set index runs on from the
    warm-up, so every set comes back exactly `rotate` launches later, and callers size `rotate` so that well
    over 256 MB of output is written between two uses of a set (sc1-stored lines stay in the MALL). Two
    events around `iters` back-to-back launches, `reps` times; median and min of the per-launch means."""
    pos = 0
    for _ in range(3):
        fn(pos % rotate)
        pos += 1
    fmi_amd.sync()
    means = []
    for _ in range(reps):
        e0, e1 = Event(), Event()
        e0.record()
        for _ in range(iters):
            fn(pos % rotate)
            pos += 1
        e1.record()
        e1.sync()
        means.append(e0.elapsed_ms(e1) / iters)
        e0.destroy()
        e1.destroy()
    return statistics.median(means), min(means)


def out_sets(out_bytes_per_launch, budget=1536 * MIB):
    """Output buffer sets for timed_fresh: >= `budget` bytes of output between two uses of a set."""
    return max(2, -(-budget // out_bytes_per_launch) + 1)


def fused_fresh_rows(it):
    """The fused P-way rows of DESIGN.md §5 under the no-re-use protocol: C3's scan and the P = 8 trees over
    64 MiB buckets, trees over 1 GiB of input for P = 2 / 4 / 16 and the P > 16 programs, outputs rotating
    over out_sets(...) buffers (inputs are only read, with nontemporal loads)."""
    rows = [("C3 scan scan f32 P=8 x 64MiB", "scan", Alg.SCAN, 8, 64), ("C3 scan scan_ltr f32 P=8 x 64MiB", "scan", Alg.SCAN_LTR, 8, 64),
            ("tree allreduce f32 P=8 x 64MiB", "tree", Alg.ALLREDUCE, 8, 64), ("tree reduce f32 P=8 x 64MiB", "tree", Alg.REDUCE, 8, 64),
            ("tree reduce_ltr f32 P=8 x 64MiB", "tree", Alg.REDUCE_LTR, 8, 64)]
    for P in (2, 4, 16, 24, 32, 48, 64):
        rows.append((f"tree allreduce f32 P={P} x {1024 // P}MiB", "tree", Alg.ALLREDUCE, P, 1024 // P))
    rows += [("tree reduce f32 P=64 x 16MiB", "tree", Alg.REDUCE, 64, 16), ("tree reduce_ltr f32 P=64 x 16MiB", "tree", Alg.REDUCE_LTR, 64, 16)]
    for P in (24, 32, 64, 128):
        rows.append((f"scan scan f32 P={P} x {1024 // P}MiB", "scan", Alg.SCAN, P, 1024 // P))
    rows.append(("scan scan_ltr f32 P=64 x 16MiB", "scan", Alg.SCAN_LTR, 64, 16))
    for name, kind, alg, P, mib in rows:
        n = mib * MIB // 4
        n_in = 2 if P * mib <= 512 else 1  # input sets: only read (nt), never in the MALL
        ins = [[Bucket(n, np.float32).fill_synthetic(7 + s, p) for p in range(P)] for s in range(n_in)]
        per_out = (P if kind == "scan" else 1) * mib * MIB
        k_out = out_sets(per_out)
        outs = [[Bucket(n, np.float32) for _ in range(P if kind == "scan" else 1)] for _ in range(k_out)]

        def launch(k):
            if kind == "scan":
                fmi_amd.scan_peers(Op.SUM, alg, outs[k], ins[k % n_in])
            else:
                fmi_amd.reduce_tree(Op.SUM, alg, outs[k][0], ins[k % n_in], rank=P - 1 if alg == Alg.ALLREDUCE else 0)

        med, mn = timed_fresh(launch, max(6, it // 3), k_out)
        algo = (2 * P if kind == "scan" else P + 1) * n * 4
        row(name + " (no re-use)", algo, med, mn, output_sets=k_out, input_sets=n_in)
        del ins, outs


def row(name, algo_bytes, med_ms, min_ms, **kw):
    gbs = algo_bytes / (med_ms * 1e-3) / 1e9
    r = dict(config=name, algo_bytes=algo_bytes, median_us=round(med_ms * 1e3, 2), min_us=round(min_ms * 1e3, 2),
             gb_s=round(gbs, 1), frac_of_peak=round(gbs / PEAK, 4))
    r.update(kw)
    print(json.dumps(r), flush=True)


def pinned(n, dtype):
    p = ctypes.c_void_p()
    nbytes = n * np.dtype(dtype).itemsize
    _lib.call("fmi_host_pin_alloc", ctypes.byref(p), nbytes)
    buf = (ctypes.c_char * nbytes).from_address(p.value)
    return np.frombuffer(buf, dtype=dtype, count=n), p.value


def op_sweep_rows(it):
    """Every op x core dtype through the P = 8 fused programs (allreduce for rank 3, scan), 32 MiB buckets:
    a slow cell points at a kernel that stopped streaming (scratch, an expensive combine)."""
    P = 8
    for dt in (np.float32, np.float64, np.int32, np.int64):
        n = 32 * MIB // np.dtype(dt).itemsize
        ins = [Bucket(n, dt).fill_synthetic(7, p) for p in range(P)]
        out = Bucket(n, dt)
        outs = [Bucket(n, dt) for _ in range(P)]
        for op in (Op.SUM, Op.PROD, Op.MAX, Op.MIN):
            med, mn = timed(lambda k: fmi_amd.reduce_tree(op, Alg.ALLREDUCE, out, ins, rank=3), it, 1)
            row(f"allreduce {op.name.lower()} {np.dtype(dt).name} P=8 x 32MiB rank 3", (P + 1) * 32 * MIB, med, mn)
            med, mn = timed(lambda k: fmi_amd.scan_peers(op, Alg.SCAN, outs, ins), it, 1)
            row(f"scan {op.name.lower()} {np.dtype(dt).name} P=8 x 32MiB", 2 * P * 32 * MIB, med, mn)
        del ins, out, outs


def wide_tree_rows(it):
    """P > 16 tree reductions (fused 16-peer sub-programs) over 1 GiB of input in total. algo_bytes is the
    one-pass ideal (P reads + 1 write); `passes` is what the blocked schedule moves, in buckets."""
    passes = {(Alg.ALLREDUCE, 24): 25, (Alg.ALLREDUCE, 40): 24 + 1 + 16 + 1 + 2 + 1,
              (Alg.ALLREDUCE, 32): 32 + 2 + 2 + 1, (Alg.ALLREDUCE, 48): 32 + 1 + 16 + 1 + 2 + 1,
              (Alg.ALLREDUCE, 64): 64 + 4 + 4 + 1, (Alg.REDUCE, 64): 64 + 4 + 4 + 1,
              (Alg.REDUCE_LTR, 64): 64 + 4 + 4 + 1}
    # allreduce / reduce over 16 B peers (32, 48, 64 here) and reduce_ltr run one pass by default (P + 1
    # buckets); the blocked launches (FMI_TUNE_BLOCKS_ONE_PASS = 0) write and re-read a temp per block
    for alg, P in passes:
        n = 1024 * MIB // 4 // P
        ins = [Bucket(n, np.float32).fill_synthetic(7, p) for p in range(P)]
        out = Bucket(n, np.float32)
        forms = (1, 0) if P % 16 == 0 or alg == Alg.REDUCE_LTR else (1,)
        for one_pass in forms:
            fmi_amd.tune_set(fmi_amd.Tune.BLOCKS_ONE_PASS, one_pass)
            med, mn = timed(lambda k: fmi_amd.reduce_tree(Op.SUM, alg, out, ins, rank=P - 1), max(5, it // 2), 1)
            fmi_amd.tune_set(fmi_amd.Tune.BLOCKS_ONE_PASS, 1)
            form = "" if len(forms) == 1 else (" one-pass" if one_pass else " blocked launches")
            row(f"tree {alg.name.lower()} f32 P={P} x {n * 4 // MIB}MiB{form}", (P + 1) * n * 4, med, mn,
                bucket_passes=P + 1 if len(forms) == 2 and one_pass else passes[(alg, P)], one_pass_buckets=P + 1)
        del ins, out
    # rank-aware allreduce kernels (float max/min: operand order differs per rank) against the plain ones
    for P, op in ((16, Op.SUM), (16, Op.MAX), (24, Op.MAX), (64, Op.MAX)):
        n = 1024 * MIB // 4 // P
        ins = [Bucket(n, np.float32).fill_synthetic(7, p) for p in range(P)]
        out = Bucket(n, np.float32)
        med, mn = timed(lambda k: fmi_amd.reduce_tree(op, Alg.ALLREDUCE, out, ins, rank=5), max(5, it // 2), 1)
        row(f"tree allreduce {op.name.lower()} f32 P={P} x {n * 4 // MIB}MiB rank 5", (P + 1) * n * 4, med, mn)
        del ins, out
    # scans: P outputs; one pass would be 2P buckets, the schedule moves `bucket_passes`. scan_no_order over
    # 32..143 peers runs the one-pass kernel by default (2P, +1 carry read for a ragged block); the blocked
    # launches (FMI_TUNE_BLOCKS_ONE_PASS = 0) read the inputs of blocks >= 1 twice.
    for alg, P, moved, one_pass in ((Alg.SCAN, 24, 48, 1), (Alg.SCAN, 32, 64, 1), (Alg.SCAN, 32, 84, 0),
                                    (Alg.SCAN, 40, 81, 1), (Alg.SCAN, 48, 96, 1), (Alg.SCAN, 48, 134, 0),
                                    (Alg.SCAN, 64, 128, 1), (Alg.SCAN, 64, 184, 0),
                                    (Alg.SCAN, 128, 256, 1), (Alg.SCAN, 128, 384, 0),
                                    (Alg.SCAN_LTR, 64, 64 + 64 + 4, 1)):
        n = 1024 * MIB // 4 // P
        ins = [Bucket(n, np.float32).fill_synthetic(7, p) for p in range(P)]
        outs = [Bucket(n, np.float32) for _ in range(P)]
        fmi_amd.tune_set(fmi_amd.Tune.BLOCKS_ONE_PASS, one_pass)
        med, mn = timed(lambda k: fmi_amd.scan_peers(Op.SUM, alg, outs, ins), max(5, it // 2), 1)
        fmi_amd.tune_set(fmi_amd.Tune.BLOCKS_ONE_PASS, 1)
        form = "" if P <= 31 or alg != Alg.SCAN else (" one-pass" if one_pass else " blocked launches")
        row(f"scan {alg.name.lower()} f32 P={P} x {n * 4 // MIB}MiB{form}", 2 * P * n * 4, med, mn,
            bucket_passes=moved, one_pass_buckets=2 * P)
        del ins, outs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--c5-only", action="store_true", help="only the host-ingress allreduce rows")
    ap.add_argument("--wide-only", action="store_true", help="only the P > 16 tree rows")
    ap.add_argument("--op-sweep", action="store_true", help="only the op x dtype sweep of the P = 8 programs")
    ap.add_argument("--fused-fresh", action="store_true",
                    help="only the fused P-way rows under the no-re-use protocol (timed_fresh)")
    ap.add_argument("--torch-runtime", action="store_true",
                    help="import torch first, so the library binds to torch's bundled HIP runtime")
    args = ap.parse_args()
    if args.torch_runtime:
        import torch  # noqa: F401
    fmi_amd.init(0)
    it = args.iters
    if args.c5_only:
        host_allreduce_rows()
        return
    if args.wide_only:
        wide_tree_rows(it)
        return
    if args.op_sweep:
        op_sweep_rows(it)
        return
    if args.fused_fresh:
        fused_fresh_rows(it)
        return

    # C2 and its siblings: pairwise combine, every dtype/op, 256 MiB buckets, 4 rotating sets
    for dt in (np.float32, np.float64, np.int32, np.int64, np.uint32, np.uint64, np.int8, np.uint8, np.int16, np.uint16):
        n = 256 * MIB // np.dtype(dt).itemsize
        sets = [(Bucket(n, dt).fill_synthetic(42 + s, 0), Bucket(n, dt).fill_synthetic(42 + s, 1)) for s in range(4)]
        core = np.dtype(dt) in (np.dtype(np.float32), np.dtype(np.float64), np.dtype(np.int32), np.dtype(np.int64))
        for op in (Op.SUM, Op.MAX) if (core and not args.quick) else (Op.SUM,):
            med, mn = timed(lambda k: fmi_amd.reduce_pair(op, *sets[k]), it, 4)
            row(f"pair {op.name.lower()} {np.dtype(dt).name} 256MiB", 3 * 256 * MIB, med, mn)
        del sets

    # calibration: the library's device-to-device copy (fmi_dev_d2d_async -> copy_tile, 1 read + 1 write stream)
    # at 256 MiB, 4 rotating pairs: its sc1 stores would otherwise leave the destination in the MALL
    pairs = [(Bucket(64 * MIB, np.float32), Bucket(64 * MIB, np.float32)) for _ in range(4)]
    med, mn = timed(lambda k: pairs[k][1].copy_from(pairs[k][0]), it, 4)
    row("calibration device copy 256MiB (copy_tile, 4 rotating pairs)", 2 * 256 * MIB, med, mn,
        note="fmi_dev_d2d_async, read:write 1:1")
    del pairs

    # C3a: int64 max, 64 MiB buckets; 8 rotating sets = 1.5 GiB working set (defeats the MALL)
    n = 64 * MIB // 8
    sets = [(Bucket(n, np.int64).fill_synthetic(42 + s, 0), Bucket(n, np.int64).fill_synthetic(42 + s, 1))
            for s in range(8)]
    med, mn = timed(lambda k: fmi_amd.reduce_pair(Op.MAX, *sets[k]), it, 8)
    row("C3 pair max int64 64MiB (8 rotating sets)", 3 * 64 * MIB, med, mn)
    med, mn = timed(lambda k: fmi_amd.reduce_pair(Op.MAX, *sets[0]), it, 1)
    row("C3 pair max int64 64MiB (same set, MALL-resident)", 3 * 64 * MIB, med, mn, note="Infinity-Cache hits")
    del sets

    # C3b: peer-axis scan, P = 8 buckets of 64 MiB f32 → 8 outputs (2 rotating input sets = 1 GiB each)
    P, n = 8, 64 * MIB // 4
    ins = [[Bucket(n, np.float32).fill_synthetic(42 + s, p) for p in range(P)] for s in range(2)]
    outs = [Bucket(n, np.float32) for _ in range(P)]
    for alg in (Alg.SCAN, Alg.SCAN_LTR):
        med, mn = timed(lambda k: fmi_amd.scan_peers(Op.SUM, alg, outs, ins[k]), it, 2)
        row(f"C3 scan {alg.name.lower()} f32 P=8 x 64MiB", 2 * P * 64 * MIB, med, mn)
    # P-way tree reductions over the same buckets (one pass: P reads + 1 write)
    out = Bucket(n, np.float32)
    for alg in (Alg.ALLREDUCE, Alg.REDUCE, Alg.REDUCE_LTR):
        med, mn = timed(lambda k: fmi_amd.reduce_tree(Op.SUM, alg, out, ins[k]), it, 2)
        row(f"tree {alg.name.lower()} f32 P=8 x 64MiB", (P + 1) * 64 * MIB, med, mn)
    for P2 in (2, 4, 16):
        n2 = 1024 * MIB // 4 // P2
        ins2 = [Bucket(n2, np.float32).fill_synthetic(7, p) for p in range(P2)]
        out2 = Bucket(n2, np.float32)
        med, mn = timed(lambda k: fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, out2, ins2), max(5, it // 2), 1)
        row(f"tree allreduce f32 P={P2} x {1024 // P2}MiB", (P2 + 1) * n2 * 4, med, mn)
        del ins2, out2
    del ins, outs, out
    wide_tree_rows(it)

    # host-inclusive (C5-shaped, one GPU): pinned and pageable 256 MiB f32 pairs through the device, on a
    # quiet device (see host_allreduce_rows)
    fmi_amd.sync()
    time.sleep(1.0)
    n = 256 * MIB // 4
    ha, pa = pinned(n, np.float32)
    hb, pb = pinned(n, np.float32)
    ha[:] = 1.0
    hb[:] = 2.0
    for zero_copy, chunk in ((0, 16), (0, 64), (1, 64)):
        fmi_amd.tune_set(fmi_amd.Tune.HOST_ZERO_COPY, zero_copy)
        fmi_amd.tune_set(fmi_amd.Tune.HOST_CHUNK, chunk * MIB)
        fmi_amd.host_reduce_pair(Op.SUM, ha, hb)
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            fmi_amd.host_reduce_pair(Op.SUM, ha, hb)
            ts.append(time.perf_counter() - t0)
        med = statistics.median(ts)
        name = "zero-copy kernel" if zero_copy else f"staged pipeline chunk {chunk}MiB"
        print(json.dumps(dict(config=f"host pinned pair sum f32 256MiB {name}", median_ms=round(med * 1e3, 3),
                              bucket_gib_s=round(256 / 1024 / med, 3),
                              pcie_gb_s=round(3 * 256 * MIB / med / 1e9, 2))), flush=True)
    ha_chk = ha.copy()
    assert np.all(ha_chk == ha_chk[0]), "host pair result not uniform"
    fmi_amd.tune_set(fmi_amd.Tune.HOST_ZERO_COPY, 1)
    _lib.call("fmi_host_pin_free", pa)
    _lib.call("fmi_host_pin_free", pb)
    a = np.ones(n, np.float32)
    b = np.full(n, 2.0, np.float32)
    fmi_amd.tune_set(fmi_amd.Tune.HOST_CHUNK, 64 * MIB)
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        fmi_amd.host_reduce_pair(Op.SUM, a, b)
        ts.append(time.perf_counter() - t0)
    med = statistics.median(ts)
    print(json.dumps(dict(config="host pageable pair sum f32 256MiB", median_ms=round(med * 1e3, 3),
                          bucket_gib_s=round(256 / 1024 / med, 3))), flush=True)
    # the same pageable buckets, page-locked in place once (fmi_host_register): zero-copy from then on
    t0 = time.perf_counter()
    regs = [fmi_amd.HostRegistration(a), fmi_amd.HostRegistration(b)]
    reg_ms = (time.perf_counter() - t0) * 1e3
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        fmi_amd.host_reduce_pair(Op.SUM, a, b)
        ts.append(time.perf_counter() - t0)
    for r in regs:
        r.close()
    med = statistics.median(ts)
    print(json.dumps(dict(config="host registered pair sum f32 256MiB zero-copy", median_ms=round(med * 1e3, 3),
                          bucket_gib_s=round(256 / 1024 / med, 3), pcie_gb_s=round(3 * 256 * MIB / med / 1e9, 2),
                          register_both_ms=round(reg_ms, 2))), flush=True)
    host_allreduce_rows()


def host_allreduce_rows():
    """Config C5 shape: fmi_comm_allreduce_host over page-locked host buckets (H2D, sharded allreduce, D2H
    pipelined in chunks). N ranks are threads of this process on the one GPU (LOCAL transport), so all of
    them share one PCIe link: N = 1 is the per-GPU PCIe-bound rate of the 8-GPU node, N = 8 shows the
    schedule with 8 ranks behind one link."""
    import threading

    from fmi_amd.comm import Comm, Transport, unique_id

    for N, mib, chunks in ((1, 1024, (16, 64, 128)), (8, 128, (16, 64))):
        n = mib * MIB // 4
        bufs = [(fmi_amd.PinnedArray(n, np.float32), fmi_amd.PinnedArray(n, np.float32)) for _ in range(N)]
        for r, (s, _) in enumerate(bufs):
            s.array[:] = np.float32(r + 1)
        for chunk in chunks:
            # a quiet device first: VRAM freed by the rows before is cleared asynchronously on the copy
            # engines these H2D / D2H copies use (profiles/archive/r02_c5_after_free_probe.jsonl)
            fmi_amd.sync()
            time.sleep(1.0)
            uid = unique_id(Transport.LOCAL)
            times = [None] * N

            def worker(r):
                c = Comm(uid, N, r)
                s, o = bufs[r]
                ts = []
                for k in range(4):
                    c.barrier()
                    t0 = time.perf_counter()
                    c.allreduce_host(Op.SUM, s.array, o.array, chunk=chunk * MIB // 4)
                    c.barrier()
                    ts.append(time.perf_counter() - t0)
                times[r] = statistics.median(ts[1:])
                c.destroy()

            th = [threading.Thread(target=worker, args=(r,)) for r in range(N)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            med = max(times)
            want = np.float32(N * (N + 1) // 2)
            assert all(np.all(o.array == want) for _, o in bufs), "host allreduce result"
            print(json.dumps(dict(config=f"C5 host allreduce f32 N={N} x {mib}MiB pinned, chunk {chunk}MiB",
                                  ranks_share_one_gpu=N > 1, median_ms=round(med * 1e3, 3),
                                  per_rank_gib_s=round(mib / 1024 / med, 3),
                                  pcie_gb_s_all_ranks=round(2 * N * mib * MIB / med / 1e9, 2))), flush=True)
        for s, o in bufs:
            s.free()
            o.free()


if __name__ == "__main__":
    main()
