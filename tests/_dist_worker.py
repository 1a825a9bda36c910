"""Worker for the multi-process (gloo, CPU) tests of fmi_amd/collectives.py.

The exchange logic (shard layout, padding, all-to-all / reduce-scatter, all-gather, peer numbering)
is the product code; only the combine engine is swapped for `HostEngine`, a CPU test double that
applies the same element ops and evaluates the same P-way program the fused kernel runs
(fmi_schedule_expr). The GPU parity tests cover the HIP engine itself.
"""
import os
import re

import numpy as np
import torch
import torch.distributed as dist

from fmi_amd import collectives
from fmi_amd.device import Op

_ELEM = {
    Op.SUM: lambda a, b: a + b,
    Op.PROD: lambda a, b: a * b,
    Op.MAX: lambda a, b: np.where(a < b, b, a),
    Op.MIN: lambda a, b: np.where(b < a, b, a),
}


def _eval(expr: str, xs, f):
    """Evaluate a schedule expression like '((x0+x1)+(x2+x3))' over numpy arrays."""
    tokens = re.findall(r"\(|\)|\+|x\d+", expr)
    pos = 0

    def parse():
        nonlocal pos
        t = tokens[pos]
        pos += 1
        if t.startswith("x"):
            return xs[int(t[1:])]
        left = parse()
        assert tokens[pos] == "+"
        pos += 1
        right = parse()
        assert tokens[pos] == ")"
        pos += 1
        return f(left, right)

    return parse()


class HostEngine:
    device = torch.device("cpu")

    def reduce_pair(self, op, inout, src):
        a = inout.numpy()
        a[...] = _ELEM[op](a, src.numpy())

    def reduce_tree(self, op, alg, out, ins, rank=0):
        import fmi_amd

        expr = fmi_amd.schedule_expr(alg, len(ins), rank)
        out.numpy()[...] = _eval(expr, [t.numpy() for t in ins], _ELEM[op])

    def fill_synthetic(self, t, seed, peer):
        from oracle import fmi_oracle as orc

        t.numpy()[...] = orc.synthetic(t.numpy().dtype, t.numel(), seed, peer)


def with_edges(x, peer):
    """Signed zeros and NaNs on shared indices (every 5th element: +0 on peers 0, 3 mod 4 and -0 on the
    others; every 13th: NaN on peer 0 only): float max / min then depend on each peer's operand order."""
    x = x.copy()
    x[::5] = 0.0 if peer % 4 in (0, 3) else -0.0
    if peer == 0:
        x[3::13] = np.nan
    return x


def run(rank, world, port, n, dtype, op, path, peers_per_gpu, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ar = collectives.ShardedAllreduce(path=path, engine=HostEngine())
        from oracle import fmi_oracle as orc

        edges = dtype.endswith(":edges")
        dt = np.dtype(dtype.split(":")[0])
        buckets = []
        for j in range(peers_per_gpu):
            p = peers_per_gpu * rank + j
            x = orc.synthetic(dt, n, 42, p)
            buckets.append(torch.from_numpy(with_edges(x, p) if edges else x))
        out = torch.empty(n, dtype=buckets[0].dtype)
        ar.allreduce(Op(op), buckets, out)
        np.save(os.path.join(outdir, f"out{rank}.npy"), out.numpy())
        np.save(os.path.join(outdir, f"send{rank}.npy"), buckets[0].numpy())
    finally:
        dist.destroy_process_group()


def run_bench(rank, world, port, n, path, outdir):
    """bench.py's N>1 timed loop with the CPU engine: exercises the exact code the GPU run executes."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ar = collectives.ShardedAllreduce(path=path, engine=HostEngine())
        step_ms, kernel_ms, extra = ar.bench(n, steps=3, warmup=1, sets=2)
        import json

        with open(os.path.join(outdir, f"bench{rank}.json"), "w") as f:
            json.dump({"step_ms": step_ms, "kernel_ms": kernel_ms, "extra": extra}, f)
    finally:
        dist.destroy_process_group()


def run_fall_back(rank, world, port, failing_rank, outdir):
    """bench._fall_back over gloo: only `failing_rank` saw its step raise (or no rank, failing_rank = -1); every
    rank must reach the same verdict, and the ranks that fall back hand run_dist_torch_exchange the reason (their
    own error, or "failed on another rank"). run_dist_torch_exchange itself is recorded, not run (it needs GPUs)."""
    import json
    import sys

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench

    calls = []
    bench.run_dist_torch_exchange = lambda args, w, r, watch, err, numa: calls.append(err)

    class Watch:
        def enter(self, phase):
            pass

    class Comm:
        destroyed = False

        def destroy(self):
            Comm.destroyed = True

    err = f"RuntimeError: rank {rank} broke" if rank == failing_rank else None
    vote = dist.new_group(backend="gloo")  # bench.run_dist votes on a gloo group of its own
    fell = bench._fall_back(None, world, rank, Watch(), 0, {}, Comm(), err, "the fmi_comm allreduce", group=vote)
    with open(os.path.join(outdir, f"fall{rank}.json"), "w") as f:
        json.dump({"fell": fell, "calls": calls, "destroyed": Comm.destroyed}, f)
    dist.destroy_process_group()
