"""Multi-GPU sharded bucket allreduce: one process per GPU, torch.distributed over RCCL/xGMI.

FMI's allreduce (reference src/comm/PeerToPeer.cpp:96-130) is recursive doubling over peers that talk
through host sockets. On one MI355X node the peers' buckets sit in HBM of different GPUs, so the
exchange runs over xGMI instead, sharded so that all 7 links of every GPU carry traffic at once:

  local rounds   every GPU first folds the peers it hosts with the pairwise kernel (with two peers per
                 GPU this IS round 0 of recursive doubling: pairs (2g, 2g+1));
  path "tree"    (default, bit-exact) all-to-all of bucket shards → GPU k holds shard k of every GPU's
                 partial → ONE pass of the fused P-way kernel in allreduce_no_order order over the N
                 partials → all-gather of the reduced shards. For N a power of two this evaluates exactly
                 the reference's 2N-peer recursive-doubling bracketing, so every GPU ends with the
                 reference's bits (SURVEY.md §8e "Path B").
  path "rccl"    RCCL reduce-scatter + all-gather (SURVEY.md §8e "Path A"): same traffic, RCCL's own
                 reduction order, float results within (P-1)·u·Σ|x| of the reference.

No collective is invented: the all-to-all / reduce-scatter IS the exchange step of the reference's
allreduce, re-cut into shards.

Runtime note: torch wheels bundle their own HIP runtime. libfmi_dev.so binds to whichever
libamdhip64.so.7 is loaded first, so torch must be imported before the library is loaded (this module
imports torch at import time and refuses to run if the library was loaded before torch) — then torch,
RCCL and our kernels share one runtime, one set of streams and one address space.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from . import _lib  # noqa: E402
from .device import Alg, DType, Op  # noqa: E402

_TORCH_DTYPE = {torch.float32: DType.F32, torch.float64: DType.F64, torch.int32: DType.I32, torch.int64: DType.I64,
                torch.int8: DType.I8, torch.uint8: DType.U8, torch.int16: DType.I16}
_REDUCE_OP = {Op.SUM: dist.ReduceOp.SUM, Op.PROD: dist.ReduceOp.PRODUCT, Op.MAX: dist.ReduceOp.MAX,
              Op.MIN: dist.ReduceOp.MIN}
SHARD_ALIGN = 64  # elements: keeps every shard 256-B aligned for the 16-B vector kernels


def _dtype(t: torch.Tensor) -> DType:
    try:
        return _TORCH_DTYPE[t.dtype]
    except KeyError:
        raise TypeError(f"unsupported bucket dtype {t.dtype}") from None


class HipEngine:
    """Product engine: combines run as libfmi_dev.so kernels on torch CUDA tensors, on torch's current
    stream (so they order with RCCL collectives exactly like torch's own ops)."""

    def __init__(self, device_index: int):
        if _lib._lib is not None and not _lib.TORCH_LOADED_FIRST:
            raise RuntimeError("libfmi_dev.so was loaded before torch: two HIP runtimes would coexist; import "
                               "fmi_amd.collectives (or torch) before using fmi_amd")
        _lib.load()
        _lib.call("fmi_dev_init", device_index)
        self.device = torch.device("cuda", device_index)

    @staticmethod
    def _stream() -> int:
        return torch.cuda.current_stream().cuda_stream

    def reduce_pair(self, op: Op, inout: torch.Tensor, src: torch.Tensor) -> None:
        assert inout.is_contiguous() and src.is_contiguous() and inout.numel() == src.numel()
        _lib.call("fmi_dev_reduce_pair", int(op), int(_dtype(inout)), inout.data_ptr(), src.data_ptr(),
                  inout.numel(), self._stream())

    def reduce_tree(self, op: Op, alg: Alg, out: torch.Tensor, ins: Sequence[torch.Tensor], rank: int = 0) -> None:
        import ctypes
        ptrs = (ctypes.c_void_p * len(ins))(*[t.data_ptr() for t in ins])
        _lib.call("fmi_dev_reduce_tree", int(op), int(_dtype(out)), int(alg), out.data_ptr(), ptrs, len(ins), rank,
                  out.numel(), self._stream())

    def fill_synthetic(self, t: torch.Tensor, seed: int, peer: int) -> None:
        _lib.call("fmi_dev_fill_synthetic", int(_dtype(t)), t.data_ptr(), t.numel(), seed, peer, self._stream())


class ShardedAllreduce:
    """Allreduce of the buckets of all peers hosted by the GPUs of `group` (one process per GPU).

    `allreduce(op, buckets, out)`: `buckets` are the peer buckets hosted by this GPU (peers
    local_peers·rank … in order); every GPU's `out` receives the full reduced bucket. As in the reference
    (src/comm/PeerToPeer.cpp:103,119) the first local bucket is overwritten with the partial result.
    """

    def __init__(self, group=None, path: str = "tree", engine=None, force_exchange: bool = False):
        if path not in ("tree", "rccl"):
            raise ValueError("path must be 'tree' or 'rccl'")
        self.group = group if group is not None else dist.group.WORLD
        self.world = dist.get_world_size(self.group)
        self.rank = dist.get_rank(self.group)
        self.path = path
        self.force_exchange = force_exchange  # run the exchange even on one GPU (plumbing checks)
        if engine is None:
            engine = HipEngine(torch.cuda.current_device())
        self.engine = engine
        self._bufs = {}

    def _buf(self, key, numel, like: torch.Tensor) -> torch.Tensor:
        b = self._bufs.get(key)
        if b is None or b.numel() != numel or b.dtype != like.dtype or b.device != like.device:
            b = torch.empty(numel, dtype=like.dtype, device=like.device)
            self._bufs[key] = b
        return b

    def shard_elems(self, n: int) -> int:
        per = -(-n // self.world)
        return -(-per // SHARD_ALIGN) * SHARD_ALIGN

    def allreduce(self, op: Op, buckets: List[torch.Tensor], out: torch.Tensor) -> torch.Tensor:
        if not buckets:
            raise ValueError("need at least one local peer bucket")
        x = buckets[0]
        n = x.numel()
        for b in buckets:
            if b.numel() != n or b.dtype != x.dtype:
                raise RuntimeError("Dimensions of send and receive data must match")
        if out.numel() != n:
            raise RuntimeError("Dimensions of send and receive data must match")
        L = len(buckets)
        if L & (L - 1):
            # recursive doubling pairs the local peers among themselves only for a power-of-two count
            raise ValueError(f"{L} local peer buckets: a GPU must host a power-of-two number of peers")
        if L == 2:  # local round 0 of recursive doubling: pairs (2g, 2g+1)
            self.engine.reduce_pair(op, x, buckets[1])
        elif L > 2:  # local rounds 0..k-1: the 2^k-peer allreduce program over this GPU's peers
            self.engine.reduce_tree(op, Alg.ALLREDUCE, x, buckets, rank=0)
        N = self.world
        if N == 1 and not self.force_exchange:
            out.copy_(x)
            return out
        shard = self.shard_elems(n)
        padded = shard * N
        if padded != n:
            src = self._buf("pad_in", padded, x)
            src[:n].copy_(x)
            src[n:].zero_()
        else:
            src = x
        red = self._buf("shard", shard, x)
        if self.path == "tree":
            staging = self._buf("staging", padded, x)
            dist.all_to_all_single(staging, src, group=self.group)
            parts = [staging[j * shard:(j + 1) * shard] for j in range(N)]
            if op in (Op.MAX, Op.MIN) and x.dtype in (torch.float32, torch.float64):
                # float max / min keep the first operand on ±0 ties and NaNs, so each GPU's peer 2g ends
                # with its own bits: the shard owner computes the shard in every rank's order and an
                # all-to-all (instead of the all-gather) delivers rank r's versions (same volume)
                pers = self._buf("per_rank", padded, x)
                for r in range(N):
                    self.engine.reduce_tree(op, Alg.ALLREDUCE, pers[r * shard:(r + 1) * shard], parts, rank=r)
                gathered = out if padded == n else self._buf("pad_out", padded, x)
                dist.all_to_all_single(gathered, pers, group=self.group)
                if gathered is not out:
                    out.copy_(gathered[:n])
                return out
            self.engine.reduce_tree(op, Alg.ALLREDUCE, red, parts, rank=0)
        else:
            dist.reduce_scatter_tensor(red, src, op=_REDUCE_OP[op], group=self.group)
        gathered = out if padded == n else self._buf("pad_out", padded, x)
        dist.all_gather_into_tensor(gathered, red, group=self.group)
        if gathered is not out:
            out.copy_(gathered[:n])
        return out

    # ------------------------------------------------------------------------------------------------
    def bench(self, n: int, steps: int, warmup: int, sets: int = 2, peers_per_gpu: int = 2,
              return_result: bool = False):
        return self._bench(n, steps, warmup, sets, peers_per_gpu, return_result)

    def _bench(self, n: int, steps: int, warmup: int, sets: int = 2, peers_per_gpu: int = 2,
               return_result: bool = False):
        """Timed loop for bench.py: returns (ms_per_step max over ranks, per-step local-kernel ms, extras).

        Exactly `steps` steps are timed, bracketed by barrier + device sync on both sides; the step time
        is the max over ranks. The local pairwise kernel is also timed on the stream it runs on.
        return_result (one peer per GPU only: its bucket is never modified): extras["result"] = (out tensor,
        synthetic seed of the last step's set), for check_windows.
        """
        import time

        dev = self.engine.device
        on_gpu = dev.type == "cuda"

        def sync():
            if on_gpu:
                torch.cuda.synchronize()

        bufs = []
        for s in range(sets):
            pair = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(peers_per_gpu)]
            for j, t in enumerate(pair):
                self.engine.fill_synthetic(t, 42 + s, peers_per_gpu * self.rank + j)
            bufs.append(pair)
        out = torch.empty(n, dtype=torch.float32, device=dev)
        for k in range(warmup):
            self.allreduce(Op.SUM, bufs[k % sets], out)
        if on_gpu:
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        local_ms = []
        dist.barrier(group=self.group)
        sync()
        t0 = time.perf_counter()
        for k in range(steps):
            pair = bufs[k % sets]
            if on_gpu:
                ev[k][0].record()
            else:
                tl = time.perf_counter()
            if len(pair) == 2:
                self.engine.reduce_pair(Op.SUM, pair[0], pair[1])
            elif len(pair) > 2:
                self.engine.reduce_tree(Op.SUM, Alg.ALLREDUCE, pair[0], pair, rank=0)
            if on_gpu:
                ev[k][1].record()
            else:
                local_ms.append((time.perf_counter() - tl) * 1e3)
            self.allreduce(Op.SUM, [pair[0]], out)
        sync()
        dist.barrier(group=self.group)
        t1 = time.perf_counter()
        local = torch.tensor([(t1 - t0) * 1e3 / steps], dtype=torch.float64, device=dev)
        dist.all_reduce(local, op=dist.ReduceOp.MAX, group=self.group)
        step_ms = float(local.item())
        kernel_ms = [a.elapsed_time(b) for a, b in ev] if on_gpu else local_ms
        extra = {
            "kernel_algo_bytes": 3 * n * 4,
            "exchange": self.path,
            "shard_elems": self.shard_elems(n),
            "algbw_GiB_s": round((n * 4 / 2 ** 30) / (step_ms * 1e-3), 2),
            "busbw_GiB_s": round((n * 4 / 2 ** 30) / (step_ms * 1e-3) * 2 * (self.world - 1) / self.world, 2),
        }
        if return_result and peers_per_gpu == 1 and steps > 0:
            extra["result"] = (out, 42 + (steps - 1) % sets)
        return step_ms, kernel_ms, extra

    def max_over_ranks(self, *vals: float) -> List[float]:
        dev = (torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(self.group) == "nccl"
               else torch.device("cpu"))
        t = torch.tensor(vals, dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return [float(v) for v in t.tolist()]


def check_windows(world: int, rank: int, shard: int, n: int, seed: int, window, max_over_ranks,
                  width: int = 4096, tolerance: bool = False) -> dict:
    """Check a one-peer-per-GPU f32 sum allreduce result on sampled windows, on every rank: for each window
    (the head, the tail and a random interior range of every shard) this rank regenerates every peer's
    synthetic bucket over that range (fmi_dev_fill_synthetic_at) and reduces them on its own GPU with the
    single-GPU fused kernel in allreduce_no_order order for its own rank (fmi_dev_reduce_tree). The sharded
    result (`window(start, count)` -> numpy) must equal it bit for bit (tolerance=False: the reference's
    bracketing) or lie within (N-1)·2^-24·Σ|x_p| of it (tolerance=True: RCCL's order). Returns the counts, max
    over ranks; "ok" is the verdict every rank agrees on."""
    import sys

    import numpy as np

    from . import device as fdev

    N, r = world, rank
    rng = np.random.default_rng(977 + r)
    starts = set()
    for j in range(N):
        lo = j * shard
        if lo >= n:
            break
        hi = min(n, lo + shard)
        starts.update({lo, max(lo, hi - width), int(rng.integers(lo, max(lo + 1, hi - width)))})
    peers = [fdev.Bucket(width, np.float32) for _ in range(N)]
    ref = fdev.Bucket(width, np.float32)
    mismatches = checked = 0
    worst = 0.0
    for st in sorted(starts):
        w = min(width, n - st)
        pv = [p.view(0, w) for p in peers]
        for p in range(N):
            pv[p].fill_synthetic(seed, p, first=st)
        rv = ref.view(0, w)
        fdev.reduce_tree(Op.SUM, Alg.ALLREDUCE, rv, pv, rank=r)
        got, want = window(st, w), rv.numpy()
        if tolerance:
            xs = np.stack([v.numpy() for v in pv]).astype(np.float64)
            bound = (N - 1) * 2.0 ** -24 * np.abs(xs).sum(axis=0)
            err = np.abs(got.astype(np.float64) - want.astype(np.float64))
            mismatches += int(np.count_nonzero(err > bound))
            worst = max(worst, float(np.max(err / np.maximum(bound, 1e-300))) if w else 0.0)
        else:
            bad = np.nonzero(got.view(np.uint32) != want.view(np.uint32))[0]
            if bad.size and mismatches == 0:  # where it went wrong, for the log (the line carries counts)
                i = int(bad[0])
                print(f"self_check rank {r}: first mismatch at element {st + i}: got {got[i]!r} want {want[i]!r} "
                      f"(shard {(st + i) // shard} of {N})", file=sys.stderr, flush=True)
            mismatches += int(bad.size)
        checked += w
    for b in peers + [ref]:
        b.free()
    mism, chk = max_over_ranks(float(mismatches), float(checked))
    res = {"ok": mism == 0, "mismatches": int(mism), "elements_checked_per_rank": int(chk),
           "windows_per_rank": len(starts),
           "against": ("single-GPU fused reduce_tree (allreduce_no_order order, own rank) of the same "
                       "synthetic buckets rebuilt on this GPU, " +
                       ("within (N-1)*2^-24*sum|x|" if tolerance else "bit-exact"))}
    if tolerance:
        res["max_err_over_bound"] = round(max_over_ranks(worst)[0], 4)
    return res


def local_equivalent(world: int, n: int, launches: int = 10, sets: int = 2) -> dict:
    """The like-for-like single-GPU anchor of the N > 1 line: the same world-peer f32 sum-allreduce of
    n-element buckets computed on ONE GPU (this rank's) by the fused kernel (fmi_dev_reduce_tree,
    allreduce_no_order order, every bucket resident in this GPU's HBM): HBM-bound, (N + 1)·S algorithmic
    bytes per launch. `GiB_s_reduced_buckets` = N·S / t, the unit of the line's `value`. Rotating sets;
    mean of back-to-back launches on the library stream (HIP events)."""
    import numpy as np

    from . import device as fdev

    N = world
    # each set's N inputs and its output one carved group (fmi_dev_alloc_group): the placement the
    # library gives the buckets a fused kernel streams together
    groups = [fdev.Bucket.group(N + 1, n, np.float32) for _ in range(sets)]
    for s, g in enumerate(groups):
        for p in range(N):
            g[p].fill_synthetic(42 + s, p)
    for g in groups:
        fdev.reduce_tree(Op.SUM, Alg.ALLREDUCE, g[N], g[:N])
    fdev.sync()
    e0, e1 = fdev.Event(), fdev.Event()
    e0.record()
    for k in range(launches):
        g = groups[k % sets]
        fdev.reduce_tree(Op.SUM, Alg.ALLREDUCE, g[N], g[:N])
    e1.record()
    e1.sync()
    ms = e0.elapsed_ms(e1) / launches
    e0.destroy()
    e1.destroy()
    for b in [x for g in groups for x in g]:
        b.free()
    S = n * 4
    return {"workload": f"{N} peers x {S >> 20} MiB f32 sum-allreduce on ONE GPU (fused {N}-way kernel, "
                        f"fmi_dev_reduce_tree): what the N-GPU step computes, without the exchange",
            "ms": round(ms, 4), "GiB_s_reduced_buckets": round(N * S / 2 ** 30 / (ms * 1e-3), 2),
            "hbm_frac": round((N + 1) * S / (ms * 1e-3) / 8e12, 4) if N > 1 else None,
            "launches": launches, "rotating_sets": sets}


class CommAllreduce:
    """The sharded allreduce through the product C-ABI (fmi_comm_*): one FMI peer per GPU (or 2^k peers,
    folded by a local round first), then fmi_comm_allreduce — all-to-all of shards + the fused kernel in
    the reference's order + all-gather (path TREE), RCCL reduce-scatter + all-gather (path RCCL), or the
    fused kernel over IPC-mapped peer windows (path DIRECT) — everything on the library's stream.

    torch.distributed only bootstraps: it broadcasts the 128-byte communicator id and provides the barriers
    and max-over-ranks of the timed region. `transport`: "rccl" (one process per GPU, torch's backend
    "nccl") or "proc" (processes of one node on the same or different GPUs, data staged through
    shared memory; with the "gloo" backend this runs the exact bench.py N>1 code on a single GPU)."""

    def __init__(self, group=None, path: str = "tree", transport: str = "rccl"):
        from .comm import Comm, Path, Transport, unique_id

        self.group = group if group is not None else dist.group.WORLD
        self.world = dist.get_world_size(self.group)
        self.rank = dist.get_rank(self.group)
        self.path = path
        self._path = {"tree": Path.TREE, "rccl": Path.RCCL, "direct": Path.DIRECT}[path]
        self.transport = transport
        tr = {"rccl": Transport.RCCL, "proc": Transport.PROC}[transport]
        # max-over-ranks and flags travel on the process group's own device: GPU for nccl, host for gloo
        self._red_dev = (torch.device("cuda", torch.cuda.current_device())
                         if dist.get_backend(self.group) == "nccl" else torch.device("cpu"))
        _lib.load()
        _lib.call("fmi_dev_init", torch.cuda.current_device())
        box = [None]
        if self.rank == 0:  # a failure here must still reach the broadcast every other rank is waiting in
            try:
                box[0] = unique_id(tr)
            except Exception as e:  # noqa: BLE001 - re-raised on every rank below
                box[0] = f"{type(e).__name__}: {e}"
        dist.broadcast_object_list(box, src=0, group=self.group)
        if isinstance(box[0], str):
            raise RuntimeError(f"communicator id on rank 0 failed: {box[0]}")
        self.comm = Comm(box[0], self.world, self.rank)

    def topology(self) -> dict:
        """What every rank runs on, all-gathered: the transport's own view of the communicator (RCCL:
        ncclCommCount / ncclCommUserRank / ncclCommCuDevice through fmi_comm_query), the torch device ordinal
        and the GPU's PCI bus id. ok: the transport saw exactly `world` ranks, each rank at its own index,
        and (RCCL) no two ranks share a GPU. PROC ranks may share one GPU by design: labelled, not an error."""
        from . import device as fdev
        from .comm import runtime_info

        q = self.comm.query()
        dev = torch.cuda.current_device()
        mine = {"rank": self.rank, "transport_count": q["count"], "transport_rank": q["rank"],
                "transport_device": q["device"], "torch_device": dev, "pci_bus_id": fdev.pci_bus_id(dev),
                "runtime": runtime_info()}
        every = [None] * self.world
        dist.all_gather_object(every, mine, group=self.group)
        return judge_topology(every, self.world, self.transport)

    def local_equivalent(self, n: int, launches: int = 10, sets: int = 2) -> dict:
        """local_equivalent() for this communicator's world size."""
        return local_equivalent(self.world, n, launches, sets)

    def max_over_ranks(self, *vals: float) -> List[float]:
        t = torch.tensor(vals, dtype=torch.float64, device=self._red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return [float(v) for v in t.tolist()]

    def shard_elems(self, n: int) -> int:
        per = -(-n // self.world)
        return -(-per // SHARD_ALIGN) * SHARD_ALIGN

    def bench(self, n: int, steps: int, warmup: int, sets: int = 2, peers_per_gpu: int = 1,
              overlap: bool = False, seed: int = 42, path: Optional[str] = None):
        """Timed loop: exactly `steps` allreduces of n-element f32 buckets, bracketed by barrier + device
        sync on both sides; returns (ms_per_step max over ranks, per-step local-round ms, extras). Step k
        reduces buffer set k % sets, whose peer buckets are the synthetic buckets (seed + set, peer).

        peers_per_gpu = 1: FMI's one peer per process, the bucket goes straight into fmi_comm_allreduce and
        is never modified, so extras["result"] = (out bucket, seed of the last step's set) can be checked
        against the same synthetic buckets (self_check). peers_per_gpu = 2: a local pairwise round first
        (round 0 of recursive doubling); it folds in place, so repeated steps drift and no check applies.
        overlap=True: the local round of step k+1 runs on a second stream while step k's exchange is in
        flight (steps are independent: each reduces its own buffer set); events order set reuse."""
        import time

        import numpy as np

        from . import device as fdev

        from .comm import Path

        if peers_per_gpu & (peers_per_gpu - 1):
            raise ValueError(f"{peers_per_gpu} peers per GPU: recursive doubling needs a power of two")
        path_name = self.path if path is None else path
        path_id = {"tree": Path.TREE, "rccl": Path.RCCL, "direct": Path.DIRECT}[path_name]
        direct = path_id == Path.DIRECT  # the reduced bucket must live in a symmetric window

        def first(s):
            b = self.comm.window(n, np.float32) if direct else fdev.Bucket(n, np.float32)
            return b.fill_synthetic(seed + s, peers_per_gpu * self.rank)

        bufs = [[first(s)] + [fdev.Bucket(n, np.float32).fill_synthetic(seed + s, peers_per_gpu * self.rank + j)
                              for j in range(1, peers_per_gpu)] for s in range(sets)]
        out = fdev.Bucket(n, np.float32)
        side = fdev.Stream() if overlap else None
        ready = [fdev.Event() for _ in range(sets)]
        freed = [fdev.Event() for _ in range(sets)]

        def step(k, ev=None):
            s = k % sets
            pair = bufs[s]
            if overlap:
                freed[s].wait_on(side)
            if ev:
                ev[0].record(side)
            if len(pair) == 2:  # round 0 of recursive doubling: pairs (2g, 2g+1)
                fdev.reduce_pair(Op.SUM, pair[0], pair[1], stream=side)
            elif len(pair) > 2:  # rounds 0..k-1: the 2^k-peer allreduce program over this GPU's peers
                fdev.reduce_tree(Op.SUM, Alg.ALLREDUCE, pair[0], pair, stream=side)
            if ev:
                ev[1].record(side)
            if overlap:
                ready[s].record(side)
                ready[s].wait_on(None)
            self.comm.allreduce(Op.SUM, pair[0], out, path=path_id)
            if overlap:
                freed[s].record(None)

        for k in range(warmup):
            step(k)
        fdev.sync()
        evs = [(fdev.Event(), fdev.Event()) for _ in range(steps)]
        dist.barrier(group=self.group)
        fdev.sync()
        self.comm.timing(True)  # event pairs around every shard-kernel launch of the timed steps
        t0 = time.perf_counter()
        for k in range(steps):
            step(k, evs[k])
        fdev.sync()
        dist.barrier(group=self.group)
        t1 = time.perf_counter()
        shard_ms, launches = self.comm.timing_read()
        self.comm.timing(False)
        step_ms, shard_avg_ms = self.max_over_ranks((t1 - t0) * 1e3 / steps, shard_ms / max(1, launches))
        kernel_ms = [a.elapsed_ms(b) for a, b in evs]
        for a, b in evs:
            a.destroy()
            b.destroy()
        gib = n * 4 / 2 ** 30
        extra = {
            "exchange": f"fmi_comm/{path_name}",
            "transport": self.transport,
            "shard_kernel_avg_ms": shard_avg_ms,
            "shard_kernel_launches": launches,
            "shard_elems": self.shard_elems(n),
            "algbw_GiB_s": round(gib / (step_ms * 1e-3), 2),
            "busbw_GiB_s": round(gib / (step_ms * 1e-3) * 2 * (self.world - 1) / self.world, 2),
        }
        if overlap:
            extra["overlap_steps"] = True
            side.destroy()
        for e in ready + freed:
            e.destroy()
        fdev.sync()
        for s, pair in enumerate(bufs):
            if direct:
                self.comm.window_free(pair[0])
            else:
                pair[0].free()
            for b in pair[1:]:
                b.free()
        if peers_per_gpu == 1 and steps > 0:
            extra["result"] = (out, seed + (steps - 1) % sets)
        else:
            out.free()
        return step_ms, kernel_ms, extra

    def self_check(self, out, n: int, seed: int, width: int = 4096, tolerance: bool = False) -> dict:
        """check_windows() of the out bucket of bench() (path TREE / DIRECT bit-exact, RCCL within tolerance)."""
        return check_windows(self.world, self.rank, self.shard_elems(n), n, seed,
                             lambda st, w: out.view(st, w).numpy(), self.max_over_ranks, width, tolerance)

    def shard_kernel(self, n: int, launches: int = 20, sets: int = 2) -> dict:
        """The dominant kernel of path TREE on this GPU: the fused N-way tree over n/N-element shards
        (what fmi_comm_allreduce launches between its all-to-all and all-gather), timed with events on the
        library stream over `launches` back-to-back launches on rotating input sets. Algorithmic HBM bytes
        per launch: (N + 1) · shard · 4 (N shard reads + 1 write)."""
        import numpy as np

        from . import device as fdev

        N = self.world
        shard = self.shard_elems(n)
        ins = [[fdev.Bucket(shard, np.float32).fill_synthetic(3 + s, p) for p in range(N)] for s in range(sets)]
        out = fdev.Bucket(shard, np.float32)
        for s in range(sets):
            fdev.reduce_tree(Op.SUM, Alg.ALLREDUCE, out, ins[s])
        fdev.sync()
        e0, e1 = fdev.Event(), fdev.Event()
        e0.record()
        for k in range(launches):
            fdev.reduce_tree(Op.SUM, Alg.ALLREDUCE, out, ins[k % sets])
        e1.record()
        e1.sync()
        ms = e0.elapsed_ms(e1) / launches
        e0.destroy()
        e1.destroy()
        for b in [out] + [x for s in ins for x in s]:
            b.free()
        ms = self.max_over_ranks(ms)[0]
        return {"kernel": f"tree_kernel<OpSum,float,kAllreduce,P={N}>" if N > 1 else "P=1: device copy",
                "kernel_avg_us": round(ms * 1e3, 2), "algorithmic_bytes_per_launch": (N + 1) * shard * 4,
                "launches": launches, "rotating_sets": sets}

    def check_direct(self, n: int) -> bool:
        """Path DIRECT against path TREE on the same window bucket: bit-identical on every rank?"""
        import numpy as np

        from . import device as fdev
        from .comm import Path

        w = self.comm.window(n, np.float32).fill_synthetic(5, self.rank)
        a, b = fdev.Bucket(n, np.float32), fdev.Bucket(n, np.float32)
        self.comm.allreduce(Op.SUM, w, a, path=Path.TREE)
        self.comm.allreduce(Op.SUM, w, b, path=Path.DIRECT)
        fdev.sync()
        same = bool(np.array_equal(a.numpy().view(np.uint32), b.numpy().view(np.uint32)))
        self.comm.window_free(w)
        a.free()
        b.free()
        return self.max_over_ranks(0.0 if same else 1.0)[0] == 0.0

    def host_bench(self, n: int, iters: int = 3, chunk: int = 64 << 18) -> dict:
        """Config C5: fmi_comm_allreduce_host of an n-element f32 bucket in page-locked host memory on every
        rank — H2D, sharded allreduce and D2H pipelined in `chunk`-element pieces. Returns the median wall
        time (max over ranks), the per-rank host-bucket rate and whether the result is right (every rank
        holds rank + 1, so every element must be N (N + 1) / 2, exact in f32). 64 MiB chunks: 16 MiB chunks
        measured up to 2x slower on some boxes."""
        import statistics
        import time

        import numpy as np

        from .device import PinnedArray

        send, recv = PinnedArray(n, np.float32), PinnedArray(n, np.float32)
        try:
            send.array[:] = np.float32(self.rank + 1)
            times = []
            for k in range(iters + 1):
                dist.barrier(group=self.group)
                t0 = time.perf_counter()
                self.comm.allreduce_host(Op.SUM, send.array, recv.array, path=self._path, chunk=chunk)
                dist.barrier(group=self.group)
                if k:
                    times.append(time.perf_counter() - t0)
            ms = self.max_over_ranks(statistics.median(times) * 1e3)[0]
            ok = bool(np.all(recv.array == np.float32(self.world * (self.world + 1) // 2)))
            ok = self.max_over_ranks(0.0 if ok else 1.0)[0] == 0.0
        finally:
            send.free()
            recv.free()
        return {"bucket_mib": n * 4 // (1 << 20), "chunk_mib": chunk * 4 / (1 << 20), "ms": round(ms, 3),
                "per_rank_GiB_s": round(n * 4 / 2 ** 30 / (ms * 1e-3), 2), "result_ok": ok}

    def destroy(self) -> None:
        self.comm.destroy()


def judge_topology(every: List[dict], world: int, transport: str) -> dict:
    """The verdict of CommAllreduce.topology over every rank's report (host logic, CPU-tested): ok when the
    transport saw exactly `world` ranks, each rank at its own index, and (RCCL) no two ranks share a GPU (PCI
    bus id). Several PROC ranks on one GPU is what that transport is for: labelled, not an error."""
    counts = sorted({e["transport_count"] for e in every})
    pci = [e["pci_bus_id"] for e in every]
    distinct = len(set(pci)) == len(pci)
    ranks_ok = len(every) == world and counts == [world] and all(e["transport_rank"] == e["rank"] for e in every)
    shared_ok = transport == "proc"
    res = {"transport": transport, "rccl_ranks": counts[0] if len(counts) == 1 else counts,
           "ranks": [{k: e[k] for k in ("transport_rank", "transport_device", "torch_device", "pci_bus_id")}
                     for e in every],
           "distinct_gpus": distinct, "ok": bool(ranks_ok and (distinct or shared_ok))}
    # the librccl and visibility environment: rank 0's, plus every rank that differs from it
    rt = [e.get("runtime") or {} for e in every]
    res["runtime"] = rt[0]
    differ = {e["rank"]: r for e, r in zip(every, rt) if r != rt[0]}
    if differ:
        res["runtime_differs"] = differ
    if transport != "rccl":
        res["rccl_ranks"] = None
        res["transport_ranks"] = counts[0] if len(counts) == 1 else counts
    if not distinct and shared_ok:
        res["note"] = "PROC transport: ranks share GPUs by design (single-GPU runs of the N > 1 path)"
    return res


def phase_breakdown(n: int, group=None, iters: int = 5) -> dict:
    """Untimed diagnostic for bench.py at N > 1: mean duration (ms, max over ranks) of each phase of the
    sharded allreduce of an n-element f32 bucket, measured with events on torch's stream — the local
    pairwise round, the all-to-all, the fused shard kernel, the all-gather, RCCL's reduce-scatter
    (the alternative to all-to-all + kernel) and RCCL's whole-bucket allreduce (reference point)."""
    group = group if group is not None else dist.group.WORLD
    world = dist.get_world_size(group)
    dev = torch.device("cuda", torch.cuda.current_device())
    eng = HipEngine(dev.index)
    per = -(-n // world)
    shard = -(-per // SHARD_ALIGN) * SHARD_ALIGN
    padded = shard * world
    a = torch.empty(padded, dtype=torch.float32, device=dev)
    b = torch.empty(padded, dtype=torch.float32, device=dev)
    eng.fill_synthetic(a, 7, 0)
    eng.fill_synthetic(b, 7, 1)
    staging = torch.empty(padded, dtype=torch.float32, device=dev)
    red = torch.empty(shard, dtype=torch.float32, device=dev)
    out = torch.empty(padded, dtype=torch.float32, device=dev)
    parts = [staging[j * shard:(j + 1) * shard] for j in range(world)]

    phases = {
        "local_pair": lambda: eng.reduce_pair(Op.SUM, a, b),
        "all_to_all": lambda: dist.all_to_all_single(staging, a, group=group),
        "shard_tree_kernel": lambda: eng.reduce_tree(Op.SUM, Alg.ALLREDUCE, red, parts, rank=0),
        "all_gather": lambda: dist.all_gather_into_tensor(out, red, group=group),
        "reduce_scatter": lambda: dist.reduce_scatter_tensor(red, a, group=group),
        # RCCL's own whole-bucket allreduce: the floor for any exchange built from RCCL collectives
        "rccl_allreduce_whole_bucket": lambda: dist.all_reduce(a, group=group),
    }
    result = {}
    for name, fn in phases.items():
        fn()
        torch.cuda.synchronize()
        dist.barrier(group=group)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        t = torch.tensor([e0.elapsed_time(e1) / iters], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        result[name] = round(float(t.item()), 4)
    return result
