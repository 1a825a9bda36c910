#!/usr/bin/env python3
"""Benchmark of FMI's bucket reduction on MI355X (BASELINE.json metric:
"GiB/s device-resident float32 sum-reduce, 256 MiB buckets, 1/2/4/8 GPU").

One *step* = one pass of the hot path over one batch of synthetic, HBM-resident buckets: every GPU holds
two peers' 256 MiB float32 buckets and performs the pairwise combine a = a + b — the reference's
`f.f(a, b)` (include/Communicator.h:180-189) on the device (config C2). The combine is element-wise and
pairs are independent, so at N > 1 the pairs shard over the GPUs with no data-path collective (weak
scaling, 2N peers); only the barrier + max-over-ranks timing crosses GPUs.
value = (N × 256 MiB of reduced bucket) / (wall time per step, max over ranks), in GiB/s.

Also reported (one JSON line on rank 0):
  roofline      — the pairwise kernel: algorithmic bytes 3·n·4 per launch ÷ its mean duration from HIP
                  events on the stream it runs on; peak = 8000 GB/s HBM3E; traffic from the committed
                  rocprofv3 PMC summary of the same kernel (profiles/).
  cpu_baseline  — (N = 1) oracle/cpu_baseline (a C++ port of the reference's CPU path) on this host: the
                  reference-faithful 6-copy adapter around std::transform, 1 thread, same 256 MiB buckets.
  config.allreduce, xgmi_roofline — (N > 1) the path with a real exchange step, measured after `value`:
                  the 2N-peer allreduce of 256 MiB buckets (config C4's shape) — local pairwise round, then
                  all-to-all of shards over RCCL/xGMI + the fused P-way kernel in allreduce_no_order order +
                  all-gather (fmi_amd/collectives.py), bit-identical to the reference's 2N-peer allreduce;
                  its step time, and its egress bytes per GPU against the N-1 xGMI links' peak.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MIB = 1 << 20
GIB = 1 << 30
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, MI355X_MICROARCH.md §Chip-level parameters
XGMI_LINK_GBS_PER_DIR = 76.8  # one xGMI link: 153.6 GB/s bidirectional (7 links per GPU, fully connected node)
METRIC = "GiB/s device-resident float32 sum-reduce, 256 MiB buckets, 1/2/4/8 GPU"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--bucket-mib", type=int, default=256)
    ap.add_argument("--sets", type=int, default=4, help="rotating bucket sets (defeats the 256 MiB MALL)")
    ap.add_argument("--path", default="tree", choices=["tree", "rccl", "direct"],
                    help="N>1 exchange: tree = all-to-all + fused kernel (bit-exact), rccl = reduce-scatter, "
                         "direct = fused kernel over IPC-mapped peer windows (bit-exact, fmi backend only)")
    ap.add_argument("--backend", default="fmi", choices=["fmi", "torch"],
                    help="N>1 exchange driver: fmi = the C-ABI communicator fmi_comm_* (RCCL transport), "
                         "torch = torch.distributed collectives + our kernels on torch's stream")
    ap.add_argument("--overlap-steps", action="store_true",
                    help="N>1, fmi backend: run step k+1's local round on a second stream during step k's exchange")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-diagnostics", action="store_true", help="skip the untimed N>1 phase breakdown")
    ap.add_argument("--diag-deadline", type=float, default=240.0,
                    help="seconds the N>1 allreduce measurement + diagnostics (run after `value`) may take before "
                         "the line is printed without the rest of them")
    ap.add_argument("--diag-direct", action="store_true",
                    help="N>1 diagnostics: also check and time path DIRECT (IPC-mapped peer windows)")
    ap.add_argument("--force-dist", action="store_true",
                    help="run the N>1 code path (RCCL exchange) even at world size 1 — plumbing check only")
    ap.add_argument("--cpu-reps", type=int, default=30, help="adapter combines timed (≈10 s of CPU work)")
    return ap.parse_args()


def pmc_traffic(kernel_substr: str):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC summary."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(path):
        return None, None
    try:
        data = json.load(open(path))
        for k in data.get("kernels", []):
            if kernel_substr in k.get("kernel", ""):
                return k.get("hbm_bytes_per_launch"), data.get("source")
    except Exception:
        return None, None
    return None, None


def cpu_baseline(args):
    exe = os.path.join(ROOT, "oracle", "build", "cpu_baseline")
    if not os.path.exists(exe):
        return None
    try:
        out = subprocess.run([exe, "--mode", "adapter", "--dtype", "f32", "--op", "sum", "--mib", str(args.bucket_mib),
                              "--reps", str(args.cpu_reps)], check=True, capture_output=True, text=True, timeout=600)
        adapter = json.loads(out.stdout.strip().splitlines()[-1])
        out = subprocess.run([exe, "--mode", "bare", "--dtype", "f32", "--op", "sum", "--mib", str(args.bucket_mib),
                              "--reps", "9"], check=True, capture_output=True, text=True, timeout=600)
        bare = json.loads(out.stdout.strip().splitlines()[-1])
        # the same loop over the host threads this job may use (OMP_NUM_THREADS): a CPU roofline for scale
        out = subprocess.run([exe, "--mode", "omp", "--dtype", "f32", "--op", "sum", "--mib", str(args.bucket_mib),
                              "--reps", "9"], check=True, capture_output=True, text=True, timeout=600)
        omp = json.loads(out.stdout.strip().splitlines()[-1])
    except Exception as e:  # the baseline is reported, never required
        return {"error": str(e)}
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {
        "value": round(adapter["bucket_gib_s"], 4),
        "unit": "GiB/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"reference-faithful adapter (include/Communicator.h:182-187, 6 bucket copies) around "
                   f"std::transform(std::plus<float>), 1 thread, {args.bucket_mib} MiB f32 pair, median of "
                   f"{adapter['reps']} after 1 warm-up: {adapter['median_ms']:.1f} ms/combine; bare std::transform "
                   f"1 thread: {bare['median_ms']:.2f} ms = {bare['bucket_gib_s']:.2f} GiB/s; host '{model}', "
                   f"{os.cpu_count()} CPUs visible"),
        "bare_loop_gib_s": round(bare["bucket_gib_s"], 4),
        "all_threads_loop": {"gib_s": round(omp["bucket_gib_s"], 4), "threads": omp["threads"],
                             "median_ms": round(omp["median_ms"], 3)},
        "c1": c1_host(),
    }


def c1_host():
    """Config C1 (CPU, no GPU): 2-peer f32 sum-allreduce of 1 MiB buckets through the C++ FMI::Communicator,
    peers as fork()ed processes over a socketpair channel, with the reference adapter (untagged lambda)
    and with the built-in in-place op (build/cpp/c1_bench, fmi_amd/cpp/tools/c1_bench.cpp)."""
    exe = os.path.join(ROOT, "build", "cpp", "c1_bench")
    if not os.path.exists(exe):
        return None
    try:
        out = subprocess.run([exe, "--mib", "1", "--reps", "41"], check=True, capture_output=True, text=True,
                             timeout=120)
        return json.loads(out.stdout.strip().splitlines()[-1])
    except Exception as e:  # reported, never required
        return {"error": str(e)}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if args.gpus > 1 and world == 1:
            raise SystemExit(f"--gpus {args.gpus} needs torch.distributed.run with {args.gpus} processes")
        args.gpus = world

    import numpy as np

    dist = None
    use_dist = world > 1 or args.force_dist
    if use_dist:
        # torch first: libfmi_dev.so then binds to the HIP runtime torch already loaded (one runtime
        # per process, shared streams/pointers with RCCL) — see DESIGN.md §Runtime.
        import torch
        import torch.distributed as dist

        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    import fmi_amd
    from fmi_amd import Bucket, Event, Op

    fmi_amd.init(local_rank)
    n = args.bucket_mib * MIB // 4
    nbytes = n * 4

    # ---- the timed measurement: every rank combines its own peer pairs (C2's unit of work) -------------
    sets = [tuple(Bucket(n, np.float32).fill_synthetic(42 + s, 2 * rank + j) for j in range(2))
            for s in range(args.sets)]
    fmi_amd.sync()

    def step(k):
        a, b = sets[k % len(sets)]
        fmi_amd.reduce_pair(Op.SUM, a, b)

    def bracket():  # barrier + device sync (both sides of the timed region)
        fmi_amd.sync()
        if dist is not None:
            dist.barrier()
            torch.cuda.synchronize()

    for k in range(args.warmup):
        step(k)
    bracket()
    # Timed region: exactly K back-to-back launches on the library stream; two HIP events on that stream
    # bracket them (no markers between launches).
    ev0, ev1 = Event(), Event()
    t0 = time.perf_counter()
    ev0.record()
    for k in range(args.steps):
        step(k)
    ev1.record()
    bracket()
    t1 = time.perf_counter()
    step_ms = (t1 - t0) * 1e3 / args.steps
    # mean launch duration over the timed region (includes the ~1-2 us dispatch gaps between launches)
    kernel_avg_ms = ev0.elapsed_ms(ev1) / args.steps
    if dist is not None:  # max over ranks
        step_ms, kernel_avg_ms = _max_over_ranks(dist, step_ms, kernel_avg_ms)
    # diagnostic, untimed: per-launch event pairs give the launch duration without the gaps
    probe = min(args.steps, 32)
    pairs = [(Event(), Event()) for _ in range(probe)]
    for k in range(probe):
        pairs[k][0].record()
        step(k)
        pairs[k][1].record()
    fmi_amd.sync()
    isolated_us = 1e3 * sum(a.elapsed_ms(b) for a, b in pairs) / probe
    for a, b in sets:
        a.free()
        b.free()
    dominant = "pair_tile"
    algo_bytes = 3 * nbytes
    if world == 1:
        workload = "C2: 1-GPU pairwise float32 sum-reduce of two 256 MiB device-resident peer buckets"
        parallelism = "single GPU (2 peers resident)"
    else:
        workload = (f"C2 on every GPU: {world} GPUs each combine their own pair of 256 MiB device-resident "
                    f"peer buckets ({2 * world} peers)")
        parallelism = f"dp{world}: pairs sharded over GPUs, no data-path collective (barrier + max-over-ranks timing)"
    roofline_extra = {"kernel_avg_us_isolated": round(isolated_us, 2),
                      "kernel_avg_source": "HIP events bracketing the K timed launches on the library stream"
                                           + (", max over ranks" if dist is not None else "")}
    value = args.gpus * (nbytes / GIB) / (step_ms * 1e-3)
    achieved = algo_bytes / (kernel_avg_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(dominant)
    line = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": args.gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_ms, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (splitmix64 counter generator, SURVEY.md §8d), device-resident in HBM",
        "config": {"workload": workload, "bucket_mib": args.bucket_mib, "elements": n,
                   "peers": 2 * args.gpus, "parallelism": parallelism, "rotating_sets": args.sets},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel": dominant, "kernel_avg_us": round(kernel_avg_ms * 1e3, 2),
                     "algorithmic_bytes_per_launch": algo_bytes,
                     "traffic_source": traffic_src},
    }
    line["roofline"].update(roofline_extra)
    if rank == 0 and not use_dist and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args)
    emit = _Emitter(line, rank)
    watchdog = None
    if use_dist:
        # The timed measurement is complete and `line` holds it. The sharded allreduce and the diagnostics
        # below run other paths; a per-rank deadline (kept until teardown is done, since a rank that failed
        # alone would leave its peers waiting in a collective) guarantees that a hang there cannot cost
        # the measured line.
        state = line["config"]["allreduce"] = {}
        watchdog = threading.Timer(args.diag_deadline, emit.deadline, args=(state,))
        watchdog.daemon = True
        watchdog.start()
        try:
            ar = measure_allreduce(args, n, world, dist, line, state)
            if not args.no_diagnostics:
                state["diagnostics"] = {}
                run_diagnostics(args, ar, n, dist, state["diagnostics"])
        except Exception as e:  # never fails the measured line
            state["failed"] = f"{type(e).__name__}: {e}"
    emit.emit()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if watchdog is not None:
        watchdog.cancel()


class _Emitter:
    """Prints the one JSON line exactly once (rank 0), from the main thread or from the diagnostics
    deadline — whichever comes first."""

    def __init__(self, line, rank):
        self.line, self.rank = line, rank
        self.lock = threading.Lock()
        self.done = False

    def emit(self):
        with self.lock:
            if self.done:
                return
            self.done = True
            if self.rank == 0:
                try:
                    text = json.dumps(self.line)
                except RuntimeError:  # the main thread was still writing the after-`value` section
                    self.line["config"]["allreduce"] = {"incomplete": "deadline reached while recording"}
                    text = json.dumps(self.line)
                print(text, flush=True)

    def deadline(self, state):
        state["incomplete"] = "deadline reached; the timed measurement (value, roofline) is unaffected"
        self.emit()
        print("bench: diagnostics deadline reached, exiting", file=sys.stderr, flush=True)
        os._exit(0)


def _max_over_ranks(dist, *vals):
    import torch

    t = torch.tensor(vals, dtype=torch.float64, device=torch.cuda.current_device())
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.tolist()]


def measure_allreduce(args, n, world, dist, line, state):
    """Config C4's shape at this node size: the 2N-peer float32 sum-allreduce of 256 MiB buckets, two peers
    per GPU (the local pairwise round, then the exchange over xGMI: all-to-all of shards + fused kernel in
    allreduce_no_order order + all-gather, bit-exact with the reference's 2N-peer bracketing). K steps,
    barrier + sync on both sides, max over ranks. Reported beside `value`, with its xGMI roofline: per step
    every GPU sends (N-1)/N of its bucket in the all-to-all (or reduce-scatter) and (N-1)/N in the
    all-gather over its N-1 direct links to the other GPUs (fully connected node)."""
    from fmi_amd.collectives import CommAllreduce, ShardedAllreduce

    ar = None
    backend = args.backend
    if backend == "fmi":
        try:  # the product C-ABI communicator (fmi_comm_*, RCCL transport)
            ar = CommAllreduce(dist.group.WORLD, path=args.path)
        except Exception as e:  # setup only: every rank fails alike, before any timed work
            print(f"fmi_comm setup failed ({e}); using the torch.distributed exchange", file=sys.stderr)
            backend = "torch"
    if ar is None:
        ar = ShardedAllreduce(dist.group.WORLD, path=args.path, force_exchange=args.force_dist)
    if isinstance(ar, CommAllreduce):
        step_ms, kernel_ms, extra = ar.bench(n, steps=args.steps, warmup=args.warmup, sets=args.sets,
                                             overlap=args.overlap_steps)
    else:
        step_ms, kernel_ms, extra = ar.bench(n, steps=args.steps, warmup=args.warmup, sets=args.sets)
    extra.pop("kernel_algo_bytes", None)
    state.update({
        "workload": f"C4-shaped: {2 * world}-peer float32 sum-allreduce of 256 MiB buckets, 2 peers per GPU",
        "path": {"tree": "all-to-all + fused tree kernel + all-gather over RCCL (bit-exact)",
                 "rccl": "RCCL reduce-scatter + all-gather",
                 "direct": "fused tree over IPC-mapped peer windows + direct gather (bit-exact)"}[args.path],
        "backend": backend,
        "ms_per_step": round(step_ms, 5),
        "GiB_s_reduced_buckets": round(world * (n * 4 / GIB) / (step_ms * 1e-3), 2),
        "local_pair_kernel_ms": round(sum(kernel_ms) / len(kernel_ms), 5),
    })
    state.update(extra)
    if world > 1:
        egress = 2 * (world - 1) * n * 4 / world
        xg = egress / (step_ms * 1e-3) / 1e9
        xpeak = (world - 1) * XGMI_LINK_GBS_PER_DIR
        line["xgmi_roofline"] = {"bound": "xgmi", "achieved": round(xg, 1), "peak": round(xpeak, 1), "unit": "GB/s",
                                 "frac": round(xg / xpeak, 4), "bytes_per_step_per_gpu": int(egress),
                                 "kernel": "sharded allreduce step (config.allreduce)",
                                 "note": "egress bytes per GPU / allreduce step time (local round included); "
                                         "peak = N-1 links x 76.8 GB/s per direction"}
    return ar


def run_diagnostics(args, ar, n, dist, diag):
    """Untimed N>1 diagnostics for the next optimisation round, each max over ranks: the other exchange
    path's step time, the per-phase breakdown, the other step schedule, config C5 (host-resident buckets)
    and, last and only with --diag-direct, path DIRECT (xGMI reads of IPC-mapped peer windows). Results are
    written into `diag` as they complete."""
    from fmi_amd.collectives import CommAllreduce, phase_breakdown

    other = "rccl" if args.path == "tree" else "tree"
    short = dict(steps=max(10, args.steps // 4), warmup=3, sets=min(2, args.sets))
    if isinstance(ar, CommAllreduce):
        from fmi_amd.comm import Path

        saved = ar._path
        ar._path = Path.RCCL if other == "rccl" else Path.TREE
        alt_ms, _, _ = ar.bench(n, **short)
        ar._path = saved
    else:
        saved = ar.path
        ar.path = other
        alt_ms, _, _ = ar.bench(n, **short)
        ar.path = saved
    diag[f"ms_per_step_path_{other}"] = round(alt_ms, 5)
    diag["phase_ms"] = phase_breakdown(n, dist.group.WORLD)
    if not isinstance(ar, CommAllreduce):
        return
    # the other step schedule: local round of step k+1 overlapped with step k's exchange, or not
    ov_ms, _, _ = ar.bench(n, steps=short["steps"], warmup=3, sets=args.sets, overlap=not args.overlap_steps)
    diag["ms_per_step_no_overlap" if args.overlap_steps else "ms_per_step_overlap_steps"] = round(ov_ms, 5)
    # config C5: 1 GiB host (pinned) bucket per rank, H2D + allreduce + D2H pipelined
    try:
        diag["c5_host_allreduce_1GiB"] = ar.host_bench(GIB // 4)
    except Exception as e:  # diagnostic only; never fails the bench line
        diag["c5_host_allreduce_1GiB"] = f"failed: {e}"
    # path DIRECT: bit-identical to TREE on this node? and its step time. Opt-in (--diag-direct): its
    # cross-process IPC mappings have only run on the LOCAL transport so far, and a fault there would take
    # the whole line with it.
    if not args.diag_direct:
        diag["path_direct"] = "not run (opt-in: --diag-direct)"
    elif args.path != "direct":
        saved = ar._path
        try:
            ok = ar.check_direct(1 << 20)
            ar._path = Path.DIRECT
            d_ms, _, _ = ar.bench(n, **short)
            diag["path_direct"] = {"bit_identical_to_tree": ok, "ms_per_step": round(d_ms, 5)}
        except Exception as e:  # window setup fails on every rank alike (all-or-nothing)
            diag["path_direct"] = f"unavailable: {e}"
        finally:
            ar._path = saved


if __name__ == "__main__":
    main()
