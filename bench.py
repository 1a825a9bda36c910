#!/usr/bin/env python3
"""Benchmark of FMI's bucket reduction on MI355X (BASELINE.json metric:
"GiB/s device-resident float32 sum-reduce, 256 MiB buckets, 1/2/4/8 GPU").

N = 1 (config C2). One *step* = one pairwise combine a = a + b of two 256 MiB float32 peer buckets
resident in HBM — the reference's `f.f(a, b)` (include/Communicator.h:180-189) on the device, rotating over
16 buffer sets (8 GiB; the rotation runs on from the warm-up, so no step re-reads a bucket the 256 MB
Infinity Cache still holds, see --sets). value = 256 MiB / (wall time per step). After the timed region every
set's bucket is checked bit for bit against numpy's float32 a + b repeated once per launch of that set, on three
windows (`self_check`); a mismatch prints the line and exits 1.

N > 1 (config C4's shape at the metric's bucket size). One *step* = the N-peer float32 sum-allreduce of
256 MiB buckets, ONE FMI peer per GPU (one process per GPU), through the product C-ABI communicator
fmi_comm_allreduce: all-to-all of N shards over RCCL/xGMI -> the fused N-way kernel in the reference's
allreduce_no_order order (src/comm/PeerToPeer.cpp:96-130) on every GPU's shard -> all-gather (path TREE,
bit-identical to the reference's N-peer allreduce). value = N x 256 MiB / (wall time per step, max over
ranks): reduced bucket bytes delivered per second, summed over the GPUs (weak scaling: 256 MiB per GPU).
The result of the last timed step is checked on every rank against the single-GPU fused kernel over the same
synthetic buckets rebuilt locally (`self_check`); a mismatch prints the line and exits 1.

Also reported (one JSON line on rank 0):
  roofline      — the dominant HBM kernel: N = 1 the pairwise kernel (3·n·4 bytes per launch), N > 1 the
                  fused N-way shard kernel ((N+1)·shard·4 bytes), duration from HIP events on the library
                  stream it runs on; peak = 8000 GB/s HBM3E; traffic from the committed rocprofv3 PMC summary.
  xgmi_roofline — (N > 1) egress bytes per GPU per step, 2·(N−1)/N·S, over the step time, against the N−1
                  xGMI links' peak.
  c4            — (N > 1) config C4 itself: N peers × 1 GiB f32, paths TREE and RCCL, algbw / busbw, each
                  self-checked (TREE bit-exact, RCCL within (N−1)·2^-24·Σ|x|).
  c5            — config C5: N = 1 three self-checked blocks (c5_single: the P = 1 copy, a 1 GiB page-locked
                  pair through fmi_host_reduce_pair, and the whole 8 x 1 GiB workload as 8 LOCAL ranks on
                  this GPU); N > 1 every rank's 1 GiB page-locked bucket through fmi_comm_allreduce_host.
  cpu_baseline  — (N = 1) the reference's own CPU combine (oracle/_ref) on this host, its C++ port
                  (oracle/cpu_baseline) beside it as `port_value`.
  c3            — (N = 1) config C3's kernels: i64 max pair 64 MiB, f32 peer scan 8 x 64 MiB, fraction of peak.
  c4_one_gpu    — (N = 1) config C4's data on one GPU: 8 peers x 1 GiB through the fused 8-way allreduce kernel.
  diagnostics   — (N > 1) the replicated-pair rate (C2 on every GPU, no exchange), the per-phase breakdown
                  of the exchange and, opt-in, path DIRECT.
Everything after `value` runs under a per-rank deadline (--diag-deadline); if it expires, rank 0 prints the
line with a top-level "incomplete" field and every rank exits.
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
    ap.add_argument("--c4-mib", type=int, default=1024, help="N>1: bucket per peer of the c4 block (config C4)")
    ap.add_argument("--sets", type=int, default=16,
                    help="N=1: rotating bucket sets. The pair kernel's sc1 tiles (1 of 8) leave their output lines in "
                         "the 256 MB MALL, which nontemporal reads do not displace: 16 sets put 15 x 32 MiB of sc1 "
                         "writes between two uses of a set, so no step re-reads a bucket from the MALL")
    ap.add_argument("--dist-sets", type=int, default=4, help="N>1: rotating bucket sets of the sharded allreduce")
    ap.add_argument("--path", default="tree", choices=["tree", "rccl", "direct"],
                    help="N>1 headline exchange: tree = all-to-all + fused kernel (bit-exact), rccl = "
                         "reduce-scatter + all-gather, direct = fused kernel over IPC-mapped peer windows")
    ap.add_argument("--transport", default="rccl", choices=["rccl", "proc"],
                    help="N>1: rccl = one process per GPU over RCCL/xGMI (torch backend nccl); proc = processes "
                         "of one node sharing GPUs through shared-memory staging (torch backend gloo) — runs this "
                         "exact N>1 code with several ranks on one GPU (tests)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c5", action="store_true", help="skip the host-bucket (C5) measurement")
    ap.add_argument("--no-c3", action="store_true", help="N=1: skip the config C3 kernels (i64 max, peer scan)")
    ap.add_argument("--no-c4", action="store_true",
                    help="N=1: skip config C4 on one GPU (8 peers x 1 GiB through the fused 8-way allreduce kernel)")
    ap.add_argument("--c5-mib", type=int, default=1024, help="host bucket per rank of the c5 block (config C5)")
    ap.add_argument("--no-diagnostics", action="store_true", help="N>1: skip the untimed diagnostics")
    ap.add_argument("--no-numa-bind", action="store_true",
                    help="N>1: do not pin each rank to its GPU's NUMA node (default: pinned when the host has several)")
    ap.add_argument("--diag-deadline", type=float, default=240.0,
                    help="seconds everything after `value` (c4, c5, diagnostics) may take before the line is "
                         "printed without the rest of it")
    ap.add_argument("--diag-direct", action="store_true", help="N>1 diagnostics: also check and time path DIRECT")
    ap.add_argument("--diag-pipeline", action="store_true",
                    help="N>1 diagnostics: also time the EXPERIMENTAL pipelined allreduce (FMI_TUNE_COMM_PIPELINE 4 / 8: "
                         "two RCCL communicators in flight at once, not yet run across GPUs)")
    ap.add_argument("--measure-deadline", type=float, default=900.0,
                    help="N>1: seconds the measurement up to `value` (setup, warm-up, timed steps, self-check) may "
                         "take; past it the rank names the phase it is stuck in on stderr and exits with status 3")
    ap.add_argument("--force-dist", action="store_true",
                    help="run the N>1 code path (fmi_comm over RCCL) even at world size 1 — plumbing check; the one "
                         "rank then runs the full exchange with itself (FMI_TUNE_COMM_ONE_RANK_EXCHANGE)")
    ap.add_argument("--cpu-reps", type=int, default=30, help="adapter combines timed (≈10 s of CPU work)")
    ap.add_argument("--allow-exchange-fallback", action="store_true",
                    help="N>1: if the fmi_comm communicator fails, report the torch.distributed-exchange rate as `value` "
                         "and exit 0. Default: that rate goes to `fallback_value`, `value` is null and the run exits 1, "
                         "so a product failure cannot pass as a scaling point (top-level `exchange` names whose "
                         "exchange was measured either way)")
    return ap.parse_args()


def pmc_traffic(kernel_substr: str, algo_bytes: int):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC summary: the entry whose
    instantiation contains `kernel_substr` AND whose launch moved `algo_bytes` algorithmic bytes (within
    1 %). One instantiation is profiled at several shapes (the 8-way tree at N = 8's 32 MiB shards and at
    C3's 64 MiB buckets): a launch of another shape reports nothing rather than another launch's bytes."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(path):
        return None, None
    try:
        data = json.load(open(path))
        hits = [k for k in data.get("kernels", []) if kernel_substr in k.get("kernel", "")
                and k.get("algorithmic_bytes_per_launch")
                and abs(k["algorithmic_bytes_per_launch"] / algo_bytes - 1) < 0.01]
    except Exception:
        return None, None
    if len(hits) != 1:  # absent, or ambiguous (several instantiations match): report nothing rather than a wrong kernel's bytes
        return None, None
    return hits[0].get("hbm_bytes_per_launch"), hits[0].get("source", data.get("source"))


def reference_combine_ms(n: int, reps: int):
    """The REFERENCE's own combine on one host thread: oracle/_ref's fmi_ref_time_combine with the vector adapter
    (include/Communicator.h:180-189 restated, boost being absent; include/utils/Function.h:11-13's by-value
    operator() compiled from the reference's header) around std::plus<float>, median ms of `reps`. None if
    oracle/_ref is not built."""
    try:
        from oracle import fmi_ref

        if not fmi_ref.available():
            return None, "oracle/_ref not built"
        return fmi_ref.time_combine(1, n, reps, adapter=True), None
    except Exception as e:  # reported, never required
        return None, f"{type(e).__name__}: {e}"


def cpu_baseline(args):
    """`value` is the reference's own adapter combine (oracle/_ref, "kind": "reference") of the headline pair on one
    host thread; the port's (oracle/cpu_baseline.cpp) stands beside it as `port_value` with their ratio. Only if
    oracle/_ref is missing does the port become `value` ("kind": "port")."""
    exe = os.path.join(ROOT, "oracle", "build", "cpu_baseline")
    if not os.path.exists(exe):
        return None
    n = args.bucket_mib * MIB // 4
    ref_ms, ref_err = reference_combine_ms(n, args.cpu_reps)
    try:
        port_reps = max(5, args.cpu_reps // 3) if ref_ms is not None else args.cpu_reps
        out = subprocess.run([exe, "--mode", "adapter", "--dtype", "f32", "--op", "sum", "--mib", str(args.bucket_mib),
                              "--reps", str(port_reps)], check=True, capture_output=True, text=True, timeout=600)
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
    gib = args.bucket_mib / 1024
    port_gib_s = adapter["bucket_gib_s"]
    if ref_ms is not None:
        value, kind = gib / (ref_ms * 1e-3), "reference"
        sample = (f"the reference's own adapter combine (oracle/_ref: include/utils/Function.h's by-value operator() "
                  f"compiled from the reference's header, include/Communicator.h:180-189's vector adapter restated) "
                  f"around std::plus<float>, 1 thread, {args.bucket_mib} MiB f32 pair, median of {args.cpu_reps}: "
                  f"{ref_ms:.1f} ms/combine; the port (oracle/cpu_baseline.cpp) {adapter['median_ms']:.1f} ms; bare "
                  f"std::transform 1 thread: {bare['median_ms']:.2f} ms = {bare['bucket_gib_s']:.2f} GiB/s; host "
                  f"'{model}', {os.cpu_count()} CPUs visible")
    else:
        value, kind = port_gib_s, "port"
        sample = (f"port of the reference's adapter (include/Communicator.h:182-187, 6 bucket copies) around "
                  f"std::transform(std::plus<float>), 1 thread, {args.bucket_mib} MiB f32 pair, median of "
                  f"{adapter['reps']} after 1 warm-up: {adapter['median_ms']:.1f} ms/combine ({ref_err}); bare "
                  f"std::transform 1 thread: {bare['median_ms']:.2f} ms = {bare['bucket_gib_s']:.2f} GiB/s; host "
                  f"'{model}', {os.cpu_count()} CPUs visible")
    line = {
        "value": round(value, 4),
        "unit": "GiB/s",
        "cores": 1,
        "kind": kind,
        "sample": sample,
        "port_value": round(port_gib_s, 4),
        "reference_combine_ms": round(ref_ms, 2) if ref_ms is not None else None,
        "port_combine_ms": round(adapter["median_ms"], 2),
        "reference_over_port": round(ref_ms / adapter["median_ms"], 3) if ref_ms is not None else None,
        "bare_loop_gib_s": round(bare["bucket_gib_s"], 4),
        "all_threads_loop": {"gib_s": round(omp["bucket_gib_s"], 4), "threads": omp["threads"],
                             "median_ms": round(omp["median_ms"], 3),
                             "note": f"OMP_NUM_THREADS = {os.environ.get('OMP_NUM_THREADS')}: the CPU share the "
                                     f"box allots one GPU's job, and so this box's CPU roofline; os.cpu_count() = "
                                     f"{os.cpu_count()} counts the whole machine, and the same loop on that many "
                                     "threads ran 52x slower (2.77 GiB/s, profiles/r04_allcores_bench.json)"},
    }
    if ref_err:
        line["reference_error"] = ref_err
    line.update({
        "c1": c1_host(),
        "c1_reference": c1_reference(),
        "c2_reference": c2_reference(args.bucket_mib, adapter["median_ms"], ref_ms),
        "c3": c3_cpu(exe),
        "c4_reference": c4_reference(),
    })
    return line


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


def c1_reference(reps: int = 41) -> dict:
    """Config C1 through the REFERENCE's own collective code: oracle/_ref (src/comm/PeerToPeer.cpp compiled
    unmodified; prebuilt, it travels with the tree) runs the 2-peer f32 sum-allreduce of 1 MiB buckets, peers as
    threads over in-memory FIFOs (a memcpy per message, no TCP), combining through the reference's vector
    adapter (restated: include/Communicator.h needs boost) and through std::transform in place."""
    try:
        from oracle import fmi_ref

        if not fmi_ref.available():
            return {"error": "oracle/_ref not built"}
        n = MIB // 4
        ad = fmi_ref.time_allreduce(2, n, reps, adapter=True)
        bi = fmi_ref.time_allreduce(2, n, reps, adapter=False)
    except Exception as e:  # reported, never required
        return {"error": f"{type(e).__name__}: {e}"}
    out = {"config": "C1", "kind": "reference", "peers": 2, "bucket_mib": 1, "reps": reps,
           "code": "reference src/comm/PeerToPeer.cpp (allreduce_no_order), compiled unmodified (oracle/_ref)",
           "transport": "peer threads, in-memory FIFOs (oracle/ref_harness.cpp)",
           "adapter_ms": round(ad, 4), "builtin_inplace_ms": round(bi, 4),
           "adapter_gib_s": round(1 / 1024 / (ad * 1e-3), 4), "builtin_inplace_gib_s": round(1 / 1024 / (bi * 1e-3), 4)}
    try:  # the same reference allreduce with f.f bound to the product's C-ABI
        from fmi_amd import _lib

        gpu = fmi_ref.time_allreduce_bound(2, n, reps, fmi_ref.Binding.from_library(_lib.load()))
        out["gpu_combine_ms"] = round(gpu, 4)
        out["gpu_combine"] = ("every f.f is fmi_host_reduce_pair from libfmi_dev.so (passed by address; the "
                              "reference's pageable buckets: staged H2D / kernel / D2H per combine); bit-identity "
                              "with the CPU combine: tests/test_gpu_ref_binding.py")
    except Exception as e:  # reported, never required
        out["gpu_combine_ms"] = None
        out["gpu_combine_error"] = f"{type(e).__name__}: {e}"
    return out


def c2_reference(bucket_mib: int, port_combine_ms: float, one_thread_ms=None, reps: int = 5) -> dict:
    """The headline size through the REFERENCE's own code: its 2-peer f32 sum-allreduce of `bucket_mib` buckets
    (src/comm/PeerToPeer.cpp:96-130: per peer one exchange, one combine f.f at :119, the result memcpy at :129),
    peers as threads over in-memory FIFOs, with the vector adapter and with std::transform in place. A third
    run with the reference's no-op combine (its barrier's, PeerToPeer.cpp:30) times the transport and copies
    alone, so allreduce - no-op = the combine inside the reference. The reference's adapter combine is also timed
    outside any collective, on one thread (set beside the port's adapter combine, `value`: they agree when the
    ratio is within 1 +- 0.10) and on two threads at once (what the allreduce's two peers do)."""
    try:
        from oracle import fmi_ref

        if not fmi_ref.available():
            return {"error": "oracle/_ref not built"}
        n = bucket_mib * MIB // 4
        ad = fmi_ref.time_allreduce(2, n, reps, adapter=True)
        bi = fmi_ref.time_allreduce(2, n, reps, adapter=False)
        nop = fmi_ref.time_allreduce(2, n, reps, adapter="nop")
        one = one_thread_ms if one_thread_ms is not None else fmi_ref.time_combine(1, n, reps, adapter=True)
        two = fmi_ref.time_combine(2, n, reps, adapter=True)
    except Exception as e:  # reported, never required
        return {"error": f"{type(e).__name__}: {e}"}
    try:  # the same allreduce with every f.f bound to the product's C-ABI
        from fmi_amd import _lib

        gpu = fmi_ref.time_allreduce_bound(2, n, reps, fmi_ref.Binding.from_library(_lib.load()))
    except Exception as e:  # reported, never required
        gpu = f"{type(e).__name__}: {e}"
    combine = ad - nop
    ratio = one / port_combine_ms
    return {"config": "C2 size", "kind": "reference", "peers": 2, "bucket_mib": bucket_mib, "reps": reps,
            "code": "reference src/comm/PeerToPeer.cpp (allreduce_no_order), compiled unmodified (oracle/_ref)",
            "adapter_allreduce_ms": round(ad, 2), "builtin_inplace_allreduce_ms": round(bi, 2),
            "nop_combine_allreduce_ms": round(nop, 2),
            "adapter_allreduce_gib_s": round(bucket_mib / 1024 / (ad * 1e-3), 4),
            "combine_in_reference_allreduce_ms": round(combine, 2),
            "reference_adapter_combine_1_thread_ms": round(one, 2),
            "reference_adapter_combine_2_threads_ms": round(two, 2),
            "port_adapter_combine_ms": round(port_combine_ms, 2),
            "gpu_combine_allreduce_ms": round(gpu, 2) if isinstance(gpu, float) else gpu,
            "gpu_combine": "the same reference allreduce with every f.f = fmi_host_reduce_pair (its pageable buckets, "
                           "staged through the GPU); bits: tests/test_gpu_ref_binding.py",
            "reference_over_port": round(ratio, 3), "agrees_within_10pct": bool(abs(ratio - 1) <= 0.10),
            "note": "reference_over_port compares like with like: the reference's adapter combine on one thread "
                    "against the port's (value). Inside the 2-peer allreduce both peers combine at once; "
                    "combine_in_reference_allreduce_ms (allreduce - no-op allreduce) is to be read against "
                    "reference_adapter_combine_2_threads_ms, the same two combines run concurrently outside it"}


def c3_cpu(exe: str, reps: int = 5) -> dict:
    """Config C3 on the host, beside the line's `c3` GPU block (BASELINE.md's CPU-baseline plan): the int64 max
    combine of two 64 MiB buckets through the port (oracle/cpu_baseline.cpp: the reference's vector adapter around
    its std::max functor, python/PythonCommunicator.h:137-143, and the bare loop), and the REFERENCE's own scan
    (PeerToPeer::scan -> scan_no_order, PeerToPeer.cpp:132-184, compiled unmodified in oracle/_ref) of 8 peers'
    64 MiB f32 buckets, peers as threads, through the vector adapter and std::transform in place."""
    out = {"config": "C3"}
    try:
        runs = {}
        for mode in ("adapter", "bare"):
            r = subprocess.run([exe, "--mode", mode, "--dtype", "i64", "--op", "max", "--mib", "64", "--reps",
                                str(reps)], check=True, capture_output=True, text=True, timeout=300)
            runs[mode] = json.loads(r.stdout.strip().splitlines()[-1])
        out["i64_max_pair_64MiB"] = {"kind": "port", "threads": 1, "reps": reps,
                                     "adapter_ms": round(runs["adapter"]["median_ms"], 3),
                                     "bare_ms": round(runs["bare"]["median_ms"], 3),
                                     "adapter_gib_s": round(runs["adapter"]["bucket_gib_s"], 4),
                                     "bare_gib_s": round(runs["bare"]["bucket_gib_s"], 4)}
    except Exception as e:  # reported, never required
        out["i64_max_pair_64MiB"] = {"error": f"{type(e).__name__}: {e}"}
    try:
        from oracle import fmi_ref

        if not fmi_ref.available():
            raise RuntimeError("oracle/_ref not built")
        n = 64 * MIB // 4
        ad = fmi_ref.time_scan(8, n, 3, adapter=True)
        bi = fmi_ref.time_scan(8, n, 3, adapter=False)
        out["f32_scan_P8_64MiB"] = {
            "kind": "reference", "peers": 8, "reps": 3,
            "code": "reference src/comm/PeerToPeer.cpp (scan_no_order), compiled unmodified (oracle/_ref); peers as "
                    "threads over in-memory FIFOs",
            "adapter_ms": round(ad, 2), "builtin_inplace_ms": round(bi, 2),
            "adapter_gib_s_of_outputs": round(8 * 64 / 1024 / (ad * 1e-3), 4)}
    except Exception as e:  # reported, never required
        out["f32_scan_P8_64MiB"] = {"error": f"{type(e).__name__}: {e}"}
    return out


def c4_reference(peers: int = 8, mib: int = 1024) -> dict:
    """Config C4 through the REFERENCE's own code on the host: its 8-peer f32 sum-allreduce of 1 GiB buckets
    (PeerToPeer.cpp:96-130: 3 rounds of exchange + combine per peer), peers as threads over in-memory FIFOs, once
    with std::transform in place and once through the vector adapter (its 6 bucket copies per combine: up to
    ~72 GiB of host memory at once, so only where MemAvailable holds twice that). One repetition each: the
    in-place run takes seconds, the adapter run tens of seconds. Beside it: the line's `c4_one_gpu`."""
    try:
        from oracle import fmi_ref

        if not fmi_ref.available():
            return {"error": "oracle/_ref not built"}
        n = mib * MIB // 4
        out = {"config": "C4", "kind": "reference", "peers": peers, "bucket_mib": mib, "reps": 1,
               "code": "reference src/comm/PeerToPeer.cpp (allreduce_no_order), compiled unmodified (oracle/_ref); "
                       "peers as threads over in-memory FIFOs"}
        avail = mem_available_bytes()
        if avail is None or avail < 2 * 3 * peers * n * 4:  # initial, send and recv buckets of every peer
            return dict(out, error=f"not run: MemAvailable {avail} B is under twice the run's 24 GiB of buckets")
        out["builtin_inplace_ms"] = round(fmi_ref.time_allreduce(peers, n, 1, adapter=False), 1)
        if avail >= 2 * (3 + 6) * peers * n * 4:
            out["adapter_ms"] = round(fmi_ref.time_allreduce(peers, n, 1, adapter=True), 1)
        else:
            out["adapter_ms"] = f"not run: MemAvailable {avail} B is under twice the adapter run's ~72 GiB"
        return out
    except Exception as e:  # reported, never required
        return {"error": f"{type(e).__name__}: {e}"}


_JSON_OUT = None
_LINE_PRINTED = False  # the one JSON line is out (N > 1: by the emitter, on every rank's view)
_WATCH = None  # N > 1: the phase watch of this rank (names the phase an error line reports)
# N > 1: whose exchange the line measures, at top level of every N > 1 line: the product's
# communicator, or torch.distributed's after the communicator failed (run_dist_torch_exchange)
EXCHANGE_FMI = "fmi_comm"
EXCHANGE_TORCH = "torch_fallback"
_EXCHANGE = EXCHANGE_FMI


def json_out():
    """Where the one JSON line goes: the process's original stdout, claimed by claim_stdout()."""
    return _JSON_OUT or sys.stdout


def claim_stdout() -> None:
    """Keep the process's stdout for the one JSON line only: fd 1 is duplicated for the line, then pointed
    at stderr, so whatever libraries print to stdout (RCCL prints a version banner on communicator init)
    cannot add lines to the output the driver parses."""
    global _JSON_OUT
    if _JSON_OUT is not None:
        return
    sys.stdout.flush()
    _JSON_OUT = os.fdopen(os.dup(1), "w", buffering=1)
    os.dup2(2, 1)


class _Emitter:
    """Prints the one JSON line exactly once (rank 0), from the main thread or from the deadline —
    whichever comes first."""

    def __init__(self, line, rank):
        self.line, self.rank = line, rank
        self.lock = threading.Lock()
        self.done = False

    def emit(self):
        global _LINE_PRINTED
        with self.lock:
            if self.done:
                return
            self.done = True
            _LINE_PRINTED = True
            if self.rank == 0:
                try:
                    text = json.dumps(self.line)
                except RuntimeError:  # the main thread was still writing the after-`value` section
                    self.line = {k: v for k, v in self.line.items() if k in _HEADLINE_KEYS}
                    self.line["incomplete"] = "deadline reached while recording the after-value section"
                    text = json.dumps(self.line)
                print(text, file=json_out(), flush=True)

    def deadline(self, state):
        msg = "deadline reached; the timed measurement (value, roofline, self_check) is unaffected"
        state["incomplete"] = msg
        self.line["incomplete"] = msg
        self.emit()
        print("bench: deadline reached, exiting", file=sys.stderr, flush=True)
        os._exit(0)


_HEADLINE_KEYS = ("metric", "value", "unit", "n_gpus", "workload", "steps", "warmup", "ms_per_step",
                  "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "xgmi_roofline",
                  "self_check", "cpu_baseline")

# What `value` measures, at top level of every line: the metric's 1/2/4/8-GPU curve spans two workloads. N = 1
# is the HBM-bound pairwise combine (config C2); N > 1 the xGMI-bound sharded allreduce of one bucket per GPU
# (config C4's shape at the metric's bucket size). The driver's N-over-1 ratio therefore compares two different
# workloads; each N > 1 line carries its own one-GPU anchor (`local_equivalent`, `allreduce_1peer` at N = 1).
WORKLOAD_N1 = "local_combine"
WORKLOAD_DIST = "sharded_allreduce"


def _error_line(world, error, phase, **extra):
    """The one line of a failed N > 1 run: what failed, where, and the runtime it failed on (librccl version and
    path, device visibility), so a first 8-GPU failure is diagnosable from the line alone."""
    comm_mod = sys.modules.get("fmi_amd.comm")  # never import from here: this may run on the deadline's thread
    if comm_mod is None:
        runtime = {k: os.environ.get(k) for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES",
                                                  "GPU_MAX_HW_QUEUES")}
        runtime["rccl_error"] = "the library was not loaded yet when the run failed"
    else:
        try:
            runtime = comm_mod.runtime_info()
        except Exception as e:  # the library itself may be what failed
            runtime = {"error": f"{type(e).__name__}: {e}"}
    line = {"metric": METRIC, "value": None, "unit": "GiB/s", "n_gpus": world, "workload": WORKLOAD_DIST,
            "exchange": _EXCHANGE, "higher_is_better": True, "error": error, "phase": phase, "runtime": runtime}
    line.update(extra)
    return line


def placement() -> str:
    """How the line's device buckets are placed: fmi_dev_alloc's rotating 4 KiB slots, or plain."""
    try:
        import fmi_amd

        on = fmi_amd.tune_get(fmi_amd.Tune.ALLOC_SLOTS)
    except Exception as e:  # reported, never required
        return f"unknown ({type(e).__name__}: {e})"
    return ("fmi_dev_alloc: every bucket of >= 1 MiB in the next of 16 rotating 4 KiB slots (mod 64 KiB) of its own "
            "hipMalloc (FMI_TUNE_ALLOC_SLOTS = 1)" if on else
            "fmi_dev_alloc: plain hipMalloc, 2 MiB aligned (FMI_TUNE_ALLOC_SLOTS = 0, the default: the pair kernel's "
            "best placement, profiles/r06a_placement_ab.jsonl)")


def _headline(args, value, step_ms, workload, parallelism, n, roofline):
    return {
        "metric": METRIC,
        "value": round(value, 2),
        "workload": WORKLOAD_N1 if args.gpus == 1 and not args.force_dist else WORKLOAD_DIST,
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
        "config": {"workload": workload, "bucket_mib": args.bucket_mib, "elements": n, "parallelism": parallelism,
                   "rotating_sets": args.sets, "placement": placement()},
        "roofline": roofline,
    }


def c2_kernel_signature():
    """The pair_tile instantiation C2 launches under the current tuning (fmi_dev.hip: launch_combine →
    launch_pair_vec): the PMC summary is looked up by exactly this, never by a bare kernel name that other
    instantiations (C3's i64 max) share."""
    import fmi_amd
    from fmi_amd import Tune

    nt = {0: 0, 1: 0, 2: 3, 3: 1, 4: 2}[fmi_amd.tune_get(Tune.PAIR_VARIANT)]
    form = "pair_stride" if fmi_amd.tune_get(Tune.PAIR_VARIANT) == 1 else "pair_tile"
    return f"{form}<fmi::dev::OpSum, float, {fmi_amd.tune_get(Tune.PAIR_UNROLL)}, {nt}>"


def _roofline(kernel, algo_bytes, kernel_avg_ms, source, extra=None, pmc_key=None):
    """traffic: the committed PMC bytes of exactly this instantiation at exactly this launch shape
    (pmc_traffic); null when no profile of that launch is committed (e.g. a non-default --bucket-mib)."""
    achieved = algo_bytes / (kernel_avg_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(pmc_key or kernel, algo_bytes)
    if traffic is None:
        traffic_src = "not reported: no committed PMC profile of this instantiation at this launch shape"
    r = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": kernel,
         "kernel_avg_us": round(kernel_avg_ms * 1e3, 2), "algorithmic_bytes_per_launch": algo_bytes,
         "kernel_avg_source": source, "traffic_source": traffic_src}
    r.update(extra or {})
    return r


# ------------------------------------------------------------------------------------------------------
# N = 1: config C2
# ------------------------------------------------------------------------------------------------------
def run_single(args):
    claim_stdout()
    import numpy as np

    import fmi_amd
    from fmi_amd import Bucket, Event, Op

    fmi_amd.init(0)
    n = args.bucket_mib * MIB // 4
    nbytes = n * 4
    sets = [tuple(Bucket(n, np.float32).fill_synthetic(42 + s, j) for j in range(2)) for s in range(args.sets)]
    fmi_amd.sync()
    # self-check windows (head, middle, tail of every set's buckets), read before the first launch
    win = 4096
    offs = [0, (n // 2) // 64 * 64, n - win]
    before = [[(a.view(o, win).numpy(), b.view(o, win).numpy()) for o in offs] for a, b in sets]
    launches = [0] * len(sets)

    def step(k):  # k runs on from the warm-up, so every set is re-used exactly len(sets) steps later
        a, b = sets[k % len(sets)]
        fmi_amd.reduce_pair(Op.SUM, a, b)
        launches[k % len(sets)] += 1

    for k in range(args.warmup):
        step(k)
    fmi_amd.sync()
    # Timed region: exactly K back-to-back launches on the library stream; two HIP events on that stream
    # bracket them (no markers between launches).
    ev0, ev1 = Event(), Event()
    t0 = time.perf_counter()
    ev0.record()
    for k in range(args.warmup, args.warmup + args.steps):
        step(k)
    ev1.record()
    fmi_amd.sync()
    t1 = time.perf_counter()
    step_ms = (t1 - t0) * 1e3 / args.steps
    kernel_avg_ms = ev0.elapsed_ms(ev1) / args.steps  # includes the ~1-2 us dispatch gaps between launches
    # diagnostic, untimed: per-launch event pairs give the launch duration without the gaps
    probe = min(args.steps, 32)
    pairs = [(Event(), Event()) for _ in range(probe)]
    for k in range(probe):
        pairs[k][0].record()
        step(args.warmup + args.steps + k)
        pairs[k][1].record()
    fmi_amd.sync()
    isolated_us = 1e3 * sum(a.elapsed_ms(b) for a, b in pairs) / probe
    check = c2_self_check(sets, offs, win, before, launches)
    for a, b in sets:
        a.free()
        b.free()
    roof = _roofline("pair_tile", 3 * nbytes, kernel_avg_ms,
                     "HIP events bracketing the K timed launches on the library stream",
                     {"kernel_avg_us_isolated": round(isolated_us, 2)}, pmc_key=c2_kernel_signature())
    line = _headline(args, (nbytes / GIB) / (step_ms * 1e-3), step_ms,
                     "C2: 1-GPU pairwise float32 sum-reduce of two 256 MiB device-resident peer buckets",
                     "single GPU (2 peers resident)", n, roof)
    line["config"]["peers"] = 2
    line["self_check"] = check
    line["allreduce_1peer"] = one_peer_allreduce(n)
    if not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args)
    if not args.no_c3:
        try:
            line["c3"] = c3_single()
        except Exception as e:  # reported, never fails the measured line
            line["c3"] = f"failed: {type(e).__name__}: {e}"
    if not args.no_c4:
        try:
            line["c4_one_gpu"] = c4_single()
        except Exception as e:  # reported, never fails the measured line
            line["c4_one_gpu"] = f"failed: {type(e).__name__}: {e}"
    if not args.no_c5:
        line["c5"] = c5_single(args.c5_mib)
    print(json.dumps(line), file=json_out(), flush=True)
    failed = failed_checks(line)
    if failed:
        print("bench: self-check FAILED: " + ", ".join(failed), file=sys.stderr, flush=True)
        sys.exit(1)


def failed_checks(line) -> list:
    """Every in-run check of an N = 1 line that ran and did not pass (C2, the P = 1 allreduce, C3's two kernels,
    C5's three blocks): any of them makes the run exit 1, as the headline's own check does. A block that raised
    instead of producing a result is reported in the line (its "error"), not counted here."""
    failed = [] if line["self_check"]["ok"] else ["c2"]
    if not line.get("allreduce_1peer", {}).get("result_ok", True):
        failed.append("allreduce_1peer")
    c3 = line.get("c3")
    if isinstance(c3, dict):
        for k in ("i64_max_pair_64MiB", "f32_scan_P8_64MiB"):
            if not c3[k]["self_check"]["ok"]:
                failed.append(f"c3 {k}")
    c4 = line.get("c4_one_gpu")
    if isinstance(c4, dict) and not c4["self_check"]["ok"]:
        failed.append("c4_one_gpu")
    for k, block in (line.get("c5") or {}).items():
        if "error" not in block and not block["self_check"]["ok"]:
            failed.append(f"c5 {k}")
    return failed


def c2_self_check(sets, offs, win, before, launches) -> dict:
    """The timed C2 combines checked in the run: every set's a was combined in place with its b `launches[s]`
    times (warm-up, timed and probe launches), so on each window a must equal numpy's float32 a + b repeated
    that many times (IEEE round-to-nearest, the reference's std::plus<float>) — bit for bit."""
    import numpy as np

    bad = checked = 0
    for s, (a, b) in enumerate(sets):
        for o, (a0, b0) in zip(offs, before[s]):
            want = a0.copy()
            for _ in range(launches[s]):
                want = want + b0
            got = a.view(o, win).numpy()
            bad += int(np.count_nonzero(got.view(np.uint32) != want.view(np.uint32)))
            checked += win
    return {"ok": bad == 0, "mismatches": bad, "elements_checked": checked,
            "against": "numpy float32 a + b repeated once per launch of each set (warm-up, timed, probe), "
                       "on the head, middle and tail window of every set, bit-exact"}


def one_peer_allreduce(n: int, launches: int = 20, sets: int = 4) -> dict:
    """The N = 1 point of the N > 1 curve's own workload: fmi_comm_allreduce of one 256 MiB bucket on a
    one-rank communicator — the reference's P = 1 allreduce (PeerToPeer.cpp:96-130 with P = 1) is a copy
    of the bucket into recvbuf (2·S HBM bytes). Events around back-to-back calls on the library stream,
    rotating over `sets` (send, recv) pairs: the copy stores with sc1, so a recv bucket is rewritten only
    after (sets - 1) x 256 MiB of other writes have passed through the 256 MB MALL."""
    import numpy as np

    from fmi_amd import Bucket, Event, Op
    from fmi_amd.comm import Comm, Transport, unique_id

    comm = Comm(unique_id(Transport.LOCAL), 1, 0)
    pairs = [(Bucket(n, np.float32).fill_synthetic(11 + s, 0), Bucket(n, np.float32)) for s in range(sets)]
    try:
        for src, dst in pairs:
            comm.allreduce(Op.SUM, src, dst)
        quiet_device()  # C2 has just freed its 8 GiB of buckets (background VRAM clears share the HBM)
        e0, e1 = Event(), Event()
        e0.record()
        for k in range(launches):
            src, dst = pairs[k % sets]
            comm.allreduce(Op.SUM, src, dst)
        e1.record()
        e1.sync()
        ms = e0.elapsed_ms(e1) / launches
        e0.destroy()
        e1.destroy()
        ok = all(bool(np.array_equal(s.view(0, 4096).numpy().view(np.uint32), d.view(0, 4096).numpy().view(np.uint32)))
                 and bool(np.array_equal(s.view(n - 4096, 4096).numpy().view(np.uint32),
                                         d.view(n - 4096, 4096).numpy().view(np.uint32)))
                 for s, d in pairs)
    finally:
        for src, dst in pairs:
            src.free()
            dst.free()
        comm.destroy()
    S = n * 4
    return {"workload": f"fmi_comm_allreduce, 1 rank, {S >> 20} MiB f32 (the reference's P = 1 allreduce: a copy)",
            "ms": round(ms, 4), "GiB_s_reduced_buckets": round(S / GIB / (ms * 1e-3), 2),
            "hbm_frac": round(2 * S / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "result_ok": ok, "launches": launches,
            "rotating_sets": sets}


C3_PAIR_SETS = 64  # 63 x 8 MiB of sc1 tile writes between two uses of a set (see --sets)
# The scan's rate depends on where its 16 buckets land in HBM (0.70-0.80 by allocation draw, the
# write side bimodal); 8 sets of 16 separately allocated buckets (8 GiB) average over 8 draws instead of
# letting two decide the line.
C3_SCAN_SETS = 8


GROUP_PLACEMENT = ("fmi_dev_alloc_group: the launch's buckets as one group, bucket j in 4 KiB slot j mod 16 "
                   "(mod 64 KiB) of its own hipMalloc")


def scan_sets(sets: int, peers: int, n: int):
    """The C3 scan's buckets: each set's `peers` inputs and `peers` outputs allocated as ONE group
    (fmi_dev_alloc_group), so the 16 streams of one launch sit in 16 distinct 4 KiB slots whatever was allocated
    before (tests/test_bench_contract.py checks the order, tests/test_gpu_parity.py the slots)."""
    import numpy as np

    from fmi_amd import Bucket

    groups = [Bucket.group(2 * peers, n, np.float32) for _ in range(sets)]
    return [g[:peers] for g in groups], [g[peers:] for g in groups]


def c3_single(reps: int = 60) -> dict:
    """Config C3 on this GPU, in the driver's run: the int64 max pairwise combine of 64 MiB buckets (64
    rotating sets, 8 GiB: no set is re-read from the 256 MiB MALL) and the f32 peer-axis scan (scan_no_order)
    of 8 peers x 64 MiB (C3_SCAN_SETS rotating sets, 3 passes over them); mean launch time from two HIP events
    around back-to-back launches on the library stream, against the algorithmic bytes (3 x 64 MiB and
    2 x 8 x 64 MiB)."""
    import numpy as np

    import fmi_amd
    from fmi_amd import Alg, Bucket, Event, Op

    def timed(launch, k):  # the set index runs on from the warm-up: every set is re-used `sets` launches later
        for i in range(3):
            launch(i)
        e0, e1 = Event(), Event()
        e0.record()
        for i in range(3, 3 + k):
            launch(i)
        e1.record()
        e1.sync()
        ms = e0.elapsed_ms(e1) / k
        e0.destroy()
        e1.destroy()
        return ms

    n64 = 64 * MIB // 8
    pairs = [(Bucket(n64, np.int64).fill_synthetic(42 + s, 0), Bucket(n64, np.int64).fill_synthetic(42 + s, 1))
             for s in range(C3_PAIR_SETS)]
    win = 4096
    offs = [0, (n64 // 2) // 64 * 64, n64 - win]
    before = [[(a.view(o, win).numpy(), b.view(o, win).numpy()) for o in offs] for a, b in pairs]
    used = [0] * C3_PAIR_SETS

    def launch_max(i):
        used[i % C3_PAIR_SETS] += 1
        fmi_amd.reduce_pair(Op.MAX, *pairs[i % C3_PAIR_SETS])

    quiet_device()  # the buckets of the blocks before were just freed (background VRAM clears share the HBM)
    ms_max = timed(launch_max, reps)
    # in-run check: max is idempotent, so a pair combined at least once holds max(a0, b0) (std::max on int64)
    # and one never combined still holds a0 — on the head, middle and tail window of every pair, bit for bit
    bad = sum(int(np.count_nonzero(a.view(o, win).numpy() != (np.maximum(a0, b0) if k else a0)))
              for (a, b), wins, k in zip(pairs, before, used) for o, (a0, b0) in zip(offs, wins))
    max_check = {"ok": bad == 0, "mismatches": bad, "elements_checked": len(pairs) * len(offs) * win,
                 "against": "numpy maximum of the pair's initial windows (int64, idempotent), bit-exact"}
    for a, b in pairs:
        a.free()
        b.free()
    P, n32 = 8, 64 * MIB // 4
    S = C3_SCAN_SETS
    ins, outs = scan_sets(S, P, n32)
    for s in range(S):
        for p in range(P):
            ins[s][p].fill_synthetic(7 + s, p)
    quiet_device()  # the 8 GiB of i64 pairs were just freed
    ms_scan = timed(lambda i: fmi_amd.scan_peers(Op.SUM, Alg.SCAN, outs[i % S], ins[i % S]), 3 * S)
    per_set = [(Event(), Event()) for _ in range(S)]  # diagnostic, untimed: one launch per set, its own events
    fmi_amd.scan_peers(Op.SUM, Alg.SCAN, outs[S - 1], ins[S - 1])  # after the host wait: the first launch ramps
    for i, (a, b) in enumerate(per_set):
        a.record()
        fmi_amd.scan_peers(Op.SUM, Alg.SCAN, outs[i], ins[i])
        b.record()
    fmi_amd.sync()
    per_set_us = [round(a.elapsed_ms(b) * 1e3, 1) for a, b in per_set]
    for a, b in per_set:
        a.destroy()
        b.destroy()
    scan_check = scan_self_check(ins, outs, n32)
    for b in [x for s in ins + outs for x in s]:
        b.free()

    def row(ms, algo, key):
        traffic, src = pmc_traffic(key, algo)  # the committed PMC profile of exactly this launch
        return {"kernel_avg_us": round(ms * 1e3, 2), "algorithmic_bytes": algo,
                "GB_s": round(algo / (ms * 1e-3) / 1e9, 1), "frac": round(algo / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "traffic": traffic, "traffic_source": src}

    return {"i64_max_pair_64MiB": dict(row(ms_max, 3 * 64 * MIB, "pair_tile<fmi::dev::OpMax, long, 4, 3>"),
                                       rotating_sets=C3_PAIR_SETS, self_check=max_check),
            "f32_scan_P8_64MiB": dict(row(ms_scan, 2 * P * 64 * MIB, "scan_kernel<fmi::dev::OpSum, float, 3, 8>"),
                                      rotating_sets=C3_SCAN_SETS, per_set_launch_us=per_set_us,
                                      placement=GROUP_PLACEMENT,
                                      self_check=scan_check),
            "timing": "two HIP events around back-to-back launches on the library stream (gaps included)"}


C4_SETS = 3  # like C3's scan sets: the rate depends on where a set's 9 GiB lands, so average over draws


def c4_single(peers: int = 8, mib: int = 1024, launches: int = 15, sets: int = C4_SETS) -> dict:
    """Config C4's data on ONE GPU: 8 peers x 1 GiB f32 buckets resident in HBM, their sum-allreduce computed by
    one pass of the fused 8-way kernel (fmi_dev_reduce_tree, allreduce_no_order: the reference's recursive-doubling
    bracketing, PeerToPeer.cpp:96-130). The kernel the N > 1 path runs on every shard, at the whole bucket:
    (P + 1) x 1 GiB algorithmic bytes per launch (9 GiB, far past the 256 MB MALL). Each of `sets` buffer sets is one
    carved group; the timed launches rotate over them, so one set's placement cannot decide the line
    (round 6: one of 13 single-set lines read 0.761 against 0.827-0.847). Mean launch time from two HIP events
    around back-to-back launches on the library stream, plus one isolated launch per set (`per_set_launch_us`);
    every set's result is checked on head / middle / tail windows against numpy's float32 evaluation of rank 0's
    bracketing."""
    import numpy as np

    import fmi_amd
    from fmi_amd import Alg, Bucket, Event, Op

    n = mib * MIB // 4
    groups = [Bucket.group(peers + 1, n, np.float32) for _ in range(sets)]  # inputs + output in distinct slots
    for g in groups:
        for p in range(peers):
            g[p].fill_synthetic(11, p)
    # The driver clears the VRAM C3 just freed (9 GiB) in the background, on the same HBM: measured right after
    # C3 this launch ran at 0.68 of peak, after a quiet second at 0.76-0.78 (profiles/r04_tree8_sizes.jsonl).
    quiet_device()

    def launch(k):
        g = groups[k % sets]
        fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, g[peers], g[:peers])

    for k in range(sets):
        launch(k)
    e0, e1 = Event(), Event()
    e0.record()
    for k in range(launches):
        launch(k)
    e1.record()
    e1.sync()
    ms = e0.elapsed_ms(e1) / launches
    e0.destroy()
    e1.destroy()
    per_set = [(Event(), Event()) for _ in range(sets)]  # diagnostic, untimed: one launch per set, its own events
    for k, (a, b) in enumerate(per_set):
        a.record()
        launch(k)
        b.record()
    fmi_amd.sync()
    per_set_us = [round(a.elapsed_ms(b) * 1e3, 1) for a, b in per_set]
    for a, b in per_set:
        a.destroy()
        b.destroy()
    expr = fmi_amd.schedule_expr(Alg.ALLREDUCE, peers, 0)
    win, bad, checked = 4096, 0, 0
    for g in groups:
        for o in (0, (n // 2) // 64 * 64, n - win):
            want = eval_bracketing(expr, [b.view(o, win).numpy() for b in g[:peers]])
            bad += int(np.count_nonzero(g[peers].view(o, win).numpy().view(np.uint32) != want.view(np.uint32)))
            checked += win
    for b in [x for g in groups for x in g]:
        b.free()
    algo = (peers + 1) * n * 4
    traffic, src = pmc_traffic(f"tree_kernel<fmi::dev::OpSum, float, 0, {peers}, false>", algo)
    return {"workload": f"C4 on one GPU: {peers} peers x {mib} MiB f32 sum-allreduce, one pass of the fused "
                        f"{peers}-way kernel (allreduce_no_order bracketing)",
            "kernel_avg_us": round(ms * 1e3, 2), "algorithmic_bytes": algo,
            "GB_s": round(algo / (ms * 1e-3) / 1e9, 1), "frac": round(algo / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "GiB_s_reduced_buckets": round(peers * n * 4 / GIB / (ms * 1e-3), 2),
            "traffic": traffic, "traffic_source": src, "launches": launches, "rotating_sets": sets,
            "per_set_launch_us": per_set_us, "placement": GROUP_PLACEMENT,
            "timing": "two HIP events around back-to-back launches on the library stream (gaps included)",
            "self_check": {"ok": bad == 0, "mismatches": bad, "elements_checked": checked,
                           "against": "numpy float32 evaluation of rank 0's allreduce_no_order bracketing "
                                      "(fmi_schedule_expr) on three windows of every set, bit-exact"}}


def eval_bracketing(expr: str, xs):
    """Evaluates a bracketing such as "((x1+x0)+x2)" on numpy float32 windows: x<p> = xs[p], (a+b) = a + b
    with a the left operand (IEEE round-to-nearest, the reference's std::plus<float>)."""
    pos = 0

    def term():
        nonlocal pos
        if expr[pos] == "(":
            pos += 1
            left = term()
            assert expr[pos] == "+"
            pos += 1
            right = term()
            assert expr[pos] == ")"
            pos += 1
            return left + right
        end = pos + 1
        while end < len(expr) and expr[end].isdigit():
            end += 1
        peer = int(expr[pos + 1:end])
        pos = end
        return xs[peer]

    return term()


def scan_self_check(ins, outs, n: int, win: int = 4096) -> dict:
    """C3's scan checked in the run: on the head, middle and tail window of every set, each peer's output must
    equal numpy's float32 evaluation of that peer's scan_no_order bracketing (fmi_schedule_expr, the program
    the kernel runs, pinned to the reference's own bracketing by tests/test_ref_pinning.py), bit for bit."""
    import numpy as np

    import fmi_amd
    from fmi_amd import Alg

    P = len(ins[0])
    exprs = [fmi_amd.schedule_expr(Alg.SCAN, P, r) for r in range(P)]
    bad = checked = 0
    for set_in, set_out in zip(ins, outs):
        for o in (0, (n // 2) // 64 * 64, n - win):
            xs = [b.view(o, win).numpy() for b in set_in]
            for r in range(P):
                want = eval_bracketing(exprs[r], xs)
                bad += int(np.count_nonzero(set_out[r].view(o, win).numpy().view(np.uint32) != want.view(np.uint32)))
                checked += win
    return {"ok": bad == 0, "mismatches": bad, "elements_checked": checked,
            "against": "numpy float32 evaluation of each peer's scan_no_order bracketing on three windows per set, "
                       "bit-exact"}


QUIET_S = 1.0


def quiet_device():
    """Let the device go idle before a measurement that follows freed buckets. The driver clears freed VRAM
    asynchronously on the copy engines: right after the C3 / C4 loops free their buckets (GiBs), the H2D
    and D2H copies of C5 share those engines for ~0.3 s and C5 reads 39 ms instead of 23.5 ms
    (profiles/archive/r02_c5_after_free_probe.jsonl: the same buffers, 23.4 ms once 0.3 s have passed). A pause of QUIET_S
    seconds, outside every timed region."""
    import fmi_amd

    fmi_amd.sync()
    time.sleep(QUIET_S)


def c5_single(mib: int, peers: int = 8) -> dict:
    """Config C5 at N = 1, three blocks, each self-checked:
      p1_copy          the `mib` page-locked host bucket through fmi_comm_allreduce_host on a one-rank
                       communicator: the reference's P = 1 allreduce, a copy (H2D + D2H pipelined).
      host_pair_reduce the combine at the reference's site on host buckets: a `mib` page-locked pair through
                       fmi_host_reduce_pair (the zero-copy kernel over PCIe), a += b.
      local_peers      C5's whole workload on this one GPU: `peers` LOCAL ranks (threads), each with a `mib`
                       page-locked f32 bucket, fmi_comm_allreduce_host (H2D, sharded allreduce in the reference's
                       order, D2H pipelined in 64 MiB chunks) — every byte of the 8-GPU config through one PCIe
                       link and one GPU, sized down only if the host's MemAvailable cannot hold it."""
    out = {}
    for name, fn in (("p1_copy", lambda: c5_p1_copy(mib)), ("host_pair_reduce", lambda: c5_host_pair(mib)),
                     ("local_peers", lambda: c5_local_peers(peers, mib))):
        try:
            quiet_device()
            out[name] = dict(fn(), after_pause_s=QUIET_S)
        except Exception as e:  # reported, never fails the measured line
            out[name] = {"error": f"{type(e).__name__}: {e}"}
    return out


def c5_p1_copy(mib: int, iters: int = 3) -> dict:
    """fmi_comm_allreduce_host of a `mib` page-locked bucket on a one-rank communicator: a copy (reference
    PeerToPeer.cpp:96-130 with P = 1). Median wall time of `iters` after one warm-up; bit-exact copy check."""
    import statistics

    import numpy as np

    from fmi_amd import Op, PinnedArray
    from fmi_amd.comm import Comm, Transport, unique_id

    n = mib * MIB // 4
    comm = Comm(unique_id(Transport.LOCAL), 1, 0)
    send, recv = PinnedArray(n, np.float32), PinnedArray(n, np.float32)
    try:
        send.array[:] = np.random.default_rng(5).random(n, dtype=np.float32)
        times = []
        for k in range(iters + 1):
            recv.array[:1] = np.float32(-1.0)
            t0 = time.perf_counter()
            comm.allreduce_host(Op.SUM, send.array, recv.array, chunk=64 * MIB // 4)
            if k:
                times.append(time.perf_counter() - t0)
        ok = bool(np.array_equal(send.array.view(np.uint32), recv.array.view(np.uint32)))
    finally:
        send.free()
        recv.free()
        comm.destroy()
    ms = statistics.median(times) * 1e3
    return {"workload": f"{mib} MiB f32 page-locked host bucket, one-rank allreduce (P = 1: a copy), H2D + D2H, "
                        "64 MiB chunks",
            "ms": round(ms, 3), "host_bucket_GiB_s": round(n * 4 / GIB / (ms * 1e-3), 2),
            "pcie_GB_s_both_directions": round(2 * n * 4 / (ms * 1e-3) / 1e9, 1), "iters": iters,
            "self_check": {"ok": ok, "against": "the send bucket, whole, bit-exact"}}


def _pinned_synthetic(n: int, seed: int, peers):
    """Page-locked f32 host buckets filled with the synthetic generator on the device (fast) and copied down."""
    import numpy as np

    import fmi_amd
    from fmi_amd import Bucket, PinnedArray, _lib

    scratch = Bucket(n, np.float32)
    out = []
    try:
        for p in peers:
            h = PinnedArray(n, np.float32)
            out.append(h)
            scratch.fill_synthetic(seed, p)
            _lib.call("fmi_dev_d2h_async", h.ptr, scratch.ptr, n * 4, None)
            fmi_amd.sync()
    except BaseException:
        for h in out:
            h.free()
        raise
    finally:
        scratch.free()
    return out


def _windows(n: int, win: int = 4096):
    return [0, (n // 2) // 64 * 64, n - win], win


def c5_host_pair(mib: int, iters: int = 3) -> dict:
    """fmi_host_reduce_pair on a `mib` page-locked f32 pair (a channel recv buffer and the peer's bucket): the
    reference's f.f(a, b) (PeerToPeer.cpp:119) with both host buckets streamed through the kernel over PCIe
    (zero-copy: 2 reads + 1 write of the bucket per combine). Median of `iters` after one warm-up; then a must
    equal numpy's float32 a + b repeated once per call, bit for bit, on three windows."""
    import statistics

    import numpy as np

    import fmi_amd
    from fmi_amd import Op

    n = mib * MIB // 4
    a, b = _pinned_synthetic(n, 61, (0, 1))
    try:
        offs, win = _windows(n)
        before = [(a.array[o:o + win].copy(), b.array[o:o + win].copy()) for o in offs]
        times = []
        for k in range(iters + 1):
            t0 = time.perf_counter()
            fmi_amd.host_reduce_pair(Op.SUM, a.array, b.array)
            if k:
                times.append(time.perf_counter() - t0)
        bad = 0
        for o, (a0, b0) in zip(offs, before):
            want = a0
            for _ in range(iters + 1):
                want = want + b0
            bad += int(np.count_nonzero(a.array[o:o + win].view(np.uint32) != want.view(np.uint32)))
    finally:
        a.free()
        b.free()
    ms = statistics.median(times) * 1e3
    S = n * 4
    return {"workload": f"{mib} MiB f32 page-locked host pair, a += b through fmi_host_reduce_pair (zero-copy "
                        "kernel over PCIe)",
            "ms": round(ms, 3), "host_bucket_GiB_s": round(S / GIB / (ms * 1e-3), 2),
            "pcie_GB_s": round(3 * S / (ms * 1e-3) / 1e9, 1), "pcie_bytes_per_combine": 3 * S, "iters": iters,
            "self_check": {"ok": bad == 0, "mismatches": bad, "elements_checked": len(offs) * win,
                           "against": "numpy float32 a + b repeated once per call, three windows, bit-exact"}}


def mem_available_bytes():
    try:
        for line in open("/proc/meminfo"):
            if line.startswith("MemAvailable:"):
                return int(line.split()[1]) * 1024
    except OSError:
        pass
    return None


C5_HEADROOM = 16 * GIB  # host memory left free beside C5's page-locked buckets
_LEAKED = []  # host buckets a stuck rank may still use: never freed in this process


def c5_size_mib(peers: int, mib: int, avail) -> int:
    """The bucket size C5's local_peers block runs at: `mib`, halved until 2 x peers page-locked buckets plus
    C5_HEADROOM fit in MemAvailable (unknown MemAvailable: `mib`)."""
    size = mib
    while avail is not None and size > 1 and 2 * peers * size * MIB + C5_HEADROOM > avail:
        size //= 2
    return size


def c5_local_peers(peers: int, mib: int, iters: int = 2, chunk_mib: int = 64) -> dict:
    """C5's workload on ONE GPU: `peers` LOCAL ranks (threads of this process), each with a page-locked f32
    bucket of `mib` (1 GiB: 8 GiB in, 8 GiB out over this GPU's one PCIe link), fmi_comm_allreduce_host with
    64 MiB chunks. Per iteration every rank starts at a barrier; the iteration's time is the slowest rank's;
    median of `iters` after one warm-up. Self-check: every rank's result on three windows equals numpy's
    float32 evaluation of that rank's allreduce_no_order bracketing (PeerToPeer.cpp:96-130) over the peers'
    windows, bit-exact."""
    import statistics
    import threading

    import numpy as np

    import fmi_amd
    from fmi_amd import Alg, Op, PinnedArray
    from fmi_amd.comm import Comm, Transport, unique_id

    avail = mem_available_bytes()
    size = c5_size_mib(peers, mib, avail)
    n = size * MIB // 4
    send = _pinned_synthetic(n, 91, range(peers))
    recv = []
    stuck = False
    try:
        recv = [PinnedArray(n, np.float32) for _ in range(peers)]
        uid = unique_id(Transport.LOCAL)
        bar = threading.Barrier(peers)
        times = [[0.0] * (iters + 1) for _ in range(peers)]
        errors = []

        def rank(r):
            try:
                c = Comm(uid, peers, r, timeout_s=120)
                try:
                    for k in range(iters + 1):
                        bar.wait(timeout=300)
                        t0 = time.perf_counter()
                        c.allreduce_host(Op.SUM, send[r].array, recv[r].array, chunk=chunk_mib * MIB // 4)
                        times[r][k] = time.perf_counter() - t0
                finally:
                    c.destroy()
            except BaseException as e:  # noqa: BLE001 - reported below
                bar.abort()
                errors.append(f"rank {r}: {type(e).__name__}: {e}")

        threads = [threading.Thread(target=rank, args=(r,), daemon=True) for r in range(peers)]
        for t in threads:
            t.start()
        for t in threads:
            t.join(timeout=600)
        if any(t.is_alive() for t in threads):  # a rank still inside the library: its buckets must outlive it
            stuck = True
            raise RuntimeError("C5 local_peers: a rank did not finish within 600 s (buckets leaked, not freed)")
        if errors:
            raise RuntimeError(errors[0])
        per_iter = [max(times[r][k] for r in range(peers)) for k in range(1, iters + 1)]
        offs, win = _windows(n)
        bad = 0
        for o in offs:
            xs = [s.array[o:o + win] for s in send]
            for r in range(peers):
                want = eval_bracketing(fmi_amd.schedule_expr(Alg.ALLREDUCE, peers, r), xs)
                bad += int(np.count_nonzero(recv[r].array[o:o + win].view(np.uint32) != want.view(np.uint32)))
    finally:
        if stuck:
            _LEAKED.extend(send + recv)  # kept referenced: PinnedArray frees itself when collected
        else:
            for h in send + recv:
                h.free()
    ms = statistics.median(per_iter) * 1e3
    S = n * 4
    return {"workload": f"C5 on one GPU: {peers} LOCAL ranks x {size} MiB f32 page-locked host buckets, "
                        f"fmi_comm_allreduce_host (H2D + sharded allreduce + D2H pipelined, {chunk_mib} MiB chunks)",
            "peers": peers, "chunk_mib": chunk_mib, "bucket_mib": size, "requested_bucket_mib": mib,
            "mem_available_gib": round(avail / GIB, 1) if avail else None,
            "ms": round(ms, 2), "host_buckets_GiB_s": round(peers * S / GIB / (ms * 1e-3), 2),
            "pcie_GB_s_both_directions": round(2 * peers * S / (ms * 1e-3) / 1e9, 1), "iters": iters,
            "ceiling": ("the copies alone, issued the same way (8 x 1 GiB each way on the device's one H2D + one D2H "
                        "stream, no compute): 177.97 ms = 96.5 GB/s, profiles/r05_pcie_peers.jsonl "
                        "(tools/microbench_pcie_peers.hip); DESIGN.md section 8"),
            "self_check": {"ok": bad == 0, "mismatches": bad, "elements_checked": len(offs) * win * peers,
                           "against": "numpy float32 evaluation of each rank's allreduce_no_order bracketing "
                                      "(fmi_schedule_expr) over the peers' windows, three windows, bit-exact"}}


# ------------------------------------------------------------------------------------------------------
# N > 1: the sharded allreduce, one peer per GPU
# ------------------------------------------------------------------------------------------------------
def bind_near_gpu(dev: int) -> dict:
    """Pin this rank to the CPUs of its GPU's NUMA node (from the PCI address torch reports) before any
    host buffer is allocated: page-locked C5 buckets then sit on the GPU's socket, and RCCL's proxy threads
    run there. A no-op on one-node hosts or when the node is unknown."""
    import glob

    import torch

    try:
        pr = torch.cuda.get_device_properties(dev)
        bdf = "%04x:%02x:%02x.0" % (pr.pci_domain_id, pr.pci_bus_id, pr.pci_device_id)
        node = int(open(f"/sys/bus/pci/devices/{bdf}/numa_node").read())
        nodes = glob.glob("/sys/devices/system/node/node[0-9]*")
        if node < 0 or len(nodes) < 2:
            return {"numa_node": node, "bound": False}
        cpus = set()
        for part in open(f"/sys/devices/system/node/node{node}/cpulist").read().strip().split(","):
            lo, _, hi = part.partition("-")
            cpus.update(range(int(lo), int(hi or lo) + 1))
        allowed = cpus & os.sched_getaffinity(0)
        if len(allowed) < 2:
            return {"numa_node": node, "bound": False}
        os.sched_setaffinity(0, allowed)
        return {"numa_node": node, "bound": True, "cpus": len(allowed)}
    except (OSError, ValueError, AttributeError, RuntimeError) as e:
        return {"bound": False, "error": f"{type(e).__name__}: {e}"}


class _PhaseWatch:
    """N > 1: which phase of the measurement this rank is in; if the measurement outlives its deadline (a rank
    waiting forever in an exchange), say where on stderr and exit non-zero instead of hanging silently."""

    def __init__(self, seconds, rank):
        self.rank, self.phase, self.t0 = rank, "start", time.time()
        self.timer = threading.Timer(seconds, self._expire)
        self.timer.daemon = True
        self.timer.start()

    def enter(self, phase):
        self.phase = phase
        # test hook (tests/test_gpu_bench_dist.py): every rank fails in the named phase, as a real failure would
        if os.environ.get("FMI_BENCH_TEST_RAISE_IN") and phase.startswith(os.environ["FMI_BENCH_TEST_RAISE_IN"]):
            raise RuntimeError(f"injected failure in phase '{phase}' (FMI_BENCH_TEST_RAISE_IN)")

    def _expire(self):
        print(f"bench: rank {self.rank} still in phase '{self.phase}' after {time.time() - self.t0:.0f} s "
              f"(--measure-deadline); exiting", file=sys.stderr, flush=True)
        if self.rank == 0 and not _LINE_PRINTED:  # the one line says where the run hung
            world = int(os.environ.get("WORLD_SIZE", "1"))
            print(json.dumps(_error_line(world, "measure deadline reached", self.phase,
                                         seconds=round(time.time() - self.t0))), file=json_out(), flush=True)
        os._exit(3)

    def done(self):
        self.timer.cancel()


def run_dist(args, world, rank, local_rank):
    claim_stdout()
    # torch first: libfmi_dev.so then binds to the HIP runtime torch already loaded (one runtime per process,
    # shared streams/pointers with RCCL) — see DESIGN.md §Runtime.
    import torch
    import torch.distributed as dist

    global _WATCH
    watch = _WATCH = _PhaseWatch(args.measure_deadline, rank)

    proc = args.transport == "proc"
    # every wait of the communicator for its peers (RCCL init included) gives up after this: a broken first
    # init then leaves time for the exchange fallback within --measure-deadline
    if not proc:  # (PROC runs keep their FMI_PROC_TIMEOUT_S)
        os.environ.setdefault("FMI_COMM_TIMEOUT_S", "120")
    dev = local_rank % max(1, torch.cuda.device_count()) if proc else local_rank
    numa = bind_near_gpu(dev) if not args.no_numa_bind else {"bound": False, "disabled": True}
    torch.cuda.set_device(dev)
    watch.enter("process group init")
    if proc:
        dist.init_process_group("gloo")
        vote = None
    else:
        dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        # the fallback agreement votes on a gloo group of its own: a vote can never pair with an RCCL collective
        # of the timed loop that another rank is still inside. If gloo cannot connect on ANY rank, every
        # rank votes on the RCCL group instead: the ranks agree on that here, over the world group, before anything
        # else runs on it (ranks voting on different groups would hang).
        try:
            import datetime

            vote = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=120))
        except Exception as e:  # noqa: BLE001 - the vote still happens, on the world group
            print(f"bench: rank {rank}: no gloo group for the fallback vote ({type(e).__name__}: {e})",
                  file=sys.stderr, flush=True)
            vote = None
        have = torch.tensor([0 if vote is None else 1], dtype=torch.int32, device=torch.device("cuda", dev))
        dist.all_reduce(have, op=dist.ReduceOp.MIN)
        if int(have.item()) == 0:
            if vote is not None:
                print(f"bench: rank {rank}: another rank has no gloo group: every rank votes over the RCCL group",
                      file=sys.stderr, flush=True)
            vote = None

    import fmi_amd
    from fmi_amd.collectives import CommAllreduce

    fmi_amd.init(dev)
    one_rank_exchange = args.force_dist and world == 1
    if one_rank_exchange:  # the plumbing check runs the real exchange (RCCL calls with itself), not the P = 1 copy
        fmi_amd.tune_set(fmi_amd.Tune.COMM_ONE_RANK_EXCHANGE, 1)
    if proc:  # gloo cannot carry the device exchange: no fallback, a failure is the error line
        watch.enter("fmi_comm init (communicator id broadcast, PROC init)")
        ar = CommAllreduce(dist.group.WORLD, path=args.path, transport=args.transport)
    else:
        ar, comm_err = None, None
        try:
            watch.enter("fmi_comm init (communicator id broadcast, RCCL init)")  # (its test hook raises here)
            ar = CommAllreduce(dist.group.WORLD, path=args.path, transport=args.transport)
        except Exception as e:  # every rank reaches the agreement below, whether its own init raised or not
            comm_err = f"{type(e).__name__}: {e}"
            print(f"bench: rank {rank}: fmi_comm init failed: {comm_err}", file=sys.stderr, flush=True)
        if _fall_back(args, world, rank, watch, dev, numa, ar, comm_err, "fmi_comm init", group=vote):
            return
    watch.enter("topology check")
    topo = ar.topology()
    if not topo["ok"]:  # RCCL did not see `world` ranks, or two ranks share a GPU: the line would be wrong
        print("bench: topology check FAILED: " + json.dumps(topo), file=sys.stderr, flush=True)
        if rank == 0:
            print(json.dumps(_error_line(world, "topology check failed", "topology check", topology=topo)),
                  file=json_out(), flush=True)
        os._exit(1)
    n = args.bucket_mib * MIB // 4
    S = n * 4
    if proc:
        watch.enter("warm-up and timed allreduces")
        step_ms, _, extra = ar.bench(n, steps=args.steps, warmup=args.warmup, sets=args.dist_sets, peers_per_gpu=1)
    else:  # a communicator that fails in its first real exchanges (a timeout aborts it on every rank) falls back too
        run_err = None
        try:
            watch.enter("warm-up and timed allreduces")  # (its test hook raises here)
            step_ms, _, extra = ar.bench(n, steps=args.steps, warmup=args.warmup, sets=args.dist_sets, peers_per_gpu=1)
        except Exception as e:  # every rank reaches the agreement below
            run_err = f"fmi_comm allreduce failed: {type(e).__name__}: {e}"
            print(f"bench: rank {rank}: {run_err}", file=sys.stderr, flush=True)
        if _fall_back(args, world, rank, watch, dev, numa, ar, run_err, "the fmi_comm allreduce", group=vote):
            return
    out, seed = extra.pop("result")
    value = world * (S / GIB) / (step_ms * 1e-3)
    watch.enter("self-check")
    check = ar.self_check(out, n, seed, tolerance=args.path == "rccl")
    out.free()
    watch.enter("isolated shard-kernel timing")
    kern = ar.shard_kernel(n, launches=max(10, min(args.steps, 50)))
    watch.done()
    live = extra.pop("shard_kernel_launches") > 0
    shard_ms = extra.pop("shard_kernel_avg_ms")
    roof = _roofline("tree_kernel", kern["algorithmic_bytes_per_launch"],
                     shard_ms if live else kern["kernel_avg_us"] * 1e-3,
                     ("HIP events recorded by fmi_comm around every shard-kernel launch of the K timed allreduces, "
                      "on the stream it runs on, mean per launch, max over ranks") if live else
                     ("HIP events around back-to-back launches of the shard kernel on the library stream after the "
                      "timed region (N = 1: the allreduce launches no kernel)"),
                     {"launch_shape": kern["kernel"], "kernel_avg_us_isolated": kern["kernel_avg_us"],
                      "note": "the allreduce step is xGMI-bound (xgmi_roofline); this is its HBM-bound kernel"},
                     pmc_key=f"tree_kernel<fmi::dev::OpSum, float, 0, {world}, false>")
    path_desc = {"tree": "all-to-all + fused tree kernel + all-gather (bit-exact)",
                 "rccl": "RCCL reduce-scatter + all-gather", "direct": "fused tree over IPC-mapped peer windows"}
    line = _headline(args, value, step_ms,
                     f"C4-shaped at the metric's bucket size: {world}-peer float32 sum-allreduce, one FMI peer "
                     f"(a {args.bucket_mib} MiB device-resident bucket) per GPU, through fmi_comm_allreduce",
                     f"{world} GPUs, one peer per GPU, buckets sharded {world} ways; path {args.path}: "
                     f"{path_desc[args.path]}; transport {args.transport}", n, roof)
    line["exchange"] = EXCHANGE_FMI
    line["config"]["topology"] = topo
    if one_rank_exchange:
        line["config"]["one_rank_exchange"] = ("FMI_TUNE_COMM_ONE_RANK_EXCHANGE = 1: the one rank runs the full "
                                               "sharded exchange with itself (RCCL calls), not the P = 1 copy")
    line["config"].update({"rotating_sets": args.dist_sets, "numa_binding_rank0": numa, "peers": world,
                           "path": args.path, "transport": args.transport,
                           "algbw_GiB_s": extra["algbw_GiB_s"], "busbw_GiB_s": extra["busbw_GiB_s"],
                           "shard_elems": extra["shard_elems"]})
    line["self_check"] = check
    if world > 1:
        egress = 2 * (world - 1) * S / world
        xg = egress / (step_ms * 1e-3) / 1e9
        xpeak = (world - 1) * XGMI_LINK_GBS_PER_DIR
        line["xgmi_roofline"] = {"bound": "xgmi", "achieved": round(xg, 1), "peak": round(xpeak, 1), "unit": "GB/s",
                                 "frac": round(xg / xpeak, 4), "bytes_per_step_per_gpu": int(egress),
                                 "note": "egress bytes per GPU (all-to-all + all-gather, (N-1)/N of the bucket "
                                         "each) / step time; peak = N-1 links x 76.8 GB/s per direction"
                                         + ("; PROC transport stages through host memory" if proc else "")}
    emit = _Emitter(line, rank)
    state = {}
    watchdog = threading.Timer(args.diag_deadline, emit.deadline, args=(state,))
    watchdog.daemon = True
    watchdog.start()
    try:
        after_value(args, ar, world, dist, line, proc)
    except Exception as e:  # never fails the measured line
        line["after_value_failed"] = f"{type(e).__name__}: {e}"
    emit.emit()
    ar.destroy()
    dist.barrier()
    dist.destroy_process_group()
    watchdog.cancel()
    if not check["ok"]:
        print("bench: self-check FAILED: the sharded allreduce differs from the single-GPU kernel", file=sys.stderr,
              flush=True)
        sys.exit(1)


def _fall_back(args, world, rank, watch, dev, numa, ar, err, what, group=None) -> bool:
    """Every rank calls this at the same point, whether its own step raised (`err`) or not. If the step failed on
    any rank, the communicator is destroyed and the line is measured through torch.distributed's exchange
    (run_dist_torch_exchange); returns True then. The vote runs on `group` (a gloo group of its own, CPU tensor)
    when given, so it cannot pair with an RCCL collective a peer is still inside."""
    import torch
    import torch.distributed as dist

    watch.enter(f"agreement on {what}")
    if group is not None:
        on = torch.device("cpu")
    else:
        on = torch.device("cuda", dev) if dist.get_backend() == "nccl" else torch.device("cpu")  # gloo: CPU tests
    failed = torch.tensor([0 if err is None else 1], dtype=torch.int32, device=on)
    dist.all_reduce(failed, op=dist.ReduceOp.MAX, group=group)
    if not int(failed.item()):
        return False
    if ar is not None:
        try:
            ar.destroy()
        except Exception as e:  # an aborted communicator: its teardown is bounded, the fallback does not need it
            print(f"bench: rank {rank}: destroying the failed communicator: {e}", file=sys.stderr, flush=True)
    global _EXCHANGE
    _EXCHANGE = EXCHANGE_TORCH  # every line from here on (the measured one, or an error line) says so
    run_dist_torch_exchange(args, world, rank, watch, err or f"{what} failed on another rank", numa)
    return True


def run_dist_torch_exchange(args, world, rank, watch, comm_err, numa):
    """The N > 1 line when the product communicator (fmi_comm over RCCL) cannot be built on this node: the same
    workload — one f32 256 MiB bucket per GPU, sharded sum-allreduce, the fused tree kernel of libfmi_dev.so in the
    reference's bracketing on every shard — with the two exchanges carried by torch.distributed's own RCCL
    process group (all_to_all_single + all_gather_into_tensor, fmi_amd.collectives.ShardedAllreduce path "tree").
    Same bytes, same result bits (self-checked the same way); the line says why (`config.exchange_fallback`).
    C4 / C5 and the diagnostics need fmi_comm and are not run."""
    import torch
    import torch.distributed as dist

    from fmi_amd import Alg, Op
    from fmi_amd import device as fdev
    from fmi_amd.collectives import ShardedAllreduce, check_windows, local_equivalent
    from fmi_amd.comm import runtime_info

    print(f"bench: rank {rank}: falling back to torch.distributed's exchange ({comm_err})", file=sys.stderr, flush=True)
    watch.enter("fallback topology check")
    dev = torch.cuda.current_device()
    mine = {"rank": rank, "torch_device": dev, "pci_bus_id": fdev.pci_bus_id(dev), "runtime": runtime_info()}
    every = [None] * world
    dist.all_gather_object(every, mine)
    buses = [e["pci_bus_id"] for e in every]
    topo = {"ok": len(set(buses)) == world, "ranks": world, "distinct_gpus": len(set(buses)) == world,
            "pci_bus_ids": buses, "runtime": every[0]["runtime"], "source": "torch.distributed all_gather_object"}
    if not topo["ok"]:
        print("bench: topology check FAILED: " + json.dumps(topo), file=sys.stderr, flush=True)
        if rank == 0:
            print(json.dumps(_error_line(world, "topology check failed", "fallback topology check", topology=topo,
                                         fmi_comm_error=comm_err)), file=json_out(), flush=True)
        os._exit(1)
    n = args.bucket_mib * MIB // 4
    S = n * 4
    sar = ShardedAllreduce(dist.group.WORLD, path="tree", force_exchange=world == 1)
    watch.enter("fallback warm-up and timed allreduces")
    step_ms, _, extra = sar.bench(n, steps=args.steps, warmup=args.warmup, sets=args.dist_sets, peers_per_gpu=1,
                                  return_result=True)
    out, seed = extra.pop("result")
    value = world * (S / GIB) / (step_ms * 1e-3)
    watch.enter("fallback self-check")
    torch.cuda.synchronize()
    check = check_windows(world, rank, sar.shard_elems(n), n, seed, lambda st, w: out[st:st + w].cpu().numpy(),
                          sar.max_over_ranks)
    del out
    watch.enter("fallback shard-kernel timing")
    shard = sar.shard_elems(n)
    parts = [[torch.empty(shard, dtype=torch.float32, device=sar.engine.device) for _ in range(world)] for _ in range(2)]
    for s_, ps in enumerate(parts):
        for p, t in enumerate(ps):
            sar.engine.fill_synthetic(t, 42 + s_, p)
    red = torch.empty(shard, dtype=torch.float32, device=sar.engine.device)
    launches = max(10, min(args.steps, 50))
    for k in range(2):
        sar.engine.reduce_tree(Op.SUM, Alg.ALLREDUCE, red, parts[k % 2])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()  # torch's current stream: the one HipEngine launches on
    for k in range(launches):
        sar.engine.reduce_tree(Op.SUM, Alg.ALLREDUCE, red, parts[k % 2])
    e1.record()
    e1.synchronize()
    shard_ms = sar.max_over_ranks(e0.elapsed_time(e1) / launches)[0]
    del parts, red
    watch.done()
    roof = _roofline("tree_kernel", (world + 1) * shard * 4, shard_ms,
                     "torch.cuda.Event around back-to-back launches of the shard kernel on torch's current stream (the "
                     "stream HipEngine launches on) after the timed region, max over ranks",
                     {"note": "the allreduce step is xGMI-bound (xgmi_roofline); this is its HBM-bound kernel"},
                     pmc_key=f"tree_kernel<fmi::dev::OpSum, float, 0, {world}, false>")
    line = _headline(args, value, step_ms,
                     f"C4-shaped at the metric's bucket size: {world}-peer float32 sum-allreduce, one FMI peer "
                     f"(a {args.bucket_mib} MiB device-resident bucket) per GPU",
                     f"{world} GPUs, one peer per GPU, buckets sharded {world} ways; all-to-all + fused tree kernel "
                     f"+ all-gather (bit-exact), exchanges through torch.distributed (RCCL)", n, roof)
    line["exchange"] = EXCHANGE_TORCH
    line["config"]["topology"] = topo
    line["config"].update({"rotating_sets": args.dist_sets, "numa_binding_rank0": numa, "peers": world,
                           "path": "tree", "transport": "torch.distributed (nccl backend = RCCL)",
                           "algbw_GiB_s": extra["algbw_GiB_s"], "busbw_GiB_s": extra["busbw_GiB_s"],
                           "shard_elems": shard})
    line["config"]["exchange_fallback"] = {
        "reason": comm_err,
        "parity": ("unpinned at N > 1: this fallback's self-check (check_windows, every rank, bit-exact against the "
                   "single-GPU kernel) has run on hardware only at world size 1 (--force-dist); no multi-GPU run of it "
                   "exists yet") if world > 1 else "self-checked at world size 1",
        "exchange": "torch.distributed all_to_all_single + all_gather_into_tensor on torch's RCCL process group "
                    "(fmi_amd.collectives.ShardedAllreduce); the shard kernel is libfmi_dev.so's fused tree kernel"}
    line["self_check"] = check
    if world > 1:
        egress = 2 * (world - 1) * S / world
        xg = egress / (step_ms * 1e-3) / 1e9
        xpeak = (world - 1) * XGMI_LINK_GBS_PER_DIR
        line["xgmi_roofline"] = {"bound": "xgmi", "achieved": round(xg, 1), "peak": round(xpeak, 1), "unit": "GB/s",
                                 "frac": round(xg / xpeak, 4), "bytes_per_step_per_gpu": int(egress)}
    if rank == 0:
        try:
            le = local_equivalent(world, n)
            le["value_over_local"] = round(line["value"] / le["GiB_s_reduced_buckets"], 4)
            line["local_equivalent"] = le
        except Exception as e:  # reported; the line is still printed
            line["local_equivalent"] = {"error": f"{type(e).__name__}: {e}"}
    line["c4"] = line["c5"] = "not run (needs the fmi_comm communicator)"
    allowed = bool(getattr(args, "allow_exchange_fallback", False))
    if not allowed:  # the product failed: the rate measured through torch's exchange is not the headline
        line["fallback_value"] = line["value"]
        line["value"] = None
        line["exchange_fallback_note"] = ("fmi_comm failed (config.exchange_fallback.reason); `fallback_value` is the "
                                          "same workload through torch.distributed's exchange. Exit status 1; "
                                          "--allow-exchange-fallback reports it as `value` and exits 0")
    _Emitter(line, rank).emit()
    dist.barrier()
    dist.destroy_process_group()
    if not check["ok"]:
        print("bench: self-check FAILED: the sharded allreduce differs from the single-GPU kernel", file=sys.stderr,
              flush=True)
        sys.exit(1)
    if not allowed:
        print("bench: fmi_comm failed; the line carries the torch.distributed exchange's rate as `fallback_value` "
              "(--allow-exchange-fallback to report it as `value`)", file=sys.stderr, flush=True)
        sys.exit(1)


def after_value(args, ar, world, dist, line, proc):
    """The single-GPU anchor, config C4 at its own size, config C5, then the diagnostics — each max over
    ranks, recorded into `line` as it completes (a deadline prints whatever is there)."""
    if ar.rank == 0:  # the same N x S allreduce on ONE GPU (no exchange): separates xGMI cost from HBM cost
        try:  # rank 0 alone: a failure here must not skip the barrier the other ranks wait in
            le = ar.local_equivalent(args.bucket_mib * MIB // 4)
            le["value_over_local"] = round(line["value"] / le["GiB_s_reduced_buckets"], 4)
            line["local_equivalent"] = le
        except Exception as e:  # reported; every rank still runs the same sequence of collectives
            line["local_equivalent"] = {"error": f"{type(e).__name__}: {e}"}
    dist.barrier()
    n4 = args.c4_mib * MIB // 4
    steps4, warm4 = max(5, args.steps // 10), 2
    c4 = line["c4"] = {"workload": f"C4: {world} peers x {args.c4_mib} MiB f32 sum-allreduce, one peer per GPU",
                       "elements": n4, "steps": steps4, "warmup": warm4, "rotating_sets": 2}
    for path in ("tree", "rccl"):
        if proc and path == "rccl":
            c4[path] = "not run (path RCCL needs the RCCL transport)"
            continue
        ms, _, ex = ar.bench(n4, steps=steps4, warmup=warm4, sets=2, peers_per_gpu=1, seed=1000, path=path)
        out, seed = ex.pop("result")
        chk = ar.self_check(out, n4, seed, tolerance=path == "rccl")
        out.free()
        c4[path] = {"ms_per_step": round(ms, 4), "algbw_GiB_s": ex["algbw_GiB_s"], "busbw_GiB_s": ex["busbw_GiB_s"],
                    "GiB_s_reduced_buckets": round(world * (n4 * 4 / GIB) / (ms * 1e-3), 2), "self_check": chk}
        if not chk["ok"]:
            line["self_check"] = dict(line["self_check"], ok=False, failed_in=f"c4 path {path}")
    if not args.no_c5:
        quiet_device()
        line["c5"] = dict(ar.host_bench(args.c5_mib * MIB // 4),
                          workload=f"C5: {args.c5_mib} MiB f32 page-locked host bucket per rank, H2D + sharded "
                                   f"allreduce + D2H pipelined", after_pause_s=QUIET_S)
    if args.no_diagnostics:
        return
    diag = line["diagnostics"] = {}
    diag["replicated_pairs"] = replicated_pairs(args, ar)
    if not proc:
        from fmi_amd.collectives import phase_breakdown

        diag["phase_ms"] = phase_breakdown(args.bucket_mib * MIB // 4, dist.group.WORLD)
        diag["exchange_variants"] = exchange_variants(args, ar)
    if args.diag_direct:
        try:
            ok = ar.check_direct(1 << 20)
            ms, _, _ = ar.bench(args.bucket_mib * MIB // 4, steps=max(10, args.steps // 4), warmup=3, sets=2,
                                path="direct")
            diag["path_direct"] = {"bit_identical_to_tree": ok, "ms_per_step": round(ms, 5)}
        except Exception as e:  # window setup fails on every rank alike (all-or-nothing)
            diag["path_direct"] = f"unavailable: {e}"
    else:
        diag["path_direct"] = "not run (opt-in: --diag-direct)"


def exchange_variants(args, ar) -> dict:
    """The headline step (path TREE, 256 MiB per peer) with each RCCL realisation of its two exchanges:
    ncclAllToAll or grouped send/recv for the all-to-all (FMI_TUNE_COMM_A2A), ncclAllGather or grouped
    send/recv of the shard to every peer for the all-gather (FMI_TUNE_COMM_GATHER), and, with
    --diag-pipeline only, the allreduce pipelined in 4 or 8 chunks (FMI_TUNE_COMM_PIPELINE: chunk k's
    all-gather on a second communicator while chunk k+1's all-to-all runs — experimental: two RCCL
    communicators in flight at once have not run across GPUs yet). Every rank sets the same values (the
    loop is the same on every rank). Same bytes, same result bits (self-checked); the step time decides the
    default. Max over ranks."""
    import fmi_amd
    from fmi_amd import Tune

    n = args.bucket_mib * MIB // 4
    steps = max(10, args.steps // 10)
    out = {}
    variants = [(a2a, gather, 0) for a2a in (0, 1) for gather in (0, 1)]
    if args.diag_pipeline:
        variants += [(0, 0, 4), (0, 0, 8)]
    try:
        for a2a, gather, chunks in variants:
            fmi_amd.tune_set(Tune.COMM_A2A, a2a)
            fmi_amd.tune_set(Tune.COMM_GATHER, gather)
            fmi_amd.tune_set(Tune.COMM_PIPELINE, chunks)
            ms, _, ex = ar.bench(n, steps=steps, warmup=2, sets=2, peers_per_gpu=1, seed=77)
            res, seed = ex.pop("result")
            ok = ar.self_check(res, n, seed, width=1024)["ok"]
            res.free()
            name = f"a2a_{'grouped' if a2a else 'nccl'}+gather_{'grouped' if gather else 'nccl'}"
            out[name + (f"+pipeline{chunks}" if chunks else "")] = {"ms_per_step": round(ms, 4), "self_check_ok": ok}
    finally:
        fmi_amd.tune_set(Tune.COMM_A2A, 0)
        fmi_amd.tune_set(Tune.COMM_GATHER, 0)
        fmi_amd.tune_set(Tune.COMM_PIPELINE, 0)
    return out


def replicated_pairs(args, ar) -> dict:
    """C2 on every GPU at once (each combines its own pair of 256 MiB buckets, no data-path collective):
    what round 1 reported as value at N > 1. Max over ranks."""
    import numpy as np

    import fmi_amd
    from fmi_amd import Bucket, Event, Op

    n = args.bucket_mib * MIB // 4
    sets = [tuple(Bucket(n, np.float32).fill_synthetic(42 + s, 2 * ar.rank + j) for j in range(2))
            for s in range(args.dist_sets)]
    steps = max(20, args.steps // 4)
    for k in range(5):
        fmi_amd.reduce_pair(Op.SUM, *sets[k % len(sets)])
    fmi_amd.sync()
    e0, e1 = Event(), Event()
    e0.record()
    for k in range(steps):
        fmi_amd.reduce_pair(Op.SUM, *sets[k % len(sets)])
    e1.record()
    e1.sync()
    ms = ar.max_over_ranks(e0.elapsed_ms(e1) / steps)[0]
    for a, b in sets:
        a.free()
        b.free()
    return {"ms_per_step": round(ms, 5), "GiB_s_all_gpus": round(ar.world * (n * 4 / GIB) / (ms * 1e-3), 2),
            "steps": steps}


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def relay(cmd, env=None) -> int:
    """Run `cmd` as a CHILD process (never exec: this process may not replace itself once anything touched the
    GPU, and nothing here has) and relay its output: JSON lines go to our stdout as they arrive, everything else
    to stderr, so the one line rank 0 prints stays the only stdout line. Returns the child's exit status
    (non-zero when any rank failed: torch.distributed.run exits non-zero then)."""
    child = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, bufsize=1, env=env)
    try:
        for line in child.stdout:
            out = sys.stdout if line.lstrip().startswith("{") else sys.stderr
            out.write(line)
            out.flush()
        return child.wait()
    except BaseException:
        child.kill()
        child.wait()
        raise


def launch_ranks(n: int, argv) -> int:
    """`python bench.py --gpus N` (N > 1) started without a launcher: start N ranks, one per GPU, under
    torch.distributed.run on this node (rendezvous on 127.0.0.1) as a child process, relay rank 0's line, and
    return non-zero if any rank failed. Runs before torch or fmi_amd is imported."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    print("bench: --gpus %d without a launcher: starting %s" % (n, " ".join(cmd)), file=sys.stderr, flush=True)
    env = dict(os.environ, FMI_BENCH_LAUNCHED="1")
    return relay(cmd, env)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        if os.environ.get("FMI_BENCH_LAUNCHED"):  # a launched rank without WORLD_SIZE: never recurse
            raise SystemExit("bench: launched rank has no WORLD_SIZE")
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if world != args.gpus:
        if args.gpus > 1 and world == 1:
            raise SystemExit(f"--gpus {args.gpus} needs {args.gpus} processes (launched with WORLD_SIZE=1)")
        args.gpus = world
    if os.environ.get("FMI_BENCH_TEST_FAIL_RANK") == str(rank) and world > 1:  # CPU test of the launcher's status
        raise SystemExit(f"bench: rank {rank} failing on purpose (FMI_BENCH_TEST_FAIL_RANK)")
    if world > 1 or args.force_dist:
        try:
            run_dist(args, world, rank, local_rank)
        except Exception as e:  # a failed N > 1 run still leaves one line saying where and why, then fails
            if rank == 0 and not _LINE_PRINTED:
                print(json.dumps(_error_line(world, f"{type(e).__name__}: {e}", _WATCH.phase if _WATCH else "start")),
                      file=json_out(), flush=True)
            raise
    else:
        run_single(args)


if __name__ == "__main__":
    main()
