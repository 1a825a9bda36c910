"""Config C5 under the two HIP runtimes a process can end up with: the system ROCm runtime (libfmi_dev.so
loaded first) or torch's bundled one (torch imported first, as bench.py's N > 1 path does). Times, on a
one-rank communicator, fmi_comm_allreduce_host of a 1 GiB page-locked f32 bucket at several chunk sizes and
the bare 1 GiB H2D / D2H copies, median of 5.

    python tools/c5_runtime_probe.py [--torch-first] [--affinity none|near|far]

--affinity pins the process to the CPUs of the GPU's NUMA node (near) or of another node (far) before any
host memory is allocated: page-locked buckets land on that node, and PCIe DMA from a far node crosses the
inter-socket link.
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _cpulist(text):
    cpus = set()
    for part in text.strip().split(","):
        if part:
            lo, _, hi = part.partition("-")
            cpus.update(range(int(lo), int(hi or lo) + 1))
    return cpus


def gpu_numa():
    """NUMA node of GPU 0 (the first /sys/class/drm card with a numa_node whose vendor is AMD) and the CPUs
    of every node."""
    import glob

    nodes = {}
    for d in glob.glob("/sys/devices/system/node/node[0-9]*"):
        try:
            nodes[int(d.rsplit("node", 1)[1])] = _cpulist(open(os.path.join(d, "cpulist")).read())
        except OSError:
            pass
    cards = []
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES") or ""
    for card in sorted(glob.glob("/sys/class/drm/card[0-9]*/device")):
        try:
            if open(os.path.join(card, "vendor")).read().strip() != "0x1002":
                continue
            cards.append(int(open(os.path.join(card, "numa_node")).read()))
        except (OSError, ValueError):
            continue
    gpu_node = cards[0] if cards and cards[0] >= 0 else None
    return {"gpu_node": gpu_node, "nodes": nodes, "visible": vis, "cards": cards}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--torch-first", action="store_true")
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--affinity", default="none", choices=["none", "near", "far"])
    ap.add_argument("--comm", default="local", choices=["local", "rccl"],
                    help="rccl: a torch 'nccl' process group (world 1, as bench.py --force-dist) and an RCCL-transport "
                         "communicator instead of a LOCAL one")
    args = ap.parse_args()
    info = gpu_numa()
    if args.affinity != "none" and info["gpu_node"] is not None and len(info["nodes"]) > 1:
        node = info["gpu_node"] if args.affinity == "near" else next(k for k in info["nodes"] if k != info["gpu_node"])
        os.sched_setaffinity(0, info["nodes"][node])
    if args.torch_first or args.comm == "rccl":
        import torch

        torch.cuda.init()
    if args.comm == "rccl":
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29547")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    import numpy as np

    import fmi_amd
    from fmi_amd import Bucket, Op, PinnedArray, _lib
    from fmi_amd.comm import Comm, Transport, unique_id

    fmi_amd.init(0)
    n = args.mib * (1 << 20) // 4
    comm = Comm(unique_id(Transport.RCCL if args.comm == "rccl" else Transport.LOCAL), 1, 0)
    send, recv = PinnedArray(n, np.float32), PinnedArray(n, np.float32)
    send.array[:] = 1.0
    dev = Bucket(n, np.float32)
    res = {"runtime": "torch" if args.torch_first or args.comm == "rccl" else "system", "comm": args.comm, "mib": args.mib, "affinity": args.affinity,
           "gpu_numa_node": info["gpu_node"], "numa_nodes": len(info["nodes"]), "cards_numa": info["cards"],
           "cpus_allowed": len(os.sched_getaffinity(0)), "launcher": os.environ.get("TORCHELASTIC_RUN_ID", "direct")}

    def timed(fn, reps=5):
        fn()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return round(statistics.median(ts) * 1e3, 3)

    def h2d():
        _lib.call("fmi_dev_h2d_async", dev.ptr, send.ptr, n * 4, None)
        _lib.call("fmi_stream_sync", None)

    def d2h():
        _lib.call("fmi_dev_d2h_async", recv.ptr, dev.ptr, n * 4, None)
        _lib.call("fmi_stream_sync", None)

    res["h2d_ms"] = timed(h2d)
    res["d2h_ms"] = timed(d2h)
    for chunk_mib in (16, 32, 64, 128, 256):
        res[f"allreduce_host_chunk{chunk_mib}_ms"] = timed(
            lambda: comm.allreduce_host(Op.SUM, send.array, recv.array, chunk=chunk_mib * (1 << 20) // 4))
    res["ok"] = bool(np.all(recv.array == 1.0))
    print(json.dumps(res), flush=True)
    send.free()
    recv.free()
    dev.free()
    comm.destroy()


if __name__ == "__main__":
    main()
