"""Is bench.py's slow C5 at world size 1 (~39 ms vs 23.5 ms) a property of WHEN the page-locked host buckets
are allocated? Times fmi_comm_allreduce_host of 1 GiB with buckets allocated right after the communicator is
made (early) and after bench.py's headline + C4 device loops (late), in one process, several times each;
also reports how much of each buffer is backed by transparent huge pages (/proc/self/smaps).

    python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 \
        --master-port 29619 tools/c5_pinned_probe.py
"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
MIB = 1 << 20


def thp_kib(addr: int, size: int) -> int:
    """AnonHugePages (KiB) of the mapping that contains addr."""
    cur = None
    with open("/proc/self/smaps") as f:
        for line in f:
            head = line.split()
            if "-" in head[0] and len(head) >= 5 and all(c in "0123456789abcdef-" for c in head[0]):
                lo, hi = (int(x, 16) for x in head[0].split("-"))
                cur = (lo, hi)
            elif cur and cur[0] <= addr < cur[1] and head[0] == "AnonHugePages:":
                return int(head[1])
    return -1


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    dev = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    import fmi_amd
    from fmi_amd import Op
    from fmi_amd.collectives import CommAllreduce
    from fmi_amd.device import PinnedArray

    fmi_amd.init(dev)
    ar = CommAllreduce(dist.group.WORLD, path="tree", transport="rccl")
    n = 1024 * MIB // 4

    def alloc():
        s, r = PinnedArray(n, np.float32), PinnedArray(n, np.float32)
        s.array[:] = 1.0
        return s, r

    def timed(bufs, tag, reps=4):
        s, r = bufs
        ts = []
        for k in range(reps + 1):
            t0 = time.perf_counter()
            ar.comm.allreduce_host(Op.SUM, s.array, r.array, chunk=64 << 18)
            if k:
                ts.append((time.perf_counter() - t0) * 1e3)
        print(json.dumps({tag: round(statistics.median(ts), 3), "thp_kib_send": thp_kib(s.array.ctypes.data, n * 4),
                          "thp_kib_recv": thp_kib(r.array.ctypes.data, n * 4)}), flush=True)

    early = alloc()
    timed(early, "early_buffers_at_start")
    for nn, sets in ((256 * MIB // 4, 4), (1024 * MIB // 4, 2)):
        _, _, ex = ar.bench(nn, steps=10, warmup=2, sets=sets, peers_per_gpu=1)
        ex["result"][0].free()
    if os.environ.get("PROBE_SLEEP"):
        time.sleep(float(os.environ["PROBE_SLEEP"]))
    timed(early, "early_buffers_after_device_loops")
    late = alloc()
    timed(late, "late_buffers_after_device_loops")
    timed(early, "early_buffers_again")
    for b in early + late:
        b.free()
    ar.destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
