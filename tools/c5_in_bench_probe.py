"""Why bench.py's N > 1 path reports C5 at ~39 ms at world size 1 while a bare probe (tools/c5_runtime_probe.py
--comm rccl) gets 23.5 ms: time CommAllreduce.host_bench (1 GiB page-locked host bucket) after each stage of
bench.py's N > 1 sequence — right after the communicator is made, after the headline loop (256 MiB), after
the C4 loops (1 GiB, paths TREE and RCCL) — in one process.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 \
        --master-port 29615 tools/c5_in_bench_probe.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

MIB = 1 << 20


def main():
    import torch
    import torch.distributed as dist

    dev = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    import fmi_amd
    from fmi_amd.collectives import CommAllreduce

    fmi_amd.init(dev)
    ar = CommAllreduce(dist.group.WORLD, path="tree", transport="rccl")
    n5 = 1024 * MIB // 4
    out = {}

    def c5(tag):
        out[tag] = ar.host_bench(n5)["ms"]
        print(json.dumps({tag: out[tag]}), flush=True)

    c5("after_init")
    c5("after_init_again")
    n = 256 * MIB // 4
    _, _, ex = ar.bench(n, steps=20, warmup=3, sets=4, peers_per_gpu=1)
    res, seed = ex.pop("result")
    c5("after_headline_loop")
    ar.self_check(res, n, seed)
    res.free()
    c5("after_self_check")
    ar.shard_kernel(n, launches=20)
    c5("after_shard_kernel")
    for path in ("tree", "rccl"):
        _, _, ex = ar.bench(1024 * MIB // 4, steps=5, warmup=2, sets=2, peers_per_gpu=1, seed=1000, path=path)
        ex["result"][0].free()
        c5(f"after_c4_{path}")
    fmi_amd.sync()
    torch.cuda.empty_cache()
    c5("after_empty_cache")
    ar.destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
