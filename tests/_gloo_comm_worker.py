"""One rank of the gloo-bootstrapped CommAllreduce test (tests/test_gpu_bench_dist.py), started by
`torch.distributed.run -m tests._gloo_comm_worker OUTDIR` (a fresh interpreter per rank: the pytest process,
which already holds the system HIP runtime through libfmi_dev.so, never imports torch and its bundled runtime):
the product N>1 driver code of bench.py (fmi_amd.collectives.CommAllreduce: id
broadcast over torch.distributed, bench loop, self-check, path DIRECT check, host-bucket allreduce) over the
PROC transport, every rank a process on the one GPU. Saves what it computed; the parent compares with the
oracle (this process makes no oracle call)."""
import os

import numpy as np


def run(outdir):
    import torch
    import torch.distributed as dist

    rank = int(os.environ["RANK"])
    dist.init_process_group("gloo")
    try:
        import fmi_amd
        from fmi_amd.collectives import CommAllreduce

        torch.cuda.set_device(0)
        fmi_amd.init(0)
        ar = CommAllreduce(dist.group.WORLD, path="tree", transport="proc")
        n = 1_000_003  # ragged: the shard grid pads
        out = {}
        step_ms, _, extra = ar.bench(n, steps=2, warmup=1, sets=2, peers_per_gpu=1, seed=42)
        res, seed = extra.pop("result")
        out["tree"] = res.numpy()
        out["tree_seed"] = np.array([seed])
        out["self_check_ok"] = np.array([ar.self_check(res, n, seed)["ok"]])
        # the check must catch a wrong result: the same bucket checked against other buckets' values
        out["self_check_wrong_seed_ok"] = np.array([ar.self_check(res, n, seed + 1, width=256)["ok"]])
        res.free()
        out["step_ms"] = np.array([step_ms])
        out["direct_ok"] = np.array([ar.check_direct(4099)])
        h = ar.host_bench(3 * 65536 + 64, iters=1, chunk=65536)
        out["host_ok"] = np.array([h["result_ok"]])
        k = ar.shard_kernel(65536, launches=3)
        out["kernel_bytes"] = np.array([k["algorithmic_bytes_per_launch"]])
        ar.destroy()
        np.savez(os.path.join(outdir, f"rank{rank}.npz"), **out)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    import sys

    run(sys.argv[1])
