"""One process of tests/test_gpu_comm.py::test_comm_rccl_one_rank_runs_the_full_exchange:

    python -m tests._one_rank_worker [--torch-first]

A one-rank RCCL communicator with FMI_TUNE_COMM_ONE_RANK_EXCHANGE = 1 runs every collective through the full
sharded schedule (real RCCL calls against itself) and checks every result against the reference's P = 1 result
(the rank's own bucket, bit for bit). --torch-first imports torch before the library, so librccl is torch's
copy (what bench.py's N > 1 path runs); otherwise the system's. Prints "one-rank exchange ok" on success."""
import sys

if "--torch-first" in sys.argv:
    import torch  # noqa: F401

import numpy as np

import fmi_amd
from fmi_amd import Bucket, Op
from fmi_amd.comm import Comm, Path, Transport, unique_id
from tests.test_gpu_parity import assert_bit_equal, inputs


def librccl_path() -> str:
    for line in open("/proc/self/maps"):
        if "librccl" in line:
            return line.split()[-1]
    return "?"


def main():
    fmi_amd.init(0)
    Tn = fmi_amd.Tune
    uid = unique_id(Transport.RCCL)
    c = Comm(uid, 1, 0, timeout_s=120)
    q = c.query()
    assert q["count"] == 1 and q["rank"] == 0
    fmi_amd.tune_set(Tn.COMM_ONE_RANK_EXCHANGE, 1)
    try:
        for dtype, op in ((np.float32, Op.SUM), (np.float64, Op.MAX), (np.int64, Op.MIN)):
            for n in (4099, 64 * 1024, (1 << 20) + 64):
                x = inputs(dtype, n, 0, seed=71)
                s, out = Bucket.from_numpy(x), Bucket(n, dtype)
                variants = [(a2a, gather, 0) for a2a in (0, 1) for gather in (0, 1)]
                if n >= (1 << 20):
                    variants.append((0, 0, 4))  # pipelined: a second, split communicator on a second stream
                for a2a, gather, pipe in variants:
                    fmi_amd.tune_set(Tn.COMM_A2A, a2a)
                    fmi_amd.tune_set(Tn.COMM_GATHER, gather)
                    fmi_amd.tune_set(Tn.COMM_PIPELINE, pipe)
                    for path in (Path.TREE, Path.RCCL):
                        out.upload(np.zeros(n, dtype))
                        c.allreduce(op, s, out, path=path)
                        c.sync()
                        assert_bit_equal(out.numpy(), x, f"allreduce {np.dtype(dtype).name} n={n} {path.name} "
                                                         f"a2a={a2a} gather={gather} pipe={pipe}")
                fmi_amd.tune_set(Tn.COMM_A2A, 0)
                fmi_amd.tune_set(Tn.COMM_GATHER, 0)
                fmi_amd.tune_set(Tn.COMM_PIPELINE, 0)
                for ordered in (False, True):
                    out.upload(np.zeros(n, dtype))
                    c.reduce(op, s, out, 0, ordered=ordered)
                    c.sync()
                    assert_bit_equal(out.numpy(), x, f"reduce ordered={ordered}")
                    out.upload(np.zeros(n, dtype))
                    c.scan(op, s, out, ordered=ordered)
                    c.sync()
                    assert_bit_equal(out.numpy(), x, f"scan ordered={ordered}")
                sb = Bucket.from_numpy(x)
                out.upload(np.zeros(n, dtype))
                c.reduce(op, sb, out, 0, sendbuf_partials=True)
                c.sync()
                assert_bit_equal(out.numpy(), x, "reduce_sendbuf result")
                assert_bit_equal(sb.numpy(), x, "reduce_sendbuf partial of the root")
                for b in (s, out, sb):
                    b.free()
        # path DIRECT: the window's IPC handle exchanged by ncclAllGather and agreed by ncclAllReduce(min)
        w = c.window(4099, np.float32)
        x = inputs(np.float32, 4099, 0, seed=72)
        w.upload(x)
        out = Bucket(4099, np.float32)
        c.allreduce(Op.SUM, w, out, path=Path.DIRECT)
        c.sync()
        assert_bit_equal(out.numpy(), x, "DIRECT")
        c.window_free(w)
        out.free()
        # host pipeline (C5 shape, small): H2D / sharded allreduce / D2H
        h = np.ascontiguousarray(inputs(np.float32, 3 * 65536 + 5, 0, seed=73))
        r = np.empty_like(h)
        c.allreduce_host(Op.SUM, h, r, chunk=65536)
        assert_bit_equal(r, h, "host allreduce")
        c.barrier()
    finally:
        for key in (Tn.COMM_A2A, Tn.COMM_GATHER, Tn.COMM_PIPELINE, Tn.COMM_ONE_RANK_EXCHANGE):
            fmi_amd.tune_set(key, 0)
    c.destroy()
    print("librccl mapped:", librccl_path(), flush=True)
    print("one-rank exchange ok", flush=True)


if __name__ == "__main__":
    main()
