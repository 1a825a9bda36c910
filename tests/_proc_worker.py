"""One rank of a PROC-transport communicator, run as its own process by tests/test_gpu_proc.py:

    python -m tests._proc_worker <uid hex> <nranks> <rank> <out.npz>

Runs every collective of the C-ABI communicator on the same seeded buckets the parent regenerates, then
saves what this rank received. The parent compares each array bit for bit with the oracle; this process
only computes (no oracle calls)."""
import sys

import numpy as np

import fmi_amd
from fmi_amd import Bucket, Op
from fmi_amd.comm import Comm, Path
from tests.test_gpu_parity import inputs

# (name, dtype, op, n): n = 10 Mi + 3 floats makes every exchange larger than the 32 MiB staging slot
ALLREDUCE_CASES = [("f32_sum", np.float32, Op.SUM, 1027), ("i64_prod", np.int64, Op.PROD, 3 * 65536 + 5),
                   ("f64_max", np.float64, Op.MAX, 1), ("i32_min", np.int32, Op.MIN, 4099),
                   ("u8_sum", np.uint8, Op.SUM, 65536 + 3), ("f32_big", np.float32, Op.SUM, 10 * (1 << 20) + 3),
                   ("f32_div", np.float32, Op.SUM, 3 * (1 << 20))]  # divisible by N = 2, 3, 4: skewed shards
BIG = 10 * (1 << 20) + 3


def run(c, N, r):
    out = {}
    for name, dtype, op, n in ALLREDUCE_CASES:
        s, o = Bucket.from_numpy(inputs(dtype, n, r, seed=31)), Bucket(n, dtype)
        c.allreduce(op, s, o)
        fmi_amd.sync()
        out["allreduce_" + name] = o.numpy()
    x = inputs(np.float32, 4099, r, seed=32)
    s, o = Bucket.from_numpy(x), Bucket(4099, np.float32)
    c.allreduce(Op.SUM, s, o, ordered=True)
    fmi_amd.sync()
    out["ordered"] = o.numpy()
    for root in range(N):
        s = Bucket.from_numpy(inputs(np.float32, 2053, r, seed=33))
        o = Bucket(2053, np.float32) if r == root else None
        c.reduce(Op.SUM, s, o, root)
        fmi_amd.sync()
        if o is not None:
            out["reduce"] = o.numpy()
    for dtype, op in ((np.float32, Op.SUM), (np.int64, Op.MAX)):
        s, o = Bucket.from_numpy(inputs(dtype, 65536 + 129, r, seed=34)), Bucket(65536 + 129, dtype)
        c.scan(op, s, o)
        fmi_amd.sync()
        out["scan_" + np.dtype(dtype).name] = o.numpy()
    # path DIRECT: windows exported with hipIpcGetMemHandle and mapped by every other process
    for dtype, op, n in ((np.float32, Op.SUM, 3 * 65536 + 5), (np.int32, Op.MIN, 1027)):
        w = c.window(n + 1, dtype)
        v = w.view(1, n)  # unaligned bucket inside the window
        v.upload(inputs(dtype, n, r, seed=35))
        o = Bucket(n, dtype)
        c.allreduce(op, v, o, path=Path.DIRECT)
        fmi_amd.sync()
        out["direct_" + np.dtype(dtype).name] = o.numpy()
        c.window_free(w)
    # a DIRECT allreduce on a user stream, its window freed right away (no sync): fmi_comm_window_free must
    # drain the device before the barrier that lets the peers free the memory this rank is still reading
    st = fmi_amd.Stream()
    n = 3 * 65536 + 5
    w = c.window(n, np.float32)
    w.upload(inputs(np.float32, n, r, seed=37))
    o = Bucket(n, np.float32)
    c.allreduce(Op.SUM, w, o, path=Path.DIRECT, stream=st)
    c.window_free(w)
    st.sync()
    out["direct_stream_free"] = o.numpy()
    st.destroy()
    # host buckets through the GPU (config C5's shape), pageable, several chunks
    x = inputs(np.float64, 3 * 4099 + 17, r, seed=36)
    got = np.zeros_like(x)
    c.allreduce_host(Op.SUM, x.copy(), got, chunk=4099)
    out["host_f64"] = got
    # data movement, bcast and point-to-point larger than a slot
    b = Bucket.from_numpy(np.full(BIG, r, dtype=np.int32))
    c.bcast(b, N - 1)
    fmi_amd.sync()
    out["bcast_ok"] = np.array([bool(np.all(b.numpy() == N - 1))])
    mine = Bucket.from_numpy(np.arange(1000, dtype=np.int64) + 1000 * r)
    allb = Bucket(N * 1000, np.int64) if r == 0 else None
    c.gather(mine, allb, 0)
    src = Bucket.from_numpy(np.arange(N * 1000, dtype=np.int64)) if r == N - 1 else None
    piece = Bucket(1000, np.int64)
    c.scatter(src, piece, N - 1)
    fmi_amd.sync()
    if allb is not None:
        out["gather"] = allb.numpy()
    out["scatter"] = piece.numpy()
    ring, got = Bucket.from_numpy(np.full(BIG, r, dtype=np.int32)), Bucket(BIG, np.int32)
    if r % 2 == 0:
        c.send(ring, (r + 1) % N)
        c.recv(got, (r - 1) % N)
    else:
        c.recv(got, (r - 1) % N)
        c.send(ring, (r + 1) % N)
    c.barrier()
    fmi_amd.sync()
    out["ring_ok"] = np.array([bool(np.all(got.numpy() == (r - 1) % N))])
    return out


def main():
    uid, N, r, path = bytes.fromhex(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    fmi_amd.init(0)
    c = Comm(uid, N, r)
    out = run(c, N, r)
    c.destroy()
    np.savez(path, **out)


if __name__ == "__main__":
    main()
