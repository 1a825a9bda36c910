"""The C-ABI communicator (fmi_comm_*) — sharded allreduce / reduce / scan across ranks — run with the
LOCAL transport: N ranks are threads of this process on the one MI355X, exchanging through device copies.
The schedules (shard layout, padding, all-to-all, fused kernel in the reference's order, all-gather /
gather / all-to-all back) are exactly those the RCCL transport runs across GPUs; the result of every rank
is compared bit-exactly with the oracle's simulation of the reference collective over the same buckets.
"""
import os
import threading

import numpy as np
import pytest

import fmi_amd
from fmi_amd import Bucket, Op, PinnedArray
from fmi_amd.comm import Comm, Path, Transport, unique_id
from oracle import fmi_oracle as orc
from tests.test_gpu_parity import OPNAME, assert_bit_equal, inputs

pytestmark = pytest.mark.gpu


def run_ranks(N, body):
    uid = unique_id(Transport.LOCAL)
    errors = [None] * N
    results = [None] * N

    def worker(r):
        try:
            c = Comm(uid, N, r)
            results[r] = body(c, r)
            c.destroy()
        except BaseException as e:  # noqa: BLE001 - re-raised below
            errors[r] = e

    threads = [threading.Thread(target=worker, args=(r,)) for r in range(N)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=300)
    for e in errors:
        if e is not None:
            raise e
    return results


@pytest.mark.parametrize("N", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("n", [1, 1027, 3 * 65536 + 5])
def test_comm_allreduce_tree_bit_exact(device, N, n):
    for dtype, op in ((np.float32, Op.SUM), (np.int64, Op.PROD), (np.float64, Op.MAX), (np.int32, Op.MIN)):
        xs = [inputs(dtype, n, r, seed=11) for r in range(N)]

        def body(c, r):
            s, out = Bucket.from_numpy(xs[r]), Bucket(n, dtype)
            c.allreduce(op, s, out)
            fmi_amd.sync()
            return out.numpy(), s.numpy()

        res = run_ranks(N, body)
        with np.errstate(all="ignore"):
            want, _ = orc.allreduce(xs, orc.OPS[OPNAME[op]])
        for r in range(N):
            # every rank ends with its own reference bits (float max: each peer's own operand order)
            assert_bit_equal(res[r][0], want[r], f"N={N} n={n} {op.name} rank {r}")
            assert_bit_equal(res[r][1], xs[r], "send bucket untouched")


@pytest.mark.parametrize("N", [2, 5, 8])
def test_comm_allreduce_ordered(device, N):
    n = 4099
    xs = [inputs(np.float32, n, r, seed=3) for r in range(N)]

    def body(c, r):
        s, out = Bucket.from_numpy(xs[r]), Bucket(n, np.float32)
        c.allreduce(Op.SUM, s, out, ordered=True)
        fmi_amd.sync()
        return out.numpy()

    res = run_ranks(N, body)
    want, _ = orc.allreduce(xs, orc.op_sum, commutative=False, associative=False)
    for r in range(N):
        assert_bit_equal(res[r], want[r], f"rank {r}")


@pytest.mark.parametrize("N", [2, 3, 4, 7, 8])
def test_comm_reduce_every_root(device, N):
    n = 2053
    for ordered in (False, True):
        xs = [inputs(np.float32, n, r, seed=5) for r in range(N)]
        for root in range(N):
            def body(c, r):
                s = Bucket.from_numpy(xs[r])
                out = Bucket(n, np.float32) if r == root else None
                c.reduce(Op.SUM, s, out, root, ordered=ordered)
                fmi_amd.sync()
                return out.numpy() if out is not None else None

            res = run_ranks(N, body)
            want, _ = orc.reduce(xs, orc.op_sum, root=root, commutative=not ordered, associative=not ordered)
            assert_bit_equal(res[root], want, f"N={N} root {root} ordered={ordered}")


@pytest.mark.parametrize("N", [2, 3, 5, 8])
def test_comm_scan(device, N):
    n = 65536 + 129
    for ordered in (False, True):
        for dtype, op in ((np.float32, Op.SUM), (np.int64, Op.MAX)):
            xs = [inputs(dtype, n, r, seed=9) for r in range(N)]

            def body(c, r):
                s, out = Bucket.from_numpy(xs[r]), Bucket(n, dtype)
                c.scan(op, s, out, ordered=ordered)
                fmi_amd.sync()
                return out.numpy()

            res = run_ranks(N, body)
            with np.errstate(all="ignore"):
                want, _ = orc.scan(xs, orc.OPS[OPNAME[op]], commutative=not ordered, associative=not ordered)
            for r in range(N):
                assert_bit_equal(res[r], want[r], f"N={N} {op.name} ordered={ordered} rank {r}")


def test_comm_more_ranks_than_a_fused_kernel_holds(device):
    """N = 20 ranks: every rank's shard reduction is a 20-peer program, run as fused 16-peer blocks
    (allreduce on the TREE and DIRECT paths, reduce, scan) — bit-exact with the reference's 20-peer
    bracketing."""
    N, n = 20, 4099
    xs = [inputs(np.float32, n, r, seed=29) for r in range(N)]

    def body(c, r):
        s, out, red, sc = Bucket.from_numpy(xs[r]), Bucket(n, np.float32), Bucket(n, np.float32), Bucket(n, np.float32)
        c.allreduce(Op.SUM, s, out)
        c.reduce(Op.SUM, s, red if r == 3 else None, 3)
        c.scan(Op.SUM, s, sc)
        w, direct = c.window(n, np.float32), Bucket(n, np.float32)
        w.upload(xs[r])
        c.allreduce(Op.SUM, w, direct, path=Path.DIRECT)
        fmi_amd.sync()
        got = out.numpy(), red.numpy() if r == 3 else None, sc.numpy(), direct.numpy()
        c.window_free(w)
        return got

    res = run_ranks(N, body)
    want_ar, _ = orc.allreduce(xs, orc.op_sum)
    want_red, _ = orc.reduce(xs, orc.op_sum, root=3)
    want_sc, _ = orc.scan(xs, orc.op_sum)
    for r in range(N):
        assert_bit_equal(res[r][0], want_ar[r], f"allreduce rank {r}")
        assert_bit_equal(res[r][2], want_sc[r], f"scan rank {r}")
        assert_bit_equal(res[r][3], want_ar[r], f"allreduce DIRECT rank {r}")
    assert_bit_equal(res[3][1], want_red, "reduce root 3")


@pytest.mark.parametrize("N", [2, 3, 5, 8, 20])
def test_comm_reduce_sendbuf_partials(device, N):
    """fmi_comm_reduce_sendbuf: every rank's send ends as the reference leaves that peer's sendbuf
    (src/comm/PeerToPeer.cpp:72 — the partial an interior peer forwarded, a leaf's own bucket, the root's
    result), i.e. the oracle's second return value; recv on the root is the result. Plain fmi_comm_reduce
    leaves send untouched (include/fmi_dev.h: the documented divergence), and the ordered reduce_ltr leaves it
    intact in both (reference :44-57)."""
    n = 4099
    for dtype, op in ((np.float32, Op.SUM), (np.int64, Op.MAX), (np.float64, Op.MIN)):
        xs = [inputs(dtype, n, r, seed=47) for r in range(N)]
        for root in sorted({0, 1 % N, N - 1}):
            def body(c, r):
                s, out = Bucket.from_numpy(xs[r]), Bucket(n, dtype)
                c.reduce(op, s, out if r == root else None, root, sendbuf_partials=True)
                plain = Bucket.from_numpy(xs[r])
                c.reduce(op, plain, None if r != root else Bucket(n, dtype), root)
                ltr = Bucket.from_numpy(xs[r])
                c.reduce(op, ltr, None if r != root else Bucket(n, dtype), root, ordered=True, sendbuf_partials=True)
                fmi_amd.sync()
                return s.numpy(), out.numpy() if r == root else None, plain.numpy(), ltr.numpy()

            res = run_ranks(N, body)
            with np.errstate(all="ignore"):
                want, sends = orc.reduce(xs, orc.OPS[OPNAME[op]], root=root)
            for r in range(N):
                assert_bit_equal(res[r][0], sends[r], f"N={N} {op.name} root {root}: sendbuf of rank {r}")
                assert_bit_equal(res[r][2], xs[r], "plain reduce leaves send untouched")
                assert_bit_equal(res[r][3], xs[r], "reduce_ltr leaves sendbuf intact")
            assert_bit_equal(res[root][1], want, f"N={N} {op.name} root {root} result")


@pytest.mark.parametrize("N", [2, 5, 8])
def test_comm_allreduce_pipelined_chunks(device, N):
    """FMI_TUNE_COMM_PIPELINE = K: path TREE in K chunks (each its own sharded allreduce; the all-gathers on a
    second stream). Element-wise, so the result must equal, bit for bit, the single-GPU fused kernel over the
    whole buckets; ragged n (the last chunk pads its shards); buffer slots reused across calls."""
    from fmi_amd import Alg

    n = N * (1 << 20) + 12345
    ins = [Bucket(n, np.float32).fill_synthetic(53, r) for r in range(N)]
    ref = Bucket(n, np.float32)
    fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, ref, ins)
    fmi_amd.sync()
    want = ref.numpy()
    ref.free()
    try:
        for K in (3, 4):
            fmi_amd.tune_set(fmi_amd.Tune.COMM_PIPELINE, K)

            def body(c, r):
                out = Bucket(n, np.float32)
                for _ in range(2):  # buffer slots reused across calls
                    c.allreduce(Op.SUM, ins[r], out)
                fmi_amd.sync()
                got = out.numpy()
                out.free()
                return bool(np.array_equal(got.view(np.uint32), want.view(np.uint32)))

            assert all(run_ranks(N, body)), f"K={K}"
    finally:
        fmi_amd.tune_set(fmi_amd.Tune.COMM_PIPELINE, 0)
    for b in ins:
        b.free()


def test_comm_timing_counts_shard_kernels(device):
    """fmi_comm_timing: one event pair per shard-kernel launch of the collectives on the stream it runs on
    (TREE allreduce, DIRECT allreduce, per-rank float max); read returns the tally and starts a new one."""
    N, n = 3, 65536 + 17

    def body(c, r):
        s, out = Bucket.from_numpy(inputs(np.float32, n, r)), Bucket(n, np.float32)
        w = c.window(n, np.float32)
        w.upload(inputs(np.float32, n, r))
        c.timing(True)
        for _ in range(3):
            c.allreduce(Op.SUM, s, out)
        c.allreduce(Op.MAX, s, out)  # float max: the per-rank kernel, one launch
        c.allreduce(Op.SUM, w, out, path=Path.DIRECT)
        ms, k = c.timing_read()
        again = c.timing_read()
        c.timing(False)
        c.allreduce(Op.SUM, s, out)
        after = c.timing_read()
        c.window_free(w)
        return ms, k, again, after

    for r, (ms, k, again, after) in enumerate(run_ranks(N, body)):
        assert k == 5 and ms > 0, (r, ms, k)
        assert again == (0.0, 0) and after == (0.0, 0)


def test_comm_300_ranks(device):
    """No rank cap (the reference's collectives take any num_peers, src/comm/PeerToPeer.cpp:59-184): a
    300-rank communicator (LOCAL transport, 300 threads on the one GPU). Every shard reduction is a 300-peer
    program (three levels of fused 16-peer blocks); path DIRECT gathers through its device pointer table.
    Bit-exact vs the oracle for allreduce (TREE, DIRECT), reduce at a non-zero root and scan."""
    N, n = 300, 1027
    xs = [inputs(np.float32, n, r, seed=43) for r in range(N)]

    def body(c, r):
        s, out, red, sc = Bucket.from_numpy(xs[r]), Bucket(n, np.float32), Bucket(n, np.float32), Bucket(n, np.float32)
        c.allreduce(Op.SUM, s, out)
        c.reduce(Op.SUM, s, red if r == 37 else None, 37)
        c.scan(Op.SUM, s, sc)
        w, direct = c.window(n, np.float32), Bucket(n, np.float32)
        w.upload(xs[r])
        c.allreduce(Op.SUM, w, direct, path=Path.DIRECT)
        fmi_amd.sync()
        got = out.numpy(), red.numpy() if r == 37 else None, sc.numpy(), direct.numpy()
        c.window_free(w)
        return got

    res = run_ranks(N, body)
    with np.errstate(all="ignore"):  # the synthetic edge values include ±inf: inf + -inf = NaN, as on the GPU
        want_ar, _ = orc.allreduce(xs, orc.op_sum)
        want_red, _ = orc.reduce(xs, orc.op_sum, root=37)
        want_sc, _ = orc.scan(xs, orc.op_sum)
    for r in range(N):
        assert_bit_equal(res[r][0], want_ar[r], f"allreduce rank {r}")
        assert_bit_equal(res[r][2], want_sc[r], f"scan rank {r}")
        assert_bit_equal(res[r][3], want_ar[r], f"allreduce DIRECT rank {r}")
    assert_bit_equal(res[37][1], want_red, "reduce root 37")


def _host_allreduce(c, r, x, op, ordered, pinned, chunk):
    n, dtype = x.size, x.dtype
    if pinned:
        s, out = PinnedArray(n, dtype), PinnedArray(n, dtype)
        s.array[:] = x
        c.allreduce_host(op, s.array, out.array, ordered=ordered, chunk=chunk)
        res = out.array.copy(), s.array.copy()
        s.free()
        out.free()
        return res
    s, out = x.copy(), np.zeros(n, dtype)
    c.allreduce_host(op, s, out, ordered=ordered, chunk=chunk)
    return out, s


@pytest.mark.parametrize("N", [1, 2, 3, 8])
@pytest.mark.parametrize("pinned", [True, False])
def test_comm_allreduce_host_pipeline(device, N, pinned):
    """Host-ingress allreduce (config C5 shape): host buckets stream through the GPU in chunks (ragged last
    chunk, padded shards, slot reuse over > 2 chunks); every rank's host result equals the oracle's."""
    n, chunk = 3 * 4099 + 17, 4099
    for dtype, op, ordered in ((np.float32, Op.SUM, False), (np.int64, Op.MAX, False), (np.float64, Op.PROD, False),
                               (np.float32, Op.SUM, True)):
        xs = [inputs(dtype, n, r, seed=13) for r in range(N)]
        res = run_ranks(N, lambda c, r: _host_allreduce(c, r, xs[r], op, ordered, pinned, chunk))
        with np.errstate(all="ignore"):
            want, _ = orc.allreduce(xs, orc.OPS[OPNAME[op]], commutative=not ordered, associative=not ordered)
        for r in range(N):
            assert_bit_equal(res[r][0], want[r], f"N={N} {op.name} ordered={ordered} rank {r}")
            assert_bit_equal(res[r][1], xs[r], "send bucket untouched")


def test_comm_allreduce_host_concurrent_communicators(device):
    """Host pipelines of independent communicators at the same time (fmi_comm.hip HostPipe): three LOCAL
    communicators (1, 2 and 4 ranks: a one-rank pipeline on its own copy-stream pair at depth 2, the co-resident
    ranks of each larger one sharing their communicator's pair at depth 3) run host allreduces concurrently, several
    calls each with different chunkings, so their copies overlap on the device's DMA engines. Every rank's result
    equals the oracle's bit for bit."""
    sizes = {1: 9 * 4096 + 3, 2: 7 * 4096 + 5, 4: 11 * 4096 + 7}
    results, errors = {}, []

    def comm_job(N):
        n = sizes[N]
        xs = [[inputs(np.float32, n, r, seed=60 + N + k) for r in range(N)] for k in range(3)]

        def body(c, r):
            return [_host_allreduce(c, r, xs[k][r], Op.SUM, False, (r + k) % 2 == 0, 4096 * (k + 1))[0]
                    for k in range(3)]

        try:
            results[N] = (xs, run_ranks(N, body))
        except BaseException as e:  # noqa: BLE001 - reported below
            errors.append(f"N={N}: {e!r}")

    jobs = [threading.Thread(target=comm_job, args=(N,)) for N in sizes]
    for t in jobs:
        t.start()
    for t in jobs:
        t.join(timeout=300)
    assert not errors and not any(t.is_alive() for t in jobs), errors
    for N, (xs, res) in results.items():
        for k in range(3):
            want, _ = orc.allreduce(xs[k], orc.OPS["sum"])
            for r in range(N):
                assert_bit_equal(res[r][k], want[r], f"communicator N={N} call {k} rank {r}")


@pytest.mark.parametrize("N", [2, 3, 8])
def test_comm_allreduce_skewed_shards_same_bits(device, N):
    """FMI_TUNE_COMM_SHARD_SKEW (fmi_comm.hip shard_stride): with shards of >= 1 MiB the
    all-to-all lands shard j at stride (shard rounded up to 64 KiB) + 4 KiB and the reduced shard in the next slot.
    Divisible and padded buckets, f32 sum and i64 max, give the same bits skewed and back to back, and equal the
    oracle."""
    from fmi_amd import Tune

    cases = [(np.float32, Op.SUM, N * (1 << 18)), (np.float32, Op.SUM, N * 3 * (1 << 18) + 64 * N),
             (np.int64, Op.MAX, N * (1 << 17) + 5)]
    old = fmi_amd.tune_get(Tune.COMM_SHARD_SKEW)
    try:
        for dtype, op, n in cases:
            xs = [inputs(dtype, n, r, seed=80 + N) for r in range(N)]
            got = {}
            for skew in (1, 0):
                fmi_amd.tune_set(Tune.COMM_SHARD_SKEW, skew)

                def body(c, r):
                    s, o = Bucket.from_numpy(xs[r]), Bucket(n, dtype)
                    c.allreduce(op, s, o)
                    fmi_amd.sync()
                    res = o.numpy()
                    s.free()
                    o.free()
                    return res

                got[skew] = run_ranks(N, body)
            with np.errstate(all="ignore"):
                want, _ = orc.allreduce(xs, orc.OPS[OPNAME[op]])
            for r in range(N):
                assert got[1][r].tobytes() == got[0][r].tobytes(), f"{np.dtype(dtype).name} n={n} rank {r}"
                assert_bit_equal(got[1][r], want[r], f"{np.dtype(dtype).name} n={n} rank {r}")
    finally:
        fmi_amd.tune_set(Tune.COMM_SHARD_SKEW, old)


@pytest.mark.parametrize("N", [3, 8])
def test_comm_local_ranks_on_streams_of_their_own(device, N):
    """LOCAL ranks on the library stream and on streams of their own: allreduce, reduce (every root), scan and the
    host-ingress allreduce give the oracle's bits either way."""
    from fmi_amd import Stream

    n = 3 * 4099 + 5
    xs = [inputs(np.float32, n, r, seed=90 + N) for r in range(N)]
    with np.errstate(all="ignore"):
        want_ar, _ = orc.allreduce(xs, orc.op_sum)
        want_sc, _ = orc.scan(xs, orc.op_sum)
        want_red = [orc.reduce(xs, orc.op_sum, root=root)[0] for root in range(N)]
    for own_stream in (False, True):
        def body(c, r):
            st = Stream() if own_stream else None
            s, o = Bucket.from_numpy(xs[r]), Bucket(n, np.float32)
            c.allreduce(Op.SUM, s, o, stream=st)
            c.sync(st)
            ar = o.numpy(st)
            c.scan(Op.SUM, s, o, stream=st)
            c.sync(st)
            sc = o.numpy(st)
            red = []
            for root in range(N):
                c.reduce(Op.SUM, s, o if r == root else None, root, stream=st)
                c.sync(st)
                red.append(o.numpy(st) if r == root else None)
            host = _host_allreduce(c, r, xs[r], Op.SUM, False, r % 2 == 0, 4099)[0]
            s.free()
            o.free()
            if st is not None:
                st.destroy()
            return ar, sc, red, host

        res = run_ranks(N, body)
        for r in range(N):
            assert_bit_equal(res[r][0], want_ar[r], f"allreduce rank {r} own_stream={own_stream}")
            assert_bit_equal(res[r][1], want_sc[r], f"scan rank {r} own_stream={own_stream}")
            assert_bit_equal(res[r][3], want_ar[r], f"host allreduce rank {r} own_stream={own_stream}")
        for root in range(N):
            assert_bit_equal(res[root][2][root], want_red[root], f"reduce root {root} own_stream={own_stream}")


def test_comm_allreduce_host_after_an_aborted_communicator(device):
    """an aborted communicator must not hold up the host pipelines of later ones. A 2-rank LOCAL
    communicator whose rank 1 never calls times out in its host allreduce (rank 0 has queued chunk copies by then);
    then a new 2-rank communicator and a new one-rank communicator run host allreduces, bit-exact against the
    oracle, well inside the old communicator's timeout."""
    import time

    from fmi_amd.comm import Timeout

    uid = unique_id(Transport.LOCAL)
    n, chunk = 5 * 4099 + 3, 4099

    def absent():
        c = Comm(uid, 2, 1, timeout_s=1.0)
        time.sleep(3.0)  # present, but never calls the collective
        c.destroy()

    t = threading.Thread(target=absent)
    c0 = Comm(uid, 2, 0, timeout_s=1.0)
    t.start()
    x = inputs(np.float32, n, 0, seed=5)
    with pytest.raises(Timeout):
        c0.allreduce_host(Op.SUM, x.copy(), np.zeros(n, np.float32), chunk=chunk)
    c0.destroy()
    t.join(timeout=30)
    for N in (2, 1):
        xs = [inputs(np.float32, n, r, seed=70 + N) for r in range(N)]
        t0 = time.monotonic()
        res = run_ranks(N, lambda c, r: _host_allreduce(c, r, xs[r], Op.SUM, False, r == 0, chunk))
        assert time.monotonic() - t0 < 30
        want, _ = orc.allreduce(xs, orc.OPS["sum"])
        for r in range(N):
            assert_bit_equal(res[r][0], want[r], f"after the aborted communicator: N={N} rank {r}")


def test_comm_allreduce_host_default_chunk_matches_device(device):
    """Default chunking (FMI_TUNE_HOST_CHUNK) over a 40 MiB bucket per rank: bit-identical to the device
    allreduce of the whole bucket."""
    N, n = 4, 10 * (1 << 20) + 3
    xs = [inputs(np.float32, n, r, seed=21) for r in range(N)]

    def body(c, r):
        got, _ = _host_allreduce(c, r, xs[r], Op.SUM, False, True, 0)
        s, out = Bucket.from_numpy(xs[r]), Bucket(n, np.float32)
        c.allreduce(Op.SUM, s, out)
        fmi_amd.sync()
        return got, out.numpy()

    for r, (got, dev) in enumerate(run_ranks(N, body)):
        assert_bit_equal(got, dev, f"rank {r}")


@pytest.mark.parametrize("N", [2, 3, 4, 8])
def test_comm_allreduce_direct_windows(device, N):
    """Path DIRECT: every rank's fused kernel reads its shard of all windows in place and the reduced shards
    are gathered from the peers' windows. Bit-exact vs the oracle; windows reused across calls; recv
    aliasing the window; a bucket at an offset inside the window (aligned and unaligned)."""
    for n in (1, 1027, 3 * 65536 + 5):
        for dtype, op in ((np.float32, Op.SUM), (np.int64, Op.PROD), (np.float64, Op.MAX), (np.int32, Op.MIN)):
            xs = [inputs(dtype, n, r, seed=17) for r in range(N)]

            def body(c, r):
                w = c.window(n + 65, dtype)
                out = Bucket(n, dtype)
                res = []
                for off in (0, 64, 1):  # 64 elements keeps 16-B alignment, 1 does not
                    v = w.view(off, n)
                    v.upload(xs[r])
                    for _ in range(2):
                        c.allreduce(op, v, out, path=Path.DIRECT)
                    fmi_amd.sync()
                    res.append((out.numpy(), v.numpy()))
                w.upload(np.concatenate([xs[r], np.zeros(65, dtype)]))
                c.allreduce(op, w.view(0, n), w.view(0, n), path=Path.DIRECT)  # recv aliases the window
                fmi_amd.sync()
                alias = w.view(0, n).numpy()
                c.window_free(w)
                return res, alias

            res = run_ranks(N, body)
            with np.errstate(all="ignore"):
                want, _ = orc.allreduce(xs, orc.OPS[OPNAME[op]])
            for r in range(N):
                for k, (got, sent) in enumerate(res[r][0]):
                    assert_bit_equal(got, want[r], f"N={N} n={n} {op.name} rank {r} case {k}")
                    assert_bit_equal(sent, xs[r], "window bucket untouched")
                assert_bit_equal(res[r][1], want[r], f"N={N} n={n} {op.name} rank {r} aliased")


def test_comm_allreduce_direct_ordered_and_errors(device):
    N, n = 5, 4099
    xs = [inputs(np.float32, n, r, seed=19) for r in range(N)]

    def body(c, r):
        w = c.window(n, np.float32)
        w.upload(xs[r])
        out = Bucket(n, np.float32)
        c.allreduce(Op.SUM, w, out, ordered=True, path=Path.DIRECT)
        fmi_amd.sync()
        with pytest.raises(fmi_amd.FmiError):  # send outside any window
            c.allreduce(Op.SUM, out, out, path=Path.DIRECT)
        got = out.numpy()
        c.window_free(w)
        return got

    res = run_ranks(N, body)
    want, _ = orc.allreduce(xs, orc.op_sum, commutative=False, associative=False)
    for r in range(N):
        assert_bit_equal(res[r], want[r], f"rank {r}")


def test_comm_point_to_point_and_data_movement(device):
    N, n = 4, 1000

    def body(c, r):
        out = {}
        b = Bucket.from_numpy(np.full(n, r, dtype=np.int64))
        c.bcast(b, 2)
        out["bcast"] = b.numpy()
        mine = Bucket.from_numpy(np.arange(n, dtype=np.int64) + 1000 * r)
        allb = Bucket(N * n, np.int64) if r == 1 else None
        c.gather(mine, allb, 1)
        out["gather"] = allb.numpy() if allb is not None else None
        src = Bucket.from_numpy(np.arange(N * n, dtype=np.int64)) if r == 3 else None
        piece = Bucket(n, np.int64)
        c.scatter(src, piece, 3)
        out["scatter"] = piece.numpy()
        ring = Bucket.from_numpy(np.full(n, r, dtype=np.int64))
        got = Bucket(n, np.int64)
        if r % 2 == 0:
            c.send(ring, (r + 1) % N)
            c.recv(got, (r - 1) % N)
        else:
            c.recv(got, (r - 1) % N)
            c.send(ring, (r + 1) % N)
        out["ring"] = got.numpy()
        c.barrier()
        fmi_amd.sync()
        return out

    res = run_ranks(N, body)
    for r in range(N):
        assert np.all(res[r]["bcast"] == 2)
        assert np.array_equal(res[r]["scatter"], np.arange(r * n, (r + 1) * n))
        assert np.all(res[r]["ring"] == (r - 1) % N)
    assert np.array_equal(res[1]["gather"], np.concatenate([np.arange(n) + 1000 * j for j in range(N)]))


def test_comm_rccl_path_needs_rccl_transport(device):
    def body(c, r):
        s, out = Bucket(64, np.float32), Bucket(64, np.float32)
        with pytest.raises(fmi_amd.FmiError):
            c.allreduce(Op.SUM, s, out, path=Path.RCCL)
        return True

    assert all(run_ranks(2, body))


def test_comm_rccl_transport_single_rank(device):
    """RCCL transport plumbing on one GPU (world size 1): id, init, every collective degenerates to a copy."""
    uid = unique_id(Transport.RCCL)
    c = Comm(uid, 1, 0)
    x = inputs(np.float32, 4099, 0)
    s, out = Bucket.from_numpy(x), Bucket(4099, np.float32)
    try:
        for a2a in (0, 1):  # ncclAllToAll / grouped send-recv, ncclAllGather / grouped send-recv
            for gather in (0, 1):
                fmi_amd.tune_set(fmi_amd.Tune.COMM_A2A, a2a)
                fmi_amd.tune_set(fmi_amd.Tune.COMM_GATHER, gather)
                fmi_amd.tune_set(fmi_amd.Tune.COMM_PIPELINE, 4 * a2a)
                for path in (Path.TREE, Path.RCCL):
                    c.allreduce(Op.SUM, s, out, path=path)
                    fmi_amd.sync()
                    assert_bit_equal(out.numpy(), x)
    finally:
        fmi_amd.tune_set(fmi_amd.Tune.COMM_A2A, 0)
        fmi_amd.tune_set(fmi_amd.Tune.COMM_GATHER, 0)
        fmi_amd.tune_set(fmi_amd.Tune.COMM_PIPELINE, 0)
    c.scan(Op.SUM, s, out)
    c.reduce(Op.SUM, s, out, 0)
    c.bcast(out, 0)
    c.barrier()
    fmi_amd.sync()
    assert_bit_equal(out.numpy(), x)
    c.destroy()


@pytest.mark.parametrize("torch_first", [False, True], ids=["system_librccl", "torch_librccl"])
def test_comm_rccl_one_rank_runs_the_full_exchange(device, torch_first):
    """FMI_TUNE_COMM_ONE_RANK_EXCHANGE: a one-rank RCCL communicator (non-blocking init) runs the full sharded
    schedule against itself — ncclAllToAll / grouped send-recv, the shard kernel, ncclAllGather / grouped
    send-recv, ncclReduceScatter (path RCCL), the IPC window exchange (path DIRECT), the second communicator
    of the pipelined allreduce, reduce / reduce_sendbuf / scan, the host pipeline — so a 1-GPU box executes
    the RCCL calls the 8-GPU run makes. Every result is the reference's P = 1 result (a copy of the rank's own
    bucket, PeerToPeer.cpp:96-184 with one peer), bit for bit (tests/_one_rank_worker.py). Run in a child
    process twice: with the system librccl (fmi_amd loaded first) and with torch's (torch imported first, as
    bench.py's N > 1 path does) — the two differ in version (2.27 / 2.26)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-u", "-m", "tests._one_rank_worker"] + (["--torch-first"] if torch_first else []),
                       cwd=root, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0 and "one-rank exchange ok" in r.stdout, (r.stdout[-3000:], r.stderr[-3000:])
    mapped = [l for l in r.stdout.splitlines() if l.startswith("librccl mapped:")][0]
    assert ("torch/lib" in mapped) == torch_first, mapped  # which librccl ran: torch's or the system's


def test_c4_8peer_1gib_allreduce_full_size(device):
    """BASELINE config C4 at full size: 8 peers x 1 GiB f32, sharded allreduce (LOCAL transport on one
    GPU; the RCCL transport runs the same schedule across 8 GPUs). Every rank's 1 GiB result must equal,
    bit for bit, the single-pass fused kernel over the same 8 buckets in allreduce_no_order order, and
    the oracle's simulation of the reference collective on 2^16 sampled indices."""
    from fmi_amd import Alg

    N, n = 8, (1 << 30) // 4
    ins = [Bucket(n, np.float32).fill_synthetic(42, r) for r in range(N)]
    ref = Bucket(n, np.float32)
    fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, ref, ins)
    fmi_amd.sync()
    want_full = ref.numpy()
    ref.free()

    def body(c, r):
        out = Bucket(n, np.float32)
        c.allreduce(Op.SUM, ins[r], out)
        fmi_amd.sync()
        got = out.numpy()
        out.free()
        return bool(np.array_equal(got.view(np.uint32), want_full.view(np.uint32)))

    assert all(run_ranks(N, body))
    idx = np.sort(np.random.default_rng(0).choice(n, size=1 << 16, replace=False)).astype(np.uint64)
    xs = [orc.synthetic_at(np.float32, idx, 42, r) for r in range(N)]
    want, _ = orc.allreduce(xs, orc.op_sum)
    assert_bit_equal(want_full[idx.astype(np.int64)], want[0], "sampled oracle check")
    for b in ins:
        b.free()


def test_c5_host_allreduce_full_size(device, record_property):
    """BASELINE config C5 at its size: 8 LOCAL ranks, each with a 1 GiB f32 bucket in page-locked host memory
    (8 GiB in, 8 GiB out, all through this one GPU), fmi_comm_allreduce_host with the default 64 MiB chunks (H2D,
    sharded allreduce and D2H of successive chunks overlapped). The bucket is halved only if the host's
    MemAvailable cannot hold the 16 GiB of page-locked buckets plus bench.C5_HEADROOM (the size and the limit are
    printed and recorded). Every rank's host result must equal, bit for bit, the single-GPU fused kernel over the
    same 8 buckets (compared in 64 MiB pieces), and the oracle's simulation of the reference's 8-peer allreduce on
    2^16 sampled indices."""
    import bench
    from fmi_amd import Alg, _lib

    N = 8
    avail = bench.mem_available_bytes()
    mib = bench.c5_size_mib(N, 1024, avail)
    record_property("c5_bucket_mib", mib)
    record_property("mem_available_gib", round(avail / 2 ** 30, 1) if avail else None)
    print(f"C5 full size: {N} x {mib} MiB page-locked (MemAvailable {avail and avail / 2 ** 30:.1f} GiB)")
    n = (mib << 20) // 4
    ins = [Bucket(n, np.float32).fill_synthetic(42, r) for r in range(N)]
    ref = Bucket(n, np.float32)
    fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, ref, ins)
    fmi_amd.sync()
    piece = (64 << 20) // 4

    def body(c, r):
        s, out = PinnedArray(n, np.float32), PinnedArray(n, np.float32)
        try:
            _lib.call("fmi_dev_d2h_async", s.ptr, ins[r].ptr, n * 4, None)
            _lib.call("fmi_stream_sync", None)
            out.array[:] = np.float32(np.nan)
            c.allreduce_host(Op.SUM, s.array, out.array)  # chunk 0 = FMI_TUNE_HOST_CHUNK (64 MiB)
            same = True
            for o in range(0, n, piece):
                k = min(piece, n - o)
                same = same and bool(np.array_equal(out.array[o:o + k].view(np.uint32),
                                                    ref.view(o, k).numpy().view(np.uint32)))
            kept = bool(np.array_equal(s.array[:4096], ins[r].view(0, 4096).numpy()))
        finally:
            s.free()
            out.free()
        return same, kept

    res = run_ranks(N, body)
    for r, (same, kept) in enumerate(res):
        assert same, f"rank {r}: host allreduce differs from the single-GPU fused kernel"
        assert kept, f"rank {r}: send host bucket modified"
    idx = np.sort(np.random.default_rng(1).choice(n, size=1 << 16, replace=False)).astype(np.uint64)
    xs = [orc.synthetic_at(np.float32, idx, 42, r) for r in range(N)]
    want, _ = orc.allreduce(xs, orc.op_sum)
    full = ref.numpy()
    assert_bit_equal(full[idx.astype(np.int64)], want[0], "sampled oracle check")
    del full
    ref.free()
    for b in ins:
        b.free()


def test_collectives_on_many_caller_streams():
    """A communicator remembers the tail of every caller stream it queued work on (so destroying an aborted one
    never frees scratch such work may still read); with many short-lived caller streams the drained tails are
    forgotten instead of growing without bound. 100 streams, each used for one allreduce then destroyed; every
    result is the P = 1 allreduce's copy, bit-exact; the communicator is then destroyed cleanly."""
    from fmi_amd import Stream
    from fmi_amd.comm import Comm, Transport, unique_id

    n = 4099
    comm = Comm(unique_id(Transport.LOCAL), 1, 0)
    try:
        src = Bucket.from_numpy(np.arange(n, dtype=np.float32))
        for k in range(100):
            s = Stream()
            dst = Bucket(n, np.float32)
            comm.allreduce(Op.SUM, src, dst, stream=s)
            s.sync()
            assert np.array_equal(dst.numpy(), np.arange(n, dtype=np.float32)), k
            dst.free()
            s.destroy()
        src.free()
    finally:
        comm.destroy()
