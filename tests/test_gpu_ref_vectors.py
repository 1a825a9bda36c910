"""The HIP path against the REFERENCE's own float outputs (tests/golden/ref_vectors.npz: the reference's
src/comm/PeerToPeer.cpp, compiled unmodified and run over an in-memory transport by oracle/_ref — see
tests/golden/make_ref_vectors.py). No restatement in between: the fused P-way kernels (fmi_dev_reduce_tree /
fmi_dev_scan_peers) for every rank and the fixtures' roots, and the sharded communicator (fmi_comm_*, LOCAL
transport: ranks as threads on this GPU) including the sendbuf each peer is left with. f32 (sum, prod, max, min)
and f64 (sum, max), P = 1 .. 9, 12, 13, 16, 17, 24, 31, 32, 33, 48, 64 (f64 to 33); inputs carry signed zeros,
infinities, NaN, subnormals and peers of different magnitudes, so any other bracketing or operand order shows.
Bar: bit-exact (a NaN matches any NaN, see tests/test_gpu_parity.assert_bit_equal).
"""
import os
import threading

import numpy as np
import pytest

import fmi_amd
from fmi_amd import Alg, Bucket, Op
from tests.test_gpu_parity import assert_bit_equal

pytestmark = pytest.mark.gpu

VEC = np.load(os.path.join(os.path.dirname(__file__), "golden", "ref_vectors.npz"))
OP = {"sum": Op.SUM, "prod": Op.PROD, "max": Op.MAX, "min": Op.MIN}
CASES = sorted({tuple(k.split("/")[:3]) for k in VEC.files}, key=lambda c: (c[0], c[1], int(c[2][1:])))


def roots(key):
    return sorted(int(k.split("/")[4][4:]) for k in VEC.files
                  if k.startswith(f"{key}/reduce/root") and k.endswith("/recv"))


@pytest.mark.parametrize("case", CASES, ids=["/".join(c) for c in CASES])
def test_fused_kernels_equal_reference_outputs(device, case):
    key, op, P = "/".join(case), OP[case[1]], int(case[2][1:])
    xs = VEC[f"{key}/in"]
    dtype, n = xs.dtype, xs.shape[1]
    ins = [Bucket.from_numpy(x) for x in xs]
    out = Bucket(n, dtype)
    for r in range(P):
        fmi_amd.reduce_tree(op, Alg.ALLREDUCE, out, ins, rank=r)
        assert_bit_equal(out.numpy(), VEC[f"{key}/allreduce/recv"][r], f"{key} allreduce rank {r}")
    fmi_amd.reduce_tree(op, Alg.REDUCE_LTR, out, ins, rank=0)
    assert_bit_equal(out.numpy(), VEC[f"{key}/allreduce_ltr/recv"][0], f"{key} allreduce (left-to-right)")
    for root in roots(key):
        fmi_amd.reduce_tree(op, Alg.REDUCE, out, ins, rank=root)
        assert_bit_equal(out.numpy(), VEC[f"{key}/reduce/root{root}/recv"], f"{key} reduce root {root}")
        fmi_amd.reduce_tree(op, Alg.REDUCE_LTR, out, ins, rank=root)
        assert_bit_equal(out.numpy(), VEC[f"{key}/reduce_ltr/root{root}/recv"], f"{key} reduce_ltr root {root}")
    outs = [Bucket(n, dtype) for _ in range(P)]
    for alg, name in ((Alg.SCAN, "scan"), (Alg.SCAN_LTR, "scan_ltr")):
        fmi_amd.scan_peers(op, alg, outs, ins)
        for r in range(P):
            assert_bit_equal(outs[r].numpy(), VEC[f"{key}/{name}/recv"][r], f"{key} {name} rank {r}")
    for b in ins + outs + [out]:
        b.free()


COMM_CASES = [c for c in CASES if int(c[2][1:]) in (1, 2, 3, 5, 8, 13)]


@pytest.mark.parametrize("case", COMM_CASES, ids=["/".join(c) for c in COMM_CASES])
def test_communicator_equals_reference_outputs(device, case):
    """fmi_comm_allreduce / _reduce_sendbuf / _scan over P ranks (threads, LOCAL transport): every rank's
    recvbuf, and with sendbuf partials every rank's sendbuf, equal to what the reference leaves each peer."""
    from fmi_amd.comm import Comm, Transport, unique_id

    key, op, P = "/".join(case), OP[case[1]], int(case[2][1:])
    xs = VEC[f"{key}/in"]
    dtype, n = xs.dtype, xs.shape[1]
    rts = roots(key)
    uid = unique_id(Transport.LOCAL)
    res, errors = [None] * P, []

    def rank(r):
        try:
            c = Comm(uid, P, r)
            got = {}
            for name, ordered in (("allreduce", False), ("allreduce_ltr", True)):
                s, o = Bucket.from_numpy(xs[r]), Bucket(n, dtype)
                c.allreduce(op, s, o, ordered=ordered)
                fmi_amd.sync()
                got[name] = o.numpy()
            for name, ordered in (("scan", False), ("scan_ltr", True)):
                s, o = Bucket.from_numpy(xs[r]), Bucket(n, dtype)
                c.scan(op, s, o, ordered=ordered)
                fmi_amd.sync()
                got[name] = o.numpy()
            for root in rts:
                s, o = Bucket.from_numpy(xs[r]), Bucket(n, dtype)
                c.reduce(op, s, o if r == root else None, root, sendbuf_partials=True)
                fmi_amd.sync()
                got[f"reduce/root{root}/send"] = s.numpy()
                if r == root:
                    got[f"reduce/root{root}/recv"] = o.numpy()
                s, o = Bucket.from_numpy(xs[r]), Bucket(n, dtype)
                c.reduce(op, s, o if r == root else None, root, ordered=True)
                fmi_amd.sync()
                if r == root:
                    got[f"reduce_ltr/root{root}/recv"] = o.numpy()
            c.destroy()
            res[r] = got
        except BaseException as e:  # noqa: BLE001 - re-raised below
            errors.append(e)

    threads = [threading.Thread(target=rank, args=(r,)) for r in range(P)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    if errors:
        raise errors[0]
    for r in range(P):
        for name in ("allreduce", "allreduce_ltr", "scan", "scan_ltr"):
            assert_bit_equal(res[r][name], VEC[f"{key}/{name}/recv"][r], f"{key} comm {name} rank {r}")
        for root in rts:
            assert_bit_equal(res[r][f"reduce/root{root}/send"], VEC[f"{key}/reduce/root{root}/send"][r],
                             f"{key} comm reduce root {root}: sendbuf of rank {r}")
    for root in rts:
        assert_bit_equal(res[root][f"reduce/root{root}/recv"], VEC[f"{key}/reduce/root{root}/recv"],
                         f"{key} comm reduce root {root}")
        assert_bit_equal(res[root][f"reduce_ltr/root{root}/recv"], VEC[f"{key}/reduce_ltr/root{root}/recv"],
                         f"{key} comm reduce_ltr root {root}")


def test_empty_buckets_are_no_ops(device):
    """Zero-element buckets, which the reference accepts (Data<std::vector<A>> of size 0: size_in_bytes 0,
    PeerToPeer exchanges empty messages and combines nothing): every P-way entry point and every communicator
    collective returns success and leaves every buffer as it was. Checked against the reference itself where
    oracle/_ref travels with the tree (its allreduce / reduce / scan of empty buckets complete)."""
    from fmi_amd.comm import Comm, Transport, unique_id
    from oracle import fmi_ref as ref

    guard = Bucket(16, np.float32)
    guard.upload(np.arange(16, dtype=np.float32))
    empty = guard.view(0, 0)
    for P in (1, 2, 5, 17, 40):
        ins = [empty] * P
        for alg in (Alg.ALLREDUCE, Alg.REDUCE, Alg.REDUCE_LTR):
            fmi_amd.reduce_tree(Op.SUM, alg, empty, ins, rank=P - 1)
        for alg in (Alg.SCAN, Alg.SCAN_LTR):
            fmi_amd.scan_peers(Op.MAX, alg, [empty] * P, ins)
    fmi_amd.sync()
    assert_bit_equal(guard.numpy(), np.arange(16, dtype=np.float32), "nothing written")
    if ref.available():
        for coll in ("allreduce", "reduce", "scan"):
            recv, send, _ = ref.run(coll, "sum", [np.zeros(0, np.float32)] * 3)
            assert recv.shape == (3, 0) and send.shape == (3, 0)

    N = 3
    uid = unique_id(Transport.LOCAL)
    errors = []

    def rank(r):
        try:
            c = Comm(uid, N, r)
            s, o = Bucket(0, np.float32), Bucket(0, np.float32)
            for ordered in (False, True):
                c.allreduce(Op.SUM, s, o, ordered=ordered)
                c.scan(Op.SUM, s, o, ordered=ordered)
                c.reduce(Op.SUM, s, o if r == 1 else None, 1, ordered=ordered)
            c.reduce(Op.SUM, s, o if r == 1 else None, 1, sendbuf_partials=True)
            fmi_amd.sync()
            c.destroy()
        except BaseException as e:  # noqa: BLE001 - re-raised below
            errors.append(e)

    threads = [threading.Thread(target=rank, args=(r,)) for r in range(N)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=60)
    if errors:
        raise errors[0]
