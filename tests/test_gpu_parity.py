"""Parity of the HIP path (through the C-ABI) against the CPU oracle on the same inputs.

Bar: bit-exact for every op and dtype — integer work trivially, float work because the kernels
evaluate the reference's own bracketing. Comparisons are on raw bits (NaN payloads
and signed zeros included). Sizes: ragged small cases the oracle finishes instantly, the edge values
the reference's element semantics cover, and BASELINE.json's full configs C2 (256 MiB f32 pairwise sum)
and C3 (64 MiB i64 max, 8 × 64 MiB f32 peer scan).
"""
import os

import numpy as np
import pytest

import fmi_amd
from fmi_amd import Alg, Bucket, Op, Tune
from oracle import fmi_oracle as orc

pytestmark = pytest.mark.gpu

DTYPES = [np.float32, np.float64, np.int32, np.int64]
# the other fundamental integer widths (pairwise kernel; P-way programs as pairwise passes)
EXTRA_DTYPES = [np.uint32, np.uint64, np.int8, np.uint8, np.int16, np.uint16]
ALL_DTYPES = DTYPES + EXTRA_DTYPES
OPS = [Op.SUM, Op.PROD, Op.MAX, Op.MIN]
OPNAME = {Op.SUM: "sum", Op.PROD: "prod", Op.MAX: "max", Op.MIN: "min"}
RAGGED = [0, 1, 2, 3, 4, 5, 7, 8, 9, 15, 17, 1027, 4099, 65536 + 3]


UINT = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}


def assert_bit_equal(got, want, what=""):
    """Bit-exact comparison. The one relaxation: a NaN matches any NaN. IEEE leaves the payload/sign of a
    NaN produced by an invalid operation (inf - inf, 0 * inf) to the implementation — x86 SSE returns
    the 'default NaN' 0xFFC00000, CDNA 0x7FC00000 — so NaN-ness, not its bits, is the contract."""
    got, want = np.asarray(got), np.asarray(want)
    assert got.dtype == want.dtype and got.shape == want.shape, what
    u = UINT[got.dtype.itemsize]
    same = got.view(u) == want.view(u)
    if np.issubdtype(got.dtype, np.floating):
        same |= np.isnan(got) & np.isnan(want)
    if not same.all():
        diff = np.nonzero(~same)[0]
        i = diff[0]
        raise AssertionError(f"{what}: {diff.size} mismatching elements, first at {i}: got {got[i]!r} "
                             f"want {want[i]!r}")


def inputs(dtype, n, peer, seed=42):
    """Synthetic bucket, with edge values sprinkled in for the element semantics."""
    x = orc.synthetic(dtype, n, seed=seed, peer=peer)
    if n >= 8:
        if np.issubdtype(dtype, np.floating):
            edge = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, np.finfo(dtype).tiny / 4, -np.finfo(dtype).max,
                             np.finfo(dtype).smallest_subnormal], dtype=dtype)
        elif np.issubdtype(dtype, np.signedinteger):
            info = np.iinfo(dtype)
            edge = np.array([info.min, info.max, 0, -1, 1, info.min + 1, info.max - 1, 2], dtype=dtype)
        else:
            info = np.iinfo(dtype)
            edge = np.array([0, info.max, 1, info.max - 1, 2, info.max // 2, info.max // 2 + 1, 3], dtype=dtype)
        idx = (np.arange(8) * 7919 + peer * 13) % n
        x[idx] = np.roll(edge, peer)
    return x


def dev(arr):
    return Bucket.from_numpy(arr)


# ------------------------------------------------------------------------------------------------
# pairwise combine — the hot path (reference include/Communicator.h:180-189)
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("dtype", ALL_DTYPES, ids=lambda d: np.dtype(d).name)
@pytest.mark.parametrize("op", OPS, ids=lambda o: o.name)
def test_reduce_pair_ragged(device, op, dtype):
    for n in RAGGED:
        a, b = inputs(dtype, n, 0), inputs(dtype, n, 1)
        da, db = dev(a), dev(b)
        fmi_amd.reduce_pair(op, da, db)
        with np.errstate(all="ignore"):
            want = orc.pairwise(OPNAME[op], a, b)
        assert_bit_equal(da.numpy(), want, f"{op.name} {np.dtype(dtype).name} n={n}")
        assert_bit_equal(db.numpy(), b, "in operand must stay untouched")


@pytest.mark.parametrize("dtype", ALL_DTYPES, ids=lambda d: np.dtype(d).name)
def test_reduce_pair_unaligned_views(device, dtype):
    n = 4099
    a, b = inputs(dtype, n + 8, 0), inputs(dtype, n + 8, 1)
    for off_a, off_b in [(1, 1), (1, 2), (3, 0), (0, 5)]:
        da, db = dev(a), dev(b)
        va, vb = da.view(off_a, n), db.view(off_b, n)
        fmi_amd.reduce_pair(Op.SUM, va, vb)
        with np.errstate(all="ignore"):
            want = a.copy()
            want[off_a:off_a + n] = orc.pairwise("sum", a[off_a:off_a + n], b[off_b:off_b + n])
        assert_bit_equal(da.numpy(), want, f"offsets {off_a},{off_b}")


def test_reduce_pair_inplace_alias(device):
    a = inputs(np.float32, 10007, 0)
    da = dev(a)
    fmi_amd.reduce_pair(Op.SUM, da, da)
    with np.errstate(all="ignore"):
        assert_bit_equal(da.numpy(), a + a)


@pytest.mark.parametrize("variant,unroll,block", [(v, u, b) for v in (0, 1, 2, 3, 4) for u in (1, 2, 4, 8)
                                                  for b in (256, 1024)])
def test_reduce_pair_every_launch_variant(device, variant, unroll, block):
    n = (1 << 20) + 3
    a, b = inputs(np.float32, n, 0), inputs(np.float32, n, 1)
    old = {k: fmi_amd.tune_get(k) for k in (Tune.PAIR_VARIANT, Tune.PAIR_UNROLL, Tune.BLOCK)}
    try:
        fmi_amd.tune_set(Tune.PAIR_VARIANT, variant)
        fmi_amd.tune_set(Tune.PAIR_UNROLL, unroll)
        fmi_amd.tune_set(Tune.BLOCK, block)
        da, db = dev(a), dev(b)
        fmi_amd.reduce_pair(Op.SUM, da, db)
        assert_bit_equal(da.numpy(), a + b)
    finally:
        for k, v in old.items():
            fmi_amd.tune_set(k, v)


@pytest.mark.parametrize("dtype", [np.float32, np.int64, np.int8], ids=lambda d: np.dtype(d).name)
@pytest.mark.parametrize("sc1_of_8", [0, 1, 3, 8])
def test_reduce_pair_sc1_tiles_keep_bits(device, dtype, sc1_of_8):
    """FMI_TUNE_PAIR_SC1_OF_8 picks which tiles of a launch store with sc1 (t % 8 < k: none, 1, 3 or all 8 of
    every 8); the ragged last tile and the < 16-B tail included. Every choice gives the oracle's bits, with the
    launch shapes that honour it (one-shot tiles at unroll 1 / 4, 256 / 1024 threads)."""
    n = 12 * 4096 * 16 // np.dtype(dtype).itemsize + 4099  # 49 tiles of 16 KiB at unroll 4, ragged end
    a, b = inputs(dtype, n, 0), inputs(dtype, n, 1)
    with np.errstate(all="ignore"):
        want = orc.pairwise("max" if dtype == np.int64 else "sum", a, b)
    keys = (Tune.PAIR_SC1_OF_8, Tune.PAIR_UNROLL, Tune.BLOCK)
    old = {k: fmi_amd.tune_get(k) for k in keys}
    try:
        fmi_amd.tune_set(Tune.PAIR_SC1_OF_8, sc1_of_8)
        for unroll, block in [(4, 256), (1, 256), (4, 1024)]:
            fmi_amd.tune_set(Tune.PAIR_UNROLL, unroll)
            fmi_amd.tune_set(Tune.BLOCK, block)
            da, db = dev(a), dev(b)
            fmi_amd.reduce_pair(Op.MAX if dtype == np.int64 else Op.SUM, da, db)
            assert_bit_equal(da.numpy(), want, f"sc1 {sc1_of_8} of 8, unroll {unroll}, block {block}")
    finally:
        for k, v in old.items():
            fmi_amd.tune_set(k, v)


@pytest.mark.parametrize("nbytes", [16, 262143, 262144, 262144 + 5, (1 << 20) + 16 * 1024 + 3, 64 << 20])
def test_device_copy_bits(device, nbytes):
    """fmi_dev_d2d_async / the communicator's staging copies (device_copy): the copy_tile kernel for aligned
    device buckets of >= 256 KiB (whole tiles, a partial tile, a sub-16-B tail), hipMemcpyAsync below that,
    for unaligned views and for host (page-locked) memory: every byte, and nothing past the end."""
    rng = np.random.default_rng(nbytes)
    data = rng.integers(0, 256, nbytes, dtype=np.uint8)
    src = Bucket.from_numpy(data)
    dst = Bucket(nbytes + 64, np.uint8)
    dst.upload(np.full(nbytes + 64, 0xA5, np.uint8))
    dst.view(0, nbytes).copy_from(src)
    fmi_amd.sync()
    got = dst.numpy()
    assert np.array_equal(got[:nbytes], data) and np.all(got[nbytes:] == 0xA5)
    if nbytes >= 262144:  # unaligned destination: the hipMemcpyAsync path, same bytes
        dst.upload(np.full(nbytes + 64, 0xA5, np.uint8))
        dst.view(3, nbytes).copy_from(src)
        fmi_amd.sync()
        got = dst.numpy()
        assert np.array_equal(got[3:3 + nbytes], data) and np.all(got[:3] == 0xA5) and np.all(got[3 + nbytes:] == 0xA5)
    src.free()
    dst.free()


def test_one_rank_allreduce_is_a_copy(device):
    """The reference's P = 1 allreduce (PeerToPeer.cpp:96-130 with one peer) leaves recvbuf = sendbuf: the
    one-rank communicator's copy (device_copy kernel for 16-B aligned device buckets), bit for bit."""
    from fmi_amd.comm import Comm, Transport, unique_id

    c = Comm(unique_id(Transport.LOCAL), 1, 0)
    for n in (1, 65536 + 7, (16 << 20) + 3):
        x = inputs(np.float32, n, 0, seed=61)
        s, o = Bucket.from_numpy(x), Bucket(n, np.float32)
        c.allreduce(fmi_amd.Op.SUM, s, o)
        fmi_amd.sync()
        assert_bit_equal(o.numpy(), x, f"n={n}")
        s.free()
        o.free()
    c.destroy()


def test_combine_out_of_place(device):
    a, b = inputs(np.int64, 5003, 0), inputs(np.int64, 5003, 1)
    out = Bucket(5003, np.int64)
    fmi_amd.combine(Op.MAX, out, dev(a), dev(b))
    assert_bit_equal(out.numpy(), orc.op_max(a, b))


def test_stream_wait_event_orders_cross_stream_work(device):
    """A combine on a side stream feeding a copy on the library stream (fmi_stream_wait_event): the copy
    must see the combined bucket. 64 MiB so the combine is still running when the copy is enqueued."""
    n = 16 << 20
    a, b = Bucket(n, np.float32).fill_synthetic(3, 0), Bucket(n, np.float32).fill_synthetic(3, 1)
    want = Bucket(n, np.float32)
    fmi_amd.combine(Op.SUM, want, a, b)
    fmi_amd.sync()
    side, done = fmi_amd.Stream(), fmi_amd.Event()
    out = Bucket(n, np.float32)
    fmi_amd.reduce_pair(Op.SUM, a, b, stream=side)
    done.record(side)
    done.wait_on(None)
    out.copy_from(a)
    fmi_amd.sync()
    assert_bit_equal(out.numpy(), want.numpy())
    side.destroy()
    done.destroy()


def test_synthetic_matches_host_generator(device):
    for dtype in ALL_DTYPES:
        for peer in (0, 1, 7):
            n = 100003
            d = Bucket(n, dtype).fill_synthetic(42, peer)
            assert_bit_equal(d.numpy(), orc.synthetic(dtype, n, seed=42, peer=peer), np.dtype(dtype).name)


# ------------------------------------------------------------------------------------------------
# P-way fused kernels vs the oracle's simulation of the reference collectives
# ------------------------------------------------------------------------------------------------
PEERS = list(range(1, 17)) + [17, 20, 24, 31, 32, 33, 48, 64]


def _peer_inputs(dtype, n, P, seed=7):
    return [inputs(dtype, n, p, seed=seed) for p in range(P)]


@pytest.mark.parametrize("P", PEERS)
def test_allreduce_tree_all_ranks(device, P):
    n = 1027
    for dtype in DTYPES:
        xs = _peer_inputs(dtype, n, P)
        ins = [dev(x) for x in xs]
        for op in OPS:
            with np.errstate(all="ignore"):
                want, _ = orc.allreduce(xs, orc.OPS[OPNAME[op]])
            for rank in sorted({0, P // 2, P - 1}):
                out = Bucket(n, dtype)
                fmi_amd.reduce_tree(op, Alg.ALLREDUCE, out, ins, rank=rank)
                assert_bit_equal(out.numpy(), want[rank], f"P={P} {op.name} {np.dtype(dtype).name} rank {rank}")


@pytest.mark.parametrize("P", PEERS)
def test_reduce_tree_roots(device, P):
    n = 1029
    for dtype in (np.float32, np.int64):
        xs = _peer_inputs(dtype, n, P)
        ins = [dev(x) for x in xs]
        for op in OPS:
            for root in sorted({0, 1 % P, P - 1}):
                with np.errstate(all="ignore"):
                    want, _ = orc.reduce(xs, orc.OPS[OPNAME[op]], root=root)
                out = Bucket(n, dtype)
                fmi_amd.reduce_tree(op, Alg.REDUCE, out, ins, rank=root)
                assert_bit_equal(out.numpy(), want, f"P={P} {op.name} root {root}")


@pytest.mark.parametrize("P", PEERS)
def test_reduce_ltr(device, P):
    n = 515
    xs = _peer_inputs(np.float32, n, P)
    ins = [dev(x) for x in xs]
    for op in OPS:
        with np.errstate(all="ignore"):
            want, _ = orc.reduce(xs, orc.OPS[OPNAME[op]], root=0, commutative=False, associative=False)
        out = Bucket(n, np.float32)
        fmi_amd.reduce_tree(op, Alg.REDUCE_LTR, out, ins, rank=P - 1)
        assert_bit_equal(out.numpy(), want, f"P={P} {op.name}")


@pytest.mark.parametrize("P", PEERS)
def test_scan_peers(device, P):
    n = 1031
    for dtype in DTYPES:
        xs = _peer_inputs(dtype, n, P)
        ins = [dev(x) for x in xs]
        for op in OPS:
            for alg, ordered in ((Alg.SCAN, False), (Alg.SCAN_LTR, True)):
                with np.errstate(all="ignore"):
                    want, _ = orc.scan(xs, orc.OPS[OPNAME[op]], commutative=not ordered, associative=not ordered)
                outs = [Bucket(n, dtype) for _ in range(P)]
                fmi_amd.scan_peers(op, alg, outs, ins)
                for k in range(P):
                    assert_bit_equal(outs[k].numpy(), want[k], f"P={P} {alg.name} {op.name} peer {k}")


@pytest.mark.parametrize("P", [100, 256])
def test_many_peers_blocked_programs(device, P):
    """Beyond 64 peers, up to the 256 cap: two levels of 16-peer blocks (P = 256) and ragged blocks
    (P = 100), every algorithm, aligned (fused blocks) and unaligned (pairwise passes) buckets."""
    n = 515
    for dtype, op in ((np.float32, Op.SUM), (np.int64, Op.MAX), (np.float64, Op.MIN)):
        xs = _peer_inputs(dtype, n + 1, P, seed=23)
        big = [dev(x) for x in xs]
        for ins, sl, what in (([b.view(0, n) for b in big], slice(0, n), "aligned"),
                              ([b.view(1, n) for b in big], slice(1, n + 1), "unaligned")):
            ys = [x[sl] for x in xs]
            fn = orc.OPS[OPNAME[op]]
            with np.errstate(all="ignore"):
                want, _ = orc.allreduce(ys, fn)
                for rank in (0, P // 2 + 3, P - 1):
                    out = Bucket(n, dtype)
                    fmi_amd.reduce_tree(op, Alg.ALLREDUCE, out, ins, rank=rank)
                    assert_bit_equal(out.numpy(), want[rank], f"{what} allreduce P={P} rank {rank}")
                for root in (0, 37):
                    want, _ = orc.reduce(ys, fn, root=root)
                    out = Bucket(n, dtype)
                    fmi_amd.reduce_tree(op, Alg.REDUCE, out, ins, rank=root)
                    assert_bit_equal(out.numpy(), want, f"{what} reduce P={P} root {root}")
                want, _ = orc.reduce(ys, fn, root=0, commutative=False, associative=False)
                out = Bucket(n, dtype)
                fmi_amd.reduce_tree(op, Alg.REDUCE_LTR, out, ins)
                assert_bit_equal(out.numpy(), want, f"{what} reduce_ltr P={P}")
                for alg, ordered in ((Alg.SCAN, False), (Alg.SCAN_LTR, True)):
                    want, _ = orc.scan(ys, fn, commutative=not ordered, associative=not ordered)
                    outs = [Bucket(n, dtype) for _ in range(P)]
                    fmi_amd.scan_peers(op, alg, outs, ins)
                    for k in range(P):
                        assert_bit_equal(outs[k].numpy(), want[k], f"{what} {alg.name} P={P} peer {k}")


@pytest.mark.parametrize("P", [257, 512, 1000])
def test_beyond_256_peers(device, P):
    """No peer cap, as in the reference (src/comm/PeerToPeer.cpp:59-184 take any num_peers): P = 257, 512,
    1000 — three levels of 16-peer blocks, ragged blocks — every algorithm, every rank kind, aligned (fused
    blocks) and unaligned (pairwise passes over run-time-sized programs) buckets, bit-exact vs the oracle."""
    n = 131
    for dtype, op in ((np.float32, Op.SUM), (np.int64, Op.MAX)):
        xs = _peer_inputs(dtype, n + 1, P, seed=41)
        big = [dev(x) for x in xs]
        fn = orc.OPS[OPNAME[op]]
        for ins, sl, what in (([b.view(0, n) for b in big], slice(0, n), "aligned"),
                              ([b.view(1, n) for b in big], slice(1, n + 1), "unaligned")):
            ys = [x[sl] for x in xs]
            with np.errstate(all="ignore"):
                want, _ = orc.allreduce(ys, fn)
                for rank in (0, 257 % P, P - 1):
                    out = Bucket(n, dtype)
                    fmi_amd.reduce_tree(op, Alg.ALLREDUCE, out, ins, rank=rank)
                    assert_bit_equal(out.numpy(), want[rank], f"{what} allreduce P={P} rank {rank}")
                for root in (0, P - 3):
                    want, _ = orc.reduce(ys, fn, root=root)
                    out = Bucket(n, dtype)
                    fmi_amd.reduce_tree(op, Alg.REDUCE, out, ins, rank=root)
                    assert_bit_equal(out.numpy(), want, f"{what} reduce P={P} root {root}")
                want, _ = orc.reduce(ys, fn, root=0, commutative=False, associative=False)
                out = Bucket(n, dtype)
                fmi_amd.reduce_tree(op, Alg.REDUCE_LTR, out, ins)
                assert_bit_equal(out.numpy(), want, f"{what} reduce_ltr P={P}")
                for alg, ordered in ((Alg.SCAN, False), (Alg.SCAN_LTR, True)):
                    want, _ = orc.scan(ys, fn, commutative=not ordered, associative=not ordered)
                    outs = [Bucket(n, dtype) for _ in range(P)]
                    fmi_amd.scan_peers(op, alg, outs, ins)
                    for k in range(P):
                        assert_bit_equal(outs[k].numpy(), want[k], f"{what} {alg.name} P={P} peer {k}")


_FIRST_CALL = """
import numpy as np, fmi_amd
from fmi_amd import Alg, Bucket, Op
from oracle import fmi_oracle as orc
from tests.test_gpu_parity import assert_bit_equal, inputs
fmi_amd.init(0)
P, n = 17, 1031
xs = [inputs(np.float32, n, p, seed=7) for p in range(P)]
ins = [Bucket.from_numpy(x) for x in xs]
outs = [Bucket(n, np.float32) for _ in range(P)]
fmi_amd.scan_peers(Op.SUM, Alg.SCAN, outs, ins)   # needs no scratch at all
want, _ = orc.scan(xs, orc.op_sum)
for k in range(P):
    assert_bit_equal(outs[k].numpy(), want[k], f"peer {k}")
print("ok")
"""


def test_blocked_program_as_first_call_of_a_process(device):
    """A blocked program that needs no temporaries, before anything has sized the scratch arena."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _FIRST_CALL], cwd=root, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]


@pytest.mark.parametrize("cap", [0, 4, 32, 96, 256])
def test_fused_occupancy_cap_keeps_bits(device, cap):
    """FMI_TUNE_FUSED_INFLIGHT_KIB only reserves LDS to cap residency: results stay bit-exact (multi-wave
    grids, ragged tail)."""
    P, n = 8, (1 << 20) + 5
    xs = _peer_inputs(np.float32, n, P)
    ins = [dev(x) for x in xs]
    want_ar, _ = orc.allreduce(xs, orc.op_sum)
    want_sc, _ = orc.scan(xs, orc.op_sum)
    old = fmi_amd.tune_get(Tune.FUSED_INFLIGHT_KIB)
    try:
        fmi_amd.tune_set(Tune.FUSED_INFLIGHT_KIB, cap)
        out = Bucket(n, np.float32)
        fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, out, ins)
        assert_bit_equal(out.numpy(), want_ar[0], f"allreduce cap {cap}")
        outs = [Bucket(n, np.float32) for _ in range(P)]
        fmi_amd.scan_peers(Op.SUM, Alg.SCAN, outs, ins)
        for k in range(P):
            assert_bit_equal(outs[k].numpy(), want_sc[k], f"scan cap {cap} peer {k}")
    finally:
        fmi_amd.tune_set(Tune.FUSED_INFLIGHT_KIB, old)


@pytest.mark.parametrize("pol", [0, 2], ids=["global_nt", "buffer_sc1"])
def test_fused_access_policy_keeps_bits(device, pol):
    """FMI_TUNE_FUSED_POLICY forced to each access form for every peer count (the default picks per kernel):
    the fused tree and scan kernels, every algorithm, four dtypes and all four ops, ragged n (tail lanes) and
    a grid-stride size, against the oracle."""
    old = fmi_amd.tune_get(Tune.FUSED_POLICY)
    try:
        fmi_amd.tune_set(Tune.FUSED_POLICY, pol)
        for dtype, n in ((np.float32, 4099 * 4 + 3), (np.int64, 65536 * 3 + 1), (np.uint8, 1 << 16), (np.float64, 1027)):
            for P in (2, 3, 4, 8, 16):
                xs = _peer_inputs(dtype, n, P)
                ins = [dev(x) for x in xs]
                for op in OPS:
                    f = orc.OPS[OPNAME[op]]
                    with np.errstate(all="ignore"):
                        want_ar, _ = orc.allreduce(xs, f)
                        want_rd, _ = orc.reduce(xs, f, root=0)
                        want_sc, _ = orc.scan(xs, f)
                    out = Bucket(n, dtype)
                    fmi_amd.reduce_tree(op, Alg.ALLREDUCE, out, ins, rank=P - 1)
                    assert_bit_equal(out.numpy(), want_ar[P - 1], f"pol {pol} allreduce {op.name} P={P}")
                    fmi_amd.reduce_tree(op, Alg.REDUCE, out, ins)
                    assert_bit_equal(out.numpy(), want_rd, f"pol {pol} reduce {op.name} P={P}")
                    outs = [Bucket(n, dtype) for _ in range(P)]
                    fmi_amd.scan_peers(op, Alg.SCAN, outs, ins)
                    for k in range(P):
                        assert_bit_equal(outs[k].numpy(), want_sc[k], f"pol {pol} scan {op.name} P={P} peer {k}")
    finally:
        fmi_amd.tune_set(Tune.FUSED_POLICY, old)


@pytest.mark.parametrize("dtype", EXTRA_DTYPES, ids=lambda d: np.dtype(d).name)
def test_extra_dtypes_p_way_programs(device, dtype):
    """The other integer widths through every P-way entry point (pairwise passes in the reference's order),
    P covering the fused range and beyond, against the oracle's message simulation."""
    n = 1029
    for P in (3, 8, 17, 33):
        xs = _peer_inputs(dtype, n, P)
        ins = [dev(x) for x in xs]
        for op in OPS:
            f = orc.OPS[OPNAME[op]]
            with np.errstate(all="ignore"):
                want_ar, _ = orc.allreduce(xs, f)
                want_red, _ = orc.reduce(xs, f, root=1)
                want_sc, _ = orc.scan(xs, f)
                want_ltr, _ = orc.scan(xs, f, commutative=False, associative=False)
            out = Bucket(n, dtype)
            fmi_amd.reduce_tree(op, Alg.ALLREDUCE, out, ins, rank=P - 1)
            assert_bit_equal(out.numpy(), want_ar[P - 1], f"allreduce P={P} {op.name}")
            fmi_amd.reduce_tree(op, Alg.REDUCE, out, ins, rank=1)
            assert_bit_equal(out.numpy(), want_red, f"reduce P={P} {op.name}")
            for alg, want in ((Alg.SCAN, want_sc), (Alg.SCAN_LTR, want_ltr)):
                outs = [Bucket(n, dtype) for _ in range(P)]
                fmi_amd.scan_peers(op, alg, outs, ins)
                for k in range(P):
                    assert_bit_equal(outs[k].numpy(), want[k], f"{alg.name} P={P} {op.name} peer {k}")


@pytest.mark.parametrize("P", [32, 37, 48, 64, 79, 100, 128])
def test_one_pass_blocked_scan_matches_blocked_launches(device, P):
    """scan_no_order over 32..143 peers: the one-pass kernel (fmi_fused_scan_blocked.hip, every input read
    once) and the blocked launches (FMI_TUNE_BLOCKS_ONE_PASS = 0) give the oracle's bits, every op x core
    dtype, a multi-wave grid with a ragged tail, full and ragged last blocks."""
    n = 3 * 4096 + 5
    old = fmi_amd.tune_get(Tune.BLOCKS_ONE_PASS)
    try:
        for dtype in DTYPES:
            xs = _peer_inputs(dtype, n, P, seed=11)
            ins = [dev(x) for x in xs]
            for op in OPS:
                with np.errstate(all="ignore"):
                    want, _ = orc.scan(xs, orc.OPS[OPNAME[op]])
                for one_pass in (1, 0):
                    fmi_amd.tune_set(Tune.BLOCKS_ONE_PASS, one_pass)
                    outs = [Bucket(n, dtype) for _ in range(P)]
                    fmi_amd.scan_peers(op, Alg.SCAN, outs, ins)
                    for k in range(P):
                        assert_bit_equal(outs[k].numpy(), want[k],
                                         f"P={P} {np.dtype(dtype).name} {op.name} one_pass={one_pass} peer {k}")
    finally:
        fmi_amd.tune_set(Tune.BLOCKS_ONE_PASS, old)


@pytest.mark.parametrize("P", [17, 32, 37, 64, 100, 128, 129, 255, 300])
def test_one_pass_chain_matches_blocked_launches(device, P):
    """scan_ltr (32..128 peers) and reduce_ltr (17..128): the one-pass chain kernel (fmi_fused_chain.hip) and the
    blocked launches give the oracle's left-to-right bits, every op x core dtype, ragged peer blocks, in place.
    Beyond 128 peers the chain runs in segments of 127 continued from the previous running value
    (chain_superblocks)."""
    n = 2 * 4096 + 7
    old = fmi_amd.tune_get(Tune.BLOCKS_ONE_PASS)
    try:
        for dtype in DTYPES:
            xs = _peer_inputs(dtype, n, P, seed=17)
            ins = [dev(x) for x in xs]
            for op in OPS:
                f = orc.OPS[OPNAME[op]]
                with np.errstate(all="ignore"):
                    want_scan, _ = orc.scan(xs, f, commutative=False, associative=False)
                    want_red, _ = orc.reduce(xs, f, root=0, commutative=False, associative=False)
                for one_pass in (1, 0):
                    fmi_amd.tune_set(Tune.BLOCKS_ONE_PASS, one_pass)
                    what = f"P={P} {np.dtype(dtype).name} {op.name} one_pass={one_pass}"
                    out = Bucket(n, dtype)
                    fmi_amd.reduce_tree(op, Alg.REDUCE_LTR, out, ins, rank=P - 1)
                    assert_bit_equal(out.numpy(), want_red, f"reduce_ltr {what}")
                    if P > 31:
                        outs = [Bucket(n, dtype) for _ in range(P)]
                        fmi_amd.scan_peers(op, Alg.SCAN_LTR, outs, ins)
                        for k in range(P):
                            assert_bit_equal(outs[k].numpy(), want_scan[k], f"scan_ltr {what} peer {k}")
            if dtype == np.float32:  # in place
                for one_pass in (1, 0):
                    fmi_amd.tune_set(Tune.BLOCKS_ONE_PASS, one_pass)
                    bufs = [dev(x) for x in xs]
                    fmi_amd.scan_peers(Op.SUM, Alg.SCAN_LTR, bufs, bufs)
                    want, _ = orc.scan(xs, orc.op_sum, commutative=False, associative=False)
                    for k in range(P):
                        assert_bit_equal(bufs[k].numpy(), want[k], f"scan_ltr in place one_pass={one_pass} peer {k}")
    finally:
        fmi_amd.tune_set(Tune.BLOCKS_ONE_PASS, old)


@pytest.mark.parametrize("P", [17, 32, 33, 48, 64, 80, 100, 112, 128, 129, 256, 300, 512])
def test_one_pass_blocked_tree_matches_blocked_launches(device, P):
    """reduce over 17..128 peers (ragged last blocks at 17, 33, 100) and allreduce over 32..128 peers (pre-fold of
    full blocks at 48, 80, 112; other P take the launches): the one-pass kernels (fmi_fused_tree_blocked.hip) and
    the blocked launches (FMI_TUNE_BLOCKS_ONE_PASS = 0) give the oracle's bits for every op x core dtype, several
    roots / ranks, and in place (out = an input). Beyond 128 peers reduce runs as superblocks of 128
    (reduce_superblocks: 129 with a lone last peer, 256, 300, 512), allreduce over 2^k peers as superblocks
    of 64 (allreduce_superblocks: 256, 512; other P the block launches)."""
    n = 2 * 4096 + 3
    old = fmi_amd.tune_get(Tune.BLOCKS_ONE_PASS)
    try:
        for dtype in DTYPES:
            xs = _peer_inputs(dtype, n, P, seed=13)
            ins = [dev(x) for x in xs]
            for op in OPS:
                f = orc.OPS[OPNAME[op]]
                with np.errstate(all="ignore"):
                    want_ar, _ = orc.allreduce(xs, f)
                    want_red = {root: orc.reduce(xs, f, root=root)[0] for root in (0, 5)}
                for one_pass in (1, 0):
                    fmi_amd.tune_set(Tune.BLOCKS_ONE_PASS, one_pass)
                    what = f"P={P} {np.dtype(dtype).name} {op.name} one_pass={one_pass}"
                    out = Bucket(n, dtype)
                    for root in (0, 5):
                        fmi_amd.reduce_tree(op, Alg.REDUCE, out, ins, rank=root)
                        assert_bit_equal(out.numpy(), want_red[root], f"reduce root {root} {what}")
                    pow2 = 1 << (P.bit_length() - 1)
                    # float max / min: each rank keeps its own operand order; folded ranks >= 2^k get their
                    # partner's value
                    for rank in sorted(r for r in {0, 17, pow2 - 1, P - 1, min(pow2 + 3, P - 1)} if r < P):
                        fmi_amd.reduce_tree(op, Alg.ALLREDUCE, out, ins, rank=rank)
                        assert_bit_equal(out.numpy(), want_ar[rank], f"allreduce rank {rank} {what}")
                    acc = [dev(x) for x in xs[:1]] + ins[1:]  # in place: out is peer 0's bucket
                    fmi_amd.reduce_tree(op, Alg.ALLREDUCE, acc[0], acc, rank=0)
                    assert_bit_equal(acc[0].numpy(), want_ar[0], f"allreduce in place {what}")
    finally:
        fmi_amd.tune_set(Tune.BLOCKS_ONE_PASS, old)


@pytest.mark.parametrize("P", [8, 40, 64, 100])
def test_scan_in_place(device, P):
    """outs == ins: beyond 16 peers the blocked scan writes block prefixes into outputs whose inputs the
    later passes must no longer read."""
    n = 4096
    xs = _peer_inputs(np.float32, n, P)
    for alg, ordered in ((Alg.SCAN, False), (Alg.SCAN_LTR, True)):
        bufs = [dev(x) for x in xs]
        want, _ = orc.scan(xs, orc.op_sum, commutative=not ordered, associative=not ordered)
        fmi_amd.scan_peers(Op.SUM, alg, bufs, bufs)
        for k in range(P):
            assert_bit_equal(bufs[k].numpy(), want[k], f"{alg.name} peer {k}")


@pytest.mark.parametrize("P", [5, 40])
def test_tree_unaligned_falls_back_with_same_order(device, P):
    """Unaligned views run the pairwise-pass program (only the steps the rank's result depends on)."""
    n = 1000
    xs = _peer_inputs(np.float32, n + 1, P)
    big = [dev(x) for x in xs]
    ins = [b.view(1, n) for b in big]
    with np.errstate(all="ignore"):
        want, _ = orc.allreduce([x[1:] for x in xs], orc.op_max)
    for rank in (0, P // 2 + 1, P - 1):
        out = Bucket(n, np.float32)
        fmi_amd.reduce_tree(Op.MAX, Alg.ALLREDUCE, out, ins, rank=rank)
        assert_bit_equal(out.numpy(), want[rank], f"rank {rank}")


def test_signed_zero_max_follows_each_ranks_operand_order(device):
    # Float max on ties depends on operand order; each rank's allreduce result must be its own.
    P, n = 4, 64
    xs = [np.full(n, (-0.0 if p % 2 else 0.0), dtype=np.float32) for p in range(P)]
    ins = [dev(x) for x in xs]
    want, _ = orc.allreduce(xs, orc.op_max)
    for r in range(P):
        out = Bucket(n, np.float32)
        fmi_amd.reduce_tree(Op.MAX, Alg.ALLREDUCE, out, ins, rank=r)
        assert_bit_equal(out.numpy(), want[r], f"rank {r}")


@pytest.mark.parametrize("P", [32, 48, 64, 96, 128])
def test_one_pass_blocked_allreduce_keeps_each_ranks_operand_order(device, P):
    """Float max / min over ±0 ties beyond 31 peers: the one-pass blocked kernel keeps block rank r % 16 and
    block-level rank r / 16, so every rank gets its own reference bits (data chosen so that ranks differ)."""
    n = 4096 + 3
    rng = np.random.default_rng(P)
    xs = [np.where(rng.random(n) < 0.5, -0.0, 0.0).astype(np.float32) for _ in range(P)]
    ins = [dev(x) for x in xs]
    for op in (Op.MAX, Op.MIN):
        want, _ = orc.allreduce(xs, orc.OPS[OPNAME[op]])
        ranks = list(range(P)) if P <= 32 else [0, 1, 15, 16, 17, 31, 33, P // 2 + 5, P - 2, P - 1]
        assert any(not np.array_equal(want[0].view(np.uint32), want[r].view(np.uint32)) for r in ranks)
        for r in ranks:
            out = Bucket(n, np.float32)
            fmi_amd.reduce_tree(op, Alg.ALLREDUCE, out, ins, rank=r)
            assert_bit_equal(out.numpy(), want[r], f"P={P} {op.name} rank {r}")


def test_float_sum_tolerance_against_sequential_order(device):
    """The stated float tolerance for orders that differ from the reference's (e.g. RCCL's):
    |y - y_ref| <= (P-1) * u * sum|x_i|, u = 2^-24. Our tree result is exact;
    a sequential fold stays inside the bound."""
    P, n = 8, 1 << 16
    xs = _peer_inputs(np.float32, n, P, seed=1234)
    xs = [np.nan_to_num(x, nan=0.0, posinf=0.0, neginf=0.0) for x in xs]
    xs = [np.where(np.abs(x) > 1e30, 0, x).astype(np.float32) for x in xs]
    out = Bucket(n, np.float32)
    fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, out, [dev(x) for x in xs])
    y = out.numpy()
    seq = xs[0].copy()
    for x in xs[1:]:
        seq = seq + x
    bound = (P - 1) * 2.0 ** -24 * np.sum(np.abs(np.stack(xs).astype(np.float64)), axis=0)
    assert np.all(np.abs(y.astype(np.float64) - seq.astype(np.float64)) <= bound)


# ------------------------------------------------------------------------------------------------
# host-ingress pipeline (recv buffers in host memory)
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("n", [1, 1000, (1 << 20) + 5])
def test_host_reduce_pair(device, n):
    old = fmi_amd.tune_get(Tune.HOST_CHUNK)
    try:
        fmi_amd.tune_set(Tune.HOST_CHUNK, 1 << 16)  # many chunks: exercises both pipeline slots
        for dtype in (np.float32, np.int64):
            a, b = inputs(dtype, n, 0), inputs(dtype, n, 1)
            x = a.copy()
            fmi_amd.host_reduce_pair(Op.SUM, x, b)
            with np.errstate(all="ignore"):
                assert_bit_equal(x, orc.pairwise("sum", a, b))
    finally:
        fmi_amd.tune_set(Tune.HOST_CHUNK, old)


@pytest.mark.parametrize("zero_copy", [0, 1])
@pytest.mark.parametrize("n", [3, 4099, (1 << 22) + 1])
def test_host_reduce_pair_pinned(device, zero_copy, n):
    from fmi_amd.device import PinnedArray

    old = fmi_amd.tune_get(Tune.HOST_ZERO_COPY)
    try:
        fmi_amd.tune_set(Tune.HOST_ZERO_COPY, zero_copy)
        for dtype, op in ((np.float32, Op.SUM), (np.int64, Op.MIN), (np.float64, Op.PROD)):
            a, b = inputs(dtype, n, 0), inputs(dtype, n, 1)
            pa, pb = PinnedArray(n, dtype), PinnedArray(n, dtype)
            pa.array[:] = a
            pb.array[:] = b
            fmi_amd.host_reduce_pair(op, pa.array, pb.array)
            with np.errstate(all="ignore"):
                assert_bit_equal(pa.array.copy(), orc.pairwise(OPNAME[op], a, b), f"{op.name} zero_copy={zero_copy}")
            assert_bit_equal(pb.array.copy(), b, "in operand untouched")
            pa.free()
            pb.free()
    finally:
        fmi_amd.tune_set(Tune.HOST_ZERO_COPY, old)


_CONCURRENT_CASES = [(np.float32, Op.SUM, (1 << 20) + 7), (np.int64, Op.MIN, 4099), (np.float64, Op.PROD, 1 << 18),
                     (np.int32, Op.MAX, (1 << 19) + 1), (np.float32, Op.MAX, 33), (np.float64, Op.SUM, (1 << 20) + 3)]


def _host_pair_rounds(t, rounds, errors, start=None):
    """Thread t's share of the concurrency test: `rounds` combines of its case, pinned buckets for odd t."""
    from fmi_amd.device import PinnedArray

    dtype, op, n = _CONCURRENT_CASES[t]
    try:
        if start is not None:
            start.wait()
        for r in range(rounds):
            a, b = inputs(dtype, n, 10 * t + r), inputs(dtype, n, 10 * t + r + 1)
            if t % 2:
                pa, pb = PinnedArray(n, dtype), PinnedArray(n, dtype)
                pa.array[:] = a
                pb.array[:] = b
                fmi_amd.host_reduce_pair(op, pa.array, pb.array)
                got = pa.array.copy()
                pa.free()
                pb.free()
            else:
                got = a.copy()
                fmi_amd.host_reduce_pair(op, got, b)
            with np.errstate(all="ignore"):
                want = orc.pairwise(OPNAME[op], a, b)
            if got.tobytes() != want.tobytes():
                errors.append(f"thread {t} round {r}: {op.name} {np.dtype(dtype).name} n={n}")
    except Exception as e:  # noqa: BLE001 - reported by the caller
        errors.append(f"thread {t}: {e!r}")


def host_pair_concurrently(rounds=3):
    """All of _CONCURRENT_CASES at once, one thread each; returns the list of failures."""
    import threading

    errors = []
    start = threading.Barrier(len(_CONCURRENT_CASES))
    threads = [threading.Thread(target=_host_pair_rounds, args=(t, rounds, errors, start))
               for t in range(len(_CONCURRENT_CASES))]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    if any(th.is_alive() for th in threads):
        errors.append("a host_reduce_pair caller did not finish")
    return errors


@pytest.mark.parametrize("zero_copy", [0, 1])
def test_host_reduce_pair_concurrent_threads(device, zero_copy):
    """Each calling thread has its own staging and streams (the reference's peers combine concurrently when
    they are threads of one process): 6 threads x 3 rounds of mixed ops / dtypes / sizes, pageable and
    pinned buckets, many pipeline chunks per call, every result bit-exact."""
    old = (fmi_amd.tune_get(Tune.HOST_CHUNK), fmi_amd.tune_get(Tune.HOST_ZERO_COPY))
    try:
        fmi_amd.tune_set(Tune.HOST_CHUNK, 1 << 16)
        fmi_amd.tune_set(Tune.HOST_ZERO_COPY, zero_copy)
        errors = host_pair_concurrently()
        assert not errors, errors
    finally:
        fmi_amd.tune_set(Tune.HOST_CHUNK, old[0])
        fmi_amd.tune_set(Tune.HOST_ZERO_COPY, old[1])


def _host_pipelines():
    import re

    m = re.search(r"host_pipelines=(\d+) idle=(\d+)", fmi_amd.describe())
    assert m, fmi_amd.describe()
    return int(m.group(1)), int(m.group(2))


def _host_staging():
    import re

    m = re.search(r"host_staging_bytes=(\d+) host_pipelines_max=(\d+)", fmi_amd.describe())
    assert m, fmi_amd.describe()
    return int(m.group(1)), int(m.group(2))


def test_host_reduce_pair_short_lived_threads_reuse_staging(device):
    """The reference spawns a thread per peer for every collective; each call leases a staging set and returns it
    to the pool: 40 waves of 4 short-lived threads leave at most the pool's cap of sets (not 160), and every
    combine is bit-exact."""
    import threading

    old = fmi_amd.tune_get(Tune.HOST_CHUNK)
    try:
        fmi_amd.tune_set(Tune.HOST_CHUNK, 1 << 16)
        before, _ = _host_pipelines()
        errors = []
        for wave in range(40):
            ts = [threading.Thread(target=_host_pair_rounds, args=(t % 3 * 2, 1, errors)) for t in range(4)]
            for th in ts:
                th.start()
            for th in ts:
                th.join(timeout=120)
            assert not any(th.is_alive() for th in ts)
        assert not errors, errors
        import time

        after, idle = _host_pipelines()
        _, cap = _host_staging()
        assert after <= cap and after - before <= 4 and idle == after, (before, after, idle, cap)
    finally:
        fmi_amd.tune_set(Tune.HOST_CHUNK, old)


_MANY_SMALL_SCRIPT = """
import sys, threading, re
sys.path.insert(0, {root!r})
import numpy as np
import fmi_amd
from fmi_amd import Op
fmi_amd.init(0)
n = (256 << 10) // 4  # 256 KiB pageable buckets: staged, one chunk each
T = 48
start = threading.Barrier(T)
bad = []
def body(t):
    rng = np.random.default_rng(t)
    a, b = rng.random(n, dtype=np.float32), rng.random(n, dtype=np.float32)
    start.wait()
    for r in range(5):
        got = a.copy()
        fmi_amd.host_reduce_pair(Op.SUM, got, b)
        if not np.array_equal(got, a + b):
            bad.append((t, r))
ts = [threading.Thread(target=body, args=(t,)) for t in range(T)]
[x.start() for x in ts]
[x.join(timeout=120) for x in ts]
assert not any(x.is_alive() for x in ts), "a caller did not finish"
assert not bad, bad
d = fmi_amd.describe()
sets = int(re.search(r"host_pipelines=(\\d+)", d).group(1))
staging = int(re.search(r"host_staging_bytes=(\\d+)", d).group(1))
cap = int(re.search(r"host_pipelines_max=(\\d+)", d).group(1))
print("sets", sets, "staging", staging, "cap", cap)
assert 1 <= sets <= cap, d
assert staging <= sets * 4 * (256 << 10), d  # each set's 4 buffers sized to the 256 KiB bucket, not the 64 MiB chunk
print("ok")
"""


def test_host_reduce_pair_pool_is_bounded_for_many_small_callers(device):
    """48 threads making small pageable combines at once (the reference's peers as threads) share at
    most the pool's cap of staging sets, each sized to the bucket rather than the 64 MiB host chunk, and every
    combine is bit-exact. In a child process, so the set count starts from zero."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _MANY_SMALL_SCRIPT.format(root=root)], capture_output=True, text=True,
                       timeout=240, cwd=root)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout[-2000:] + r.stderr[-4000:]


_REINIT_SCRIPT = """
import sys
sys.path.insert(0, {root!r})
import fmi_amd
from fmi_amd import Tune
from tests import test_gpu_parity as t
for phase in range(3):
    fmi_amd.init(0)
    fmi_amd.tune_set(Tune.HOST_CHUNK, 1 << 16)
    errors = []
    t._host_pair_rounds(0, 2, errors)  # the main thread's pipeline: made, then rebuilt after every re-init
    errors += t.host_pair_concurrently(rounds=2)
    assert not errors, (phase, errors)
    fmi_amd.finalize()
print("ok")
"""


def test_host_reduce_pair_pipelines_survive_reinit(device):
    """fmi_dev_finalize frees every pooled pipeline; calls after fmi_dev_init lease fresh ones. In a child process,
    so the session's device state is left alone."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _REINIT_SCRIPT.format(root=root)], capture_output=True, text=True,
                       timeout=240, cwd=root)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout[-2000:] + r.stderr[-4000:]


def _page_aligned(n, dtype):
    """A contiguous numpy array of n elements starting on a 4 KiB boundary."""
    item = np.dtype(dtype).itemsize
    raw = np.empty(n * item + 8192, dtype=np.uint8)
    off = (-raw.ctypes.data) % 4096
    return raw[off:off + n * item].view(dtype)


@pytest.mark.parametrize("n", [5, 4099, (1 << 22) + 3])
def test_host_reduce_pair_registered(device, n):
    """fmi_host_register'd (pageable, then page-locked in place) buckets are combined zero-copy, bit-exact."""
    for dtype, op in ((np.float32, Op.SUM), (np.int32, Op.MAX)):
        a, b = inputs(dtype, n, 0), inputs(dtype, n, 1)
        ha, hb = _page_aligned(n, dtype), _page_aligned(n, dtype)
        ha[:] = a
        hb[:] = b
        with fmi_amd.HostRegistration(ha), fmi_amd.HostRegistration(hb):
            fmi_amd.host_reduce_pair(op, ha, hb)
        with np.errstate(all="ignore"):
            assert_bit_equal(ha, orc.pairwise(OPNAME[op], a, b), f"{op.name} n={n}")
        assert_bit_equal(hb, b, "in operand untouched")


def test_host_reduce_pair_partly_registered_is_refused(device):
    """A bucket that only starts inside a registered range is refused with FMI_ERR_INVALID: the zero-copy
    kernel must not read past the range, and the runtime rejects copies straddling its end. The buckets
    are left untouched."""
    n = 1 << 20
    a, b = inputs(np.float32, n, 0), inputs(np.float32, n, 1)
    ha, hb = _page_aligned(n, np.float32), _page_aligned(n, np.float32)
    ha[:] = a
    hb[:] = b
    with fmi_amd.HostRegistration(ha[: n // 2]), fmi_amd.HostRegistration(hb):
        with pytest.raises(fmi_amd.FmiError, match="straddles"):
            fmi_amd.host_reduce_pair(Op.SUM, ha, hb)
    assert_bit_equal(ha, a)
    with fmi_amd.HostRegistration(ha), fmi_amd.HostRegistration(hb):  # whole buckets: fine
        fmi_amd.host_reduce_pair(Op.SUM, ha, hb)
    assert_bit_equal(ha, a + b)


def test_host_register_errors(device):
    with pytest.raises(ValueError):
        fmi_amd.HostRegistration(np.empty(0, np.float32))
    lib = fmi_amd.load()
    assert lib.fmi_host_register(None, 16) != 0
    assert lib.fmi_host_unregister(None) != 0


# ------------------------------------------------------------------------------------------------
# BASELINE.json full-size configs
# ------------------------------------------------------------------------------------------------
def test_c2_256mib_f32_pairwise_sum(device):
    n = (256 << 20) // 4
    a = Bucket(n, np.float32).fill_synthetic(42, 0)
    b = Bucket(n, np.float32).fill_synthetic(42, 1)
    ha, hb = orc.synthetic(np.float32, n, 42, 0), orc.synthetic(np.float32, n, 42, 1)
    fmi_amd.reduce_pair(Op.SUM, a, b)
    assert_bit_equal(a.numpy(), ha + hb, "C2")


def test_c3_64mib_i64_max(device):
    n = (64 << 20) // 8
    a = Bucket(n, np.int64).fill_synthetic(42, 0)
    b = Bucket(n, np.int64).fill_synthetic(42, 1)
    fmi_amd.reduce_pair(Op.MAX, a, b)
    want = orc.op_max(orc.synthetic(np.int64, n, 42, 0), orc.synthetic(np.int64, n, 42, 1))
    assert_bit_equal(a.numpy(), want, "C3 max")


def test_c3_8peer_f32_scan_64mib(device):
    P, n = 8, (64 << 20) // 4
    ins = [Bucket(n, np.float32).fill_synthetic(42, p) for p in range(P)]
    outs = [Bucket(n, np.float32) for _ in range(P)]
    fmi_amd.scan_peers(Op.SUM, Alg.SCAN, outs, ins)
    want, _ = orc.scan([orc.synthetic(np.float32, n, 42, p) for p in range(P)], orc.op_sum)
    for k in range(P):
        assert_bit_equal(outs[k].numpy(), want[k], f"C3 scan peer {k}")


def test_beyond_2pow32_elements_64bit_indexing(device):
    """Maximum sizes: buckets of 2^32 + 1029 f32 elements (16 GiB each) through the pairwise, fused tree and
    peer-scan kernels. Every launch index is 64-bit; windows around 2^31 and 2^32 and the ragged tail are
    compared with the oracle's synthetic values."""
    from fmi_amd import Alg

    n = (1 << 32) + 1029
    windows = [(0, 4096), ((1 << 31) - 2048, 4096), ((1 << 32) - 2048, 3000), (n - 4096, 4096)]

    def host(peer, lo, m):
        return orc.synthetic_at(np.float32, np.arange(lo, lo + m, dtype=np.uint64), 42, peer)

    ins = [Bucket(n, np.float32).fill_synthetic(42, p) for p in range(3)]
    out = Bucket(n, np.float32)
    fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, out, ins)
    fmi_amd.sync()
    for lo, m in windows:
        want, _ = orc.allreduce([host(p, lo, m) for p in range(3)], orc.op_sum)
        assert_bit_equal(out.view(lo, m).numpy(), want[0], f"tree window {lo}")
    scan_out = [out, Bucket(n, np.float32)]
    fmi_amd.scan_peers(Op.SUM, Alg.SCAN, scan_out, ins[:2])
    fmi_amd.sync()
    for lo, m in windows:
        want, _ = orc.scan([host(p, lo, m) for p in range(2)], orc.op_sum)
        for k in range(2):
            assert_bit_equal(scan_out[k].view(lo, m).numpy(), want[k], f"scan peer {k} window {lo}")
    scan_out[1].free()
    out.free()
    ins[2].free()
    fmi_amd.reduce_pair(Op.SUM, ins[0], ins[1])
    fmi_amd.sync()
    for lo, m in windows:
        assert_bit_equal(ins[0].view(lo, m).numpy(), host(0, lo, m) + host(1, lo, m), f"pair window {lo}")
    for b in ins[:2]:
        b.free()


def test_dev_alloc_places_buckets_in_rotating_slots(device):
    """fmi_dev_alloc with FMI_TUNE_ALLOC_SLOTS = 1 (round 5's placement): 16 buckets of >= 1 MiB
    allocated one after another sit in 16 distinct 4 KiB slots modulo 64 KiB, are 4 KiB aligned, usable to their
    last byte and freed through fmi_dev_free; small buckets and the default (0) are plain hipMallocs; a fused kernel
    over slotted buckets gives the same bits as over plain ones."""
    n = (1 << 20) // 4 + 7
    default = fmi_amd.tune_get(Tune.ALLOC_SLOTS)
    assert default == 0
    plain_first = Bucket(16 << 20, np.float32)  # by default a plain hipMalloc: a large bucket at its aligned base
    assert plain_first.ptr % 65536 == 0, hex(plain_first.ptr)
    plain_first.free()
    fmi_amd.tune_set(Tune.ALLOC_SLOTS, 1)
    try:
        bs = [Bucket(n, np.float32) for _ in range(16)]
    finally:
        fmi_amd.tune_set(Tune.ALLOC_SLOTS, default)
    slots = {(b.ptr % 65536) // 4096 for b in bs}
    assert len(slots) == 16 and all(b.ptr % 4096 == 0 for b in bs), [hex(b.ptr) for b in bs]
    for k, b in enumerate(bs):
        b.fill_synthetic(3, k)
    xs = [b.numpy() for b in bs[:8]]
    for k, b in enumerate(bs):
        tail = b.view(n - 5, 5).numpy()
        assert np.array_equal(tail.view(np.uint32), orc.synthetic(np.float32, n, 3, k)[-5:].view(np.uint32))
    out_slotted = Bucket(n, np.float32)
    fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, out_slotted, bs[:8])
    old = fmi_amd.tune_get(Tune.ALLOC_SLOTS)
    try:
        plain = [Bucket.from_numpy(x) for x in xs]
        out_plain = Bucket(n, np.float32)
        fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, out_plain, plain)
        assert out_plain.numpy().tobytes() == out_slotted.numpy().tobytes()
        for b in plain + [out_plain]:
            b.free()
    finally:
        fmi_amd.tune_set(Tune.ALLOC_SLOTS, old)
    small = [Bucket(1000, np.float32) for _ in range(4)]  # < 1 MiB: plain allocations
    for b in bs + small + [out_slotted]:
        b.free()
    with pytest.raises(fmi_amd.FmiError):
        fmi_amd.tune_set(Tune.ALLOC_SLOTS, 2)


def test_dev_alloc_group_places_each_bucket_by_its_index(device):
    """fmi_dev_alloc_group: bucket j of a group of >= 1 MiB buckets sits in 4 KiB slot j mod 16 modulo
    64 KiB whatever was allocated before (here after 5 and 11 unrelated slotted allocations, and with
    FMI_TUNE_ALLOC_SLOTS = 0), carved from one allocation, usable to its last byte, freed through fmi_dev_free in any
    order (the range goes with the last bucket); a fused kernel over a group gives the same bits as over plain
    buckets; small groups are plain 4 KiB-aligned allocations; an impossible group fails whole (FmiError, no bucket
    handed out, and no error left behind for the next launch); count 0 is a no-op."""
    n = (1 << 20) // 4 + 7
    old = fmi_amd.tune_get(Tune.ALLOC_SLOTS)
    try:
        for before, slots_on in ((5, 1), (11, 1), (3, 0)):
            fmi_amd.tune_set(Tune.ALLOC_SLOTS, slots_on)
            others = [Bucket(n, np.float32) for _ in range(before)]
            g = Bucket.group(18, n, np.float32)
            assert [(b.ptr % 65536) // 4096 for b in g] == [j % 16 for j in range(18)], [hex(b.ptr) for b in g]
            assert len({g[j + 1].ptr - g[j].ptr for j in range(17)}) == 1  # one range, a fixed stride
            for k, b in enumerate(g):
                b.fill_synthetic(3, k)
            for k, b in enumerate(g):
                tail = b.view(n - 5, 5).numpy()
                assert np.array_equal(tail.view(np.uint32), orc.synthetic(np.float32, n, 3, k)[-5:].view(np.uint32))
            fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, g[8], g[:8])
            fmi_amd.tune_set(Tune.ALLOC_SLOTS, 0)
            plain = [Bucket.from_numpy(b.numpy()) for b in g[:8]]
            out = Bucket(n, np.float32)
            fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, out, plain)
            assert out.numpy().tobytes() == g[8].numpy().tobytes()
            for b in others + (g[::-1] if before == 11 else g) + plain + [out]:
                b.free()
    finally:
        fmi_amd.tune_set(Tune.ALLOC_SLOTS, old)
    small = Bucket.group(4, 1000, np.float32)
    assert all(b.ptr % 4096 == 0 for b in small)
    for b in small:
        b.free()
    assert Bucket.group(0, n, np.float32) == []
    with pytest.raises(fmi_amd.FmiError, match="group of 3 buckets"):
        Bucket.group(3, 1 << 46, np.uint8)  # 64 TiB each: the group's one allocation fails
    with pytest.raises(fmi_amd.FmiError, match="group too large"):
        Bucket.group(1 << 20, 1 << 45, np.uint8)  # its size does not fit in 64 bits
    a, b = Bucket.from_numpy(np.ones(4099, np.float32)), Bucket.from_numpy(np.ones(4099, np.float32))
    fmi_amd.reduce_pair(Op.SUM, a, b)  # the failed allocation left no error behind for the next launch to find
    assert np.array_equal(a.numpy(), np.full(4099, 2, np.float32))
    a.free()
    b.free()


@pytest.mark.parametrize("chunk", [(1 << 16), (3 << 20) + 4096, (64 << 20)])
def test_host_reduce_pair_staging_sizes(device, chunk):
    """The pooled staging sets grow to the largest chunk they served (a power of two from 64 KiB, capped at the
    tuned host chunk, which need not be one): pageable pairs of 1 element to 9 MiB in every dtype width, under a
    small, an odd and the default chunk, every result bit-exact."""
    old = fmi_amd.tune_get(Tune.HOST_CHUNK)
    try:
        fmi_amd.tune_set(Tune.HOST_CHUNK, chunk)
        for dtype, n in ((np.float32, 1), (np.int8, 65537), (np.float64, (1 << 17) + 3), (np.int16, (3 << 20) + 5),
                         (np.float32, (9 << 18) + 1), (np.int64, (9 << 17) - 1)):
            a, b = inputs(dtype, n, 3), inputs(dtype, n, 4)
            got = a.copy()
            fmi_amd.host_reduce_pair(Op.SUM, got, b)
            with np.errstate(all="ignore"):
                assert_bit_equal(got, orc.pairwise("sum", a, b), f"{np.dtype(dtype).name} n={n} chunk={chunk}")
    finally:
        fmi_amd.tune_set(Tune.HOST_CHUNK, old)
