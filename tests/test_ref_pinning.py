"""Pins the oracle — and the product's evaluation-order programs — to the REFERENCE ITSELF for floats:
oracle/_ref/libfmi_ref.so runs the reference's own src/comm/PeerToPeer.cpp (compiled unmodified by
oracle/Makefile, oracle/ref_harness.cpp supplies an in-memory PeerToPeer transport), and
tests/golden/{ref_vectors.npz, ref_expr.json} hold its outputs (tests/golden/make_ref_vectors.py).

  * the committed fixtures == the oracle restatement (always; bit-exact, NaN matches NaN);
  * the committed bracketing == the oracle's == the kernels' programs (fmi_schedule_expr, host-only C-ABI);
  * where the library is built (the build container): a live run still gives the fixtures, the reference's
    own integer known answers (tests/golden/reference_kats.json) come out of the harness, and the live
    bracketing equals the oracle and the programs for every rank / root up to 33 peers, and for sampled ranks /
    roots at 37, 48, 63, 64, 65, 100, 128, 129 and 257.
CPU only.
"""
import json
import os
import re

import numpy as np
import pytest

from oracle import fmi_oracle as orc
from oracle import fmi_ref as ref

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
VEC = np.load(os.path.join(GOLDEN, "ref_vectors.npz"))  # allow_pickle=False (the default)
EXPR = json.load(open(os.path.join(GOLDEN, "ref_expr.json")))
live = pytest.mark.skipif(not ref.available(), reason="oracle/_ref not built (needs /root/reference)")

UINT = {4: np.uint32, 8: np.uint64}


def assert_bits(got, want, what):
    got, want = np.asarray(got), np.asarray(want)
    assert got.dtype == want.dtype and got.shape == want.shape, what
    same = got.view(UINT[got.dtype.itemsize]) == want.view(UINT[got.dtype.itemsize])
    if np.issubdtype(got.dtype, np.floating):
        same |= np.isnan(got) & np.isnan(want)
    assert same.all(), f"{what}: {np.count_nonzero(~same)} elements differ"


def fixture_cases():
    """(dtype name, op, P) of every case in ref_vectors.npz."""
    return sorted({tuple(k.split("/")[:3]) for k in VEC.files}, key=lambda c: (c[0], c[1], int(c[2][1:])))


CASES = fixture_cases()


@pytest.mark.parametrize("case", CASES, ids=["/".join(c) for c in CASES])
def test_fixture_vectors_equal_the_oracle(case):
    dn, op, Ps = case
    key, P = "/".join(case), int(Ps[1:])
    xs = list(VEC[f"{key}/in"])
    f = orc.OPS[op]
    ltr = dict(commutative=False, associative=False)
    with np.errstate(all="ignore"):
        want, sends = orc.allreduce(xs, f)
        for r in range(P):
            assert_bits(want[r], VEC[f"{key}/allreduce/recv"][r], f"{key} allreduce rank {r}")
            assert_bits(sends[r], VEC[f"{key}/allreduce/send"][r], f"{key} allreduce sendbuf {r}")
        want, _ = orc.allreduce(xs, f, **ltr)
        for r in range(P):
            assert_bits(want[r], VEC[f"{key}/allreduce_ltr/recv"][r], f"{key} allreduce_ltr rank {r}")
        want, sends = orc.scan(xs, f)
        for r in range(P):
            assert_bits(want[r], VEC[f"{key}/scan/recv"][r], f"{key} scan rank {r}")
            assert_bits(sends[r], VEC[f"{key}/scan/send"][r], f"{key} scan sendbuf {r}")
        want, _ = orc.scan(xs, f, **ltr)
        for r in range(P):
            assert_bits(want[r], VEC[f"{key}/scan_ltr/recv"][r], f"{key} scan_ltr rank {r}")
        roots = sorted(int(k.split("/")[4][4:]) for k in VEC.files if k.startswith(f"{key}/reduce/root")
                       and k.endswith("/recv"))
        assert roots
        for root in roots:
            want, sends = orc.reduce(xs, f, root=root)
            assert_bits(want, VEC[f"{key}/reduce/root{root}/recv"], f"{key} reduce root {root}")
            for r in range(P):
                assert_bits(sends[r], VEC[f"{key}/reduce/root{root}/send"][r], f"{key} reduce sendbuf {r}")
            want, _ = orc.reduce(xs, f, root=root, **ltr)
            assert_bits(want, VEC[f"{key}/reduce_ltr/root{root}/recv"], f"{key} reduce_ltr root {root}")


def test_fixtures_are_order_sensitive():
    """The fixtures would catch a wrong bracketing: for f32 sum, the reference's allreduce differs from a plain
    left fold of the same buckets at P >= 3 on some element (the peers' magnitudes differ by 2^k)."""
    for P in (3, 5, 8, 17, 33):
        xs = VEC[f"float32/sum/P{P}/in"]
        fold = xs[0].copy()
        with np.errstate(all="ignore"):
            for p in range(1, P):
                fold = fold + xs[p]
        got = VEC[f"float32/sum/P{P}/allreduce/recv"][0]
        finite = np.isfinite(got) & np.isfinite(fold)
        assert np.any(got[finite].view(np.uint32) != fold[finite].view(np.uint32)), P


@pytest.mark.parametrize("kind", ["allreduce", "reduce", "scan"])
@pytest.mark.parametrize("ordered", [False, True], ids=["commutative", "ltr"])
def test_fixture_bracketing_equals_oracle(kind, ordered):
    table = EXPR[kind + ("_ltr" if ordered else "")]
    assert sorted(int(p) for p in table) == list(range(1, 21))
    for Ps, per_rank in table.items():
        P = int(Ps)
        for r, e in enumerate(per_rank):
            kw = dict(root=r) if kind == "reduce" else dict(rank=r)
            assert orc.expr(kind, P, ordered=ordered, **kw) == e, (kind, P, r, ordered)


SCHEDULE = {("allreduce", False): "ALLREDUCE", ("reduce", False): "REDUCE", ("scan", False): "SCAN",
            ("reduce", True): "REDUCE_LTR", ("allreduce", True): "REDUCE_LTR", ("scan", True): "SCAN_LTR"}


def program_expr(alg: str, P: int, r: int) -> str:
    """fmi_schedule_expr for rank / root r. The commutative reduce program is written in transformed ids
    (root -> 0, reference PeerToPeer.cpp:287-293): root r's expression is root 0's with x_t -> x_((t + r) % P)."""
    import fmi_amd

    if alg == "REDUCE":
        t = fmi_amd.schedule_expr(fmi_amd.Alg.REDUCE, P, 0)
        return re.sub(r"x(\d+)", lambda m: "x%d" % ((int(m.group(1)) + r) % P), t)
    return fmi_amd.schedule_expr(getattr(fmi_amd.Alg, alg), P, r)


def test_fixture_bracketing_equals_the_kernels_programs():
    """The device kernels evaluate fmi_schedule.h's programs; fmi_schedule_expr prints the bracketing a program
    computes for a rank (reduce: the root). Each must be the reference's (host-only C-ABI call, no GPU)."""
    for (kind, ordered), alg in SCHEDULE.items():
        table = EXPR[kind + ("_ltr" if ordered else "")]
        for Ps, per_rank in table.items():
            for r, e in enumerate(per_rank):
                assert program_expr(alg, int(Ps), r) == e, (kind, ordered, Ps, r)


@live
@pytest.mark.parametrize("case", CASES[::5], ids=["/".join(c) for c in CASES[::5]])
def test_live_reference_reproduces_the_fixtures(case):
    key, P = "/".join(case), int(case[2][1:])
    xs = VEC[f"{key}/in"]
    with np.errstate(all="ignore"):
        r, s, _ = ref.run("allreduce", case[1], xs)
        r2, _, _ = ref.run("scan", case[1], xs, ordered=True)
    for k in range(P):
        assert_bits(r[k], VEC[f"{key}/allreduce/recv"][k], f"{key} allreduce {k}")
        assert_bits(s[k], VEC[f"{key}/allreduce/send"][k], f"{key} allreduce sendbuf {k}")
        assert_bits(r2[k], VEC[f"{key}/scan_ltr/recv"][k], f"{key} scan_ltr {k}")


@live
@pytest.mark.parametrize("P", list(range(1, 34)) + [37, 48, 63, 64, 65, 100, 128, 129, 257])
def test_live_reference_bracketing_equals_oracle_and_programs(P):
    ranks = range(P) if P <= 33 else sorted({0, 1, 5, P // 2, P - 2, P - 1})
    for (kind, ordered), alg in SCHEDULE.items():
        for r in ranks:
            kw = dict(root=r) if kind == "reduce" else dict(rank=r)
            e = ref.expr(kind, P, ordered=ordered, **kw)
            assert e == orc.expr(kind, P, ordered=ordered, **kw), (kind, ordered, P, r)
            assert e == program_expr(alg, P, r), (kind, ordered, P, r)


@live
def test_live_reference_sendbuf_side_effects_equal_oracle():
    """The reference's sendbuf after each collective (PeerToPeer.cpp:72,103,119,160,179 overwrite it; LTR keeps
    it), symbolically for every rank: what fmi_comm_reduce_sendbuf and the C++ channel reproduce."""
    for P in (1, 2, 3, 5, 6, 8, 13, 16):
        for r in range(P):
            for kind, ordered in (("allreduce", False), ("scan", False), ("reduce", False), ("reduce", True),
                                  ("allreduce", True), ("scan", True)):
                sym = orc.symbols(P)
                flags = dict(commutative=not ordered, associative=not ordered)
                if kind == "reduce":
                    for root in sorted({0, P - 1}):
                        _, sends = orc.reduce(sym, orc.sym_combine, root=root, **flags)
                        assert ref.expr(kind, P, rank=r, root=root, ordered=ordered, which="send") == sends[r]
                else:
                    fn = orc.allreduce if kind == "allreduce" else orc.scan
                    _, sends = fn(sym, orc.sym_combine, **flags)
                    assert ref.expr(kind, P, rank=r, ordered=ordered, which="send") == sends[r], (kind, P, r)


@live
@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.int32, np.int64, np.uint32, np.uint64],
                         ids=lambda d: np.dtype(d).name)
def test_live_reference_random_buckets_equal_oracle(dtype):
    rng = np.random.default_rng(np.dtype(dtype).num)
    for P in (1, 2, 3, 6, 7, 11, 16, 19, 40):
        n = int(rng.integers(1, 40))
        if np.issubdtype(dtype, np.floating):
            xs = [(rng.standard_normal(n) * 2.0 ** float(rng.integers(-30, 30))).astype(dtype) for _ in range(P)]
        else:
            info = np.iinfo(dtype)
            xs = [rng.integers(info.min, info.max, n, dtype=dtype, endpoint=True) for _ in range(P)]
        for op in ("sum", "prod", "max", "min", "sub"):
            for ordered in (False, True):
                if op == "sub" and not ordered:
                    continue
                f = orc.OPS.get(op, lambda a, b: a - b)
                flags = dict(commutative=not ordered, associative=not ordered)
                root = int(rng.integers(0, P))
                with np.errstate(all="ignore"):
                    got = ref.allreduce(xs, op, ordered), ref.scan(xs, op, ordered), ref.reduce(xs, op, root, ordered)
                    want = (orc.allreduce(xs, f, **flags), orc.scan(xs, f, **flags),
                            orc.reduce(xs, f, root=root, **flags))
                for (gr, gs), (wr, ws), what in zip(got, want, ("allreduce", "scan", "reduce")):
                    if what == "reduce":
                        assert_bits(gr, wr, f"{what} P={P} {op} root {root}")
                    else:
                        for k in range(P):
                            assert_bits(gr[k], wr[k], f"{what} P={P} {op} ordered={ordered} rank {k}")
                    for k in range(P):
                        assert_bits(gs[k], ws[k], f"{what} sendbuf P={P} {op} ordered={ordered} rank {k}")


KATS = json.load(open(os.path.join(GOLDEN, "reference_kats.json")))["kats"]
SCALAR_KATS = [k for k in KATS if k["fn"] in ("add", "mul", "sub")]


@live
@pytest.mark.parametrize("kat", SCALAR_KATS, ids=[k["id"] for k in SCALAR_KATS])
def test_harness_reproduces_the_reference_kats(kat):
    """The harness itself (its transport and its element ops) against the reference's own known answers
    (tests/communicator.cpp, tests/channels.cpp): the scalar int KATs run through the reference's
    PeerToPeer code on the in-memory transport."""
    from tests.test_oracle import _expected_all, _inputs

    xs = _inputs(kat)
    op = {"add": "sum", "mul": "prod", "sub": "sub"}[kat["fn"]]
    ordered = not (kat["commutative"] and kat["associative"])
    if kat["kind"] == "reduce":
        res, _ = ref.reduce(xs, op, root=kat["root"], ordered=ordered)
        assert res.tolist() == kat["expected_root"]
    elif kat["kind"] == "allreduce":
        res, _ = ref.allreduce(xs, op, ordered)
        assert [r.tolist() for r in res] == _expected_all(kat)
    else:
        res, _ = ref.scan(xs, op, ordered)
        assert [r.tolist() for r in res] == _expected_all(kat)


@live
def test_reference_scan_ltr_at_one_peer_sends_to_a_missing_peer():
    """Reference quirk, recorded: scan_ltr with P = 1 sends its bucket to peer 1 (PeerToPeer.cpp:143), which does
    not exist; the harness counts the message as dropped. The result (a copy) is what the oracle gives."""
    x = np.arange(5, dtype=np.float32)
    recv, send, dropped = ref.run("scan", "sum", [x], ordered=True)
    assert dropped == 1
    assert_bits(recv[0], x, "P = 1 scan_ltr result")


@live
def test_reference_allreduce_timing_runs():
    """bench.py's cpu_baseline C1 row: the reference's allreduce timed over 2 peer threads, through the vector
    adapter and in place; the adapter (6 bucket copies per combine) is the slower of the two."""
    ad = ref.time_allreduce(2, 1 << 16, 5, adapter=True)
    bi = ref.time_allreduce(2, 1 << 16, 5, adapter=False)
    assert ad > 0 and bi > 0


@live
def test_reference_scan_timing_runs():
    """bench.py's cpu_baseline C3 row: the reference's scan timed over 8 peer threads, through the vector adapter
    and in place."""
    ad = ref.time_scan(8, 1 << 14, 3, adapter=True)
    bi = ref.time_scan(8, 1 << 14, 3, adapter=False)
    assert ad > 0 and bi > 0


@live
@pytest.mark.parametrize("P", [1, 2, 3, 5, 8, 13, 17])
def test_live_reference_bcast_and_gather_equal_oracle(P):
    """The binomial bcast and gather the oracle restates (PeerToPeer.cpp:14-27, :186-239; gather carries
    reduce_ltr), against the reference's own, every root: the root's gathered buckets in real-id order (the
    wraparound copy of :213-222 included) and every peer's bucket after the bcast."""
    rng = np.random.default_rng(P)
    xs = [rng.standard_normal(7).astype(np.float32) for _ in range(P)]
    for root in range(P):
        recv, _, _ = ref.run("gather", "sum", xs, root=root)
        want = orc.gather(xs, root)
        assert_bits(recv[root], np.concatenate(want), f"gather P={P} root {root}")
        _, send, _ = ref.run("bcast", "sum", xs, root=root)
        got = orc.bcast(xs, root)
        for p in range(P):
            assert_bits(send[p], got[p], f"bcast P={P} root {root} peer {p}")
            assert_bits(send[p], xs[root], f"bcast P={P} root {root} peer {p} holds the root's bucket")


@live
def test_reference_library_is_built_from_the_reference_alone():
    """oracle/_ref/libfmi_ref.so holds the reference's PeerToPeer code (its symbols are defined in the library)
    and needs nothing of FMI from elsewhere: no undefined FMI symbol (the link ran with -Wl,-z,defs), so no
    stand-in for a missing reference part exists; its only C entry points are the harness's."""
    import subprocess

    nm = ["nm", "-C", "--defined-only", ref.LIB_PATH]
    defined = subprocess.run(nm, check=True, capture_output=True, text=True).stdout
    for fn in ("PeerToPeer::allreduce_no_order", "PeerToPeer::scan_no_order", "PeerToPeer::reduce_no_order",
               "PeerToPeer::reduce_ltr", "PeerToPeer::scan_ltr", "PeerToPeer::gather", "PeerToPeer::bcast"):
        assert fn in defined, fn
    undefined = subprocess.run(["nm", "-C", "-D", "--undefined-only", ref.LIB_PATH], check=True,
                               capture_output=True, text=True).stdout
    assert "FMI" not in undefined, undefined
    dyn = subprocess.run(["nm", "-D", "--defined-only", ref.LIB_PATH], check=True, capture_output=True,
                         text=True).stdout
    exported = sorted(line.split()[-1] for line in dyn.splitlines() if " T " in line)
    assert exported == ["fmi_ref_expr", "fmi_ref_run", "fmi_ref_run_bound", "fmi_ref_time_allreduce",
                        "fmi_ref_time_allreduce_bound", "fmi_ref_time_combine", "fmi_ref_time_scan"], exported
    # the product's C-ABI reaches the harness only by address (fmi_ref_run_bound): nothing of it is linked
    needed = subprocess.run(["readelf", "-d", ref.LIB_PATH], check=True, capture_output=True, text=True).stdout
    assert "libfmi_dev" not in needed and "fmi_" not in undefined, (needed, undefined)
