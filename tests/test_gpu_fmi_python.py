"""The reference's Python API (`fmi` module, reference python/fmi_python.cpp) on the MI355X engine
(fmi_amd/fmi.py): the calls of the reference's own Python client (python/tests/client.py) run by P peers
(threads over the Local transport, one GPU), with the answers the reference's semantics give."""
import json
import os
import tempfile
import threading

import pytest

pytestmark = pytest.mark.gpu


def run_peers(P, body):
    import fmi_amd.fmi as fmi

    with tempfile.TemporaryDirectory() as d:
        cfg = os.path.join(d, "fmi.json")
        json.dump({"backends": {"Local": {"enabled": True, "rendezvous_dir": d, "max_timeout": 60000},
                                "Direct": {"enabled": True, "host": "127.0.0.1", "port": 10000}},
                   "model": {"FaaS": {"gib_second_price": 0.0000166667}}}, open(cfg, "w"))
        results, errors = [None] * P, [None] * P

        def worker(p):
            try:
                comm = fmi.Communicator(p, P, cfg, "pytest", 512)
                comm.hint(fmi.hints.fast)
                comm.barrier()
                results[p] = body(fmi, comm, p)
                comm.barrier()
                comm.finalize()
            except BaseException as e:  # noqa: BLE001
                errors[p] = e

        ts = [threading.Thread(target=worker, args=(p,)) for p in range(P)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=300)
        for e in errors:
            if e is not None:
                raise e
        return results


def test_reference_python_client_two_peers(device):
    def body(fmi, comm, p):
        T = fmi.types
        D = fmi.datatypes
        out = {}
        if p == 0:
            comm.send(42, 1, T(D.int))
            comm.send(14.2, 1, T(D.double))
            comm.send([1, 2], 1, T(D.int_list, 2))
            comm.send([1.32, 2.34], 1, T(D.double_list, 2))
        else:
            out["recv"] = [comm.recv(0, T(D.int)), comm.recv(0, T(D.double)), comm.recv(0, T(D.int_list, 2)),
                           comm.recv(0, T(D.double_list, 2))]
        out["bcast"] = [comm.bcast(42 if p == 0 else None, 0, T(D.int)),
                        comm.bcast([1.32, 2.34] if p == 0 else None, 0, T(D.double_list, 2))]
        out["gather"] = [comm.gather(1 + p, 0, T(D.int)), comm.gather([1.5 + p, 2.25], 0, T(D.double_list, 2))]
        out["scatter"] = comm.scatter([14, 42] if p == 0 else None, 0, T(D.int_list, 2))
        custom = fmi.func(fmi.op.custom, lambda a, b: 2 * a + 2 * b, True, True)
        out["reduce"] = [comm.reduce(42 + p, 0, fmi.func(fmi.op.sum), T(D.int)),
                         comm.reduce(14.0, 0, fmi.func(fmi.op.prod), T(D.double)),
                         comm.reduce(42 + p, 0, fmi.func(fmi.op.max), T(D.int)),
                         comm.reduce(41.0 - p, 0, fmi.func(fmi.op.min), T(D.double)),
                         comm.reduce(42, 0, custom, T(D.int)),
                         comm.reduce([42, 14], 0, fmi.func(fmi.op.prod), T(D.int_list, 2)),
                         comm.reduce([43.5 - p, 13.5 + p], 0, fmi.func(fmi.op.max), T(D.double_list, 2)),
                         comm.reduce([42, 14], 0, custom, T(D.int_list, 2))]
        out["allreduce"] = [comm.allreduce(42, fmi.func(fmi.op.sum), T(D.int)),
                            comm.allreduce(0.1, custom, T(D.double)),
                            comm.allreduce([42, 14], fmi.func(fmi.op.sum), T(D.int_list, 2))]
        out["scan"] = [comm.scan(42, fmi.func(fmi.op.sum), T(D.int)),
                       comm.scan(14.0, fmi.func(fmi.op.prod), T(D.double)),
                       comm.scan(42, custom, T(D.int)),
                       comm.scan([42, 14], fmi.func(fmi.op.sum), T(D.int_list, 2))]
        return out

    r = run_peers(2, body)
    assert r[1]["recv"] == [42, 14.2, [1, 2], [1.32, 2.34]]
    for p in range(2):
        assert r[p]["bcast"] == [42, [1.32, 2.34]]
        assert r[p]["scatter"] == [[14], [42]][p]
        assert r[p]["allreduce"] == [84, 2 * 0.1 + 2 * 0.1, [84, 28]]
    assert r[0]["gather"] == [[1, 2], [1.5, 2.25, 2.5, 2.25]]
    assert r[0]["reduce"] == [85, 196.0, 43, 40.0, 168, [1764, 196], [43.5, 14.5], [168, 56]]
    assert r[0]["scan"] == [42, 14.0, 42, [42, 14]]
    assert r[1]["scan"] == [84, 196.0, 2 * 42 + 2 * 42, [84, 28]]


@pytest.mark.parametrize("P", [3, 5])
def test_python_api_custom_op_follows_reference_order(device, P):
    """A non-associative custom op exposes the bracketing: the host evaluation uses the reference's
    programs (allreduce_no_order for commutative flags, left fold for non-commutative scalars)."""
    from oracle import fmi_oracle as orc

    f = lambda a, b: 2 * a - b  # noqa: E731 - neither commutative nor associative

    def body(fmi, comm, p):
        T, D = fmi.types, fmi.datatypes
        return [comm.allreduce(p + 1, fmi.func(fmi.op.custom, f, True, True), T(D.int)),
                comm.allreduce(p + 1, fmi.func(fmi.op.custom, f, False, False), T(D.int)),
                comm.scan(p + 1, fmi.func(fmi.op.custom, f, True, True), T(D.int)),
                comm.reduce(p + 1, P - 1, fmi.func(fmi.op.custom, f, True, True), T(D.int))]

    r = run_peers(P, body)
    xs = [p + 1 for p in range(P)]
    ar, _ = orc.allreduce(xs, f)
    ltr, _ = orc.allreduce(xs, f, commutative=False, associative=False)
    sc, _ = orc.scan(xs, f)
    red, _ = orc.reduce(xs, f, root=P - 1)
    for p in range(P):
        assert r[p][0] == ar[p] and r[p][1] == ltr[p] and r[p][2] == sc[p]
    assert r[P - 1][3] == red


def test_absent_peer_raises_fmi_timeout(device):
    """The reference's Python API raises fmi.Timeout when a peer stays away (reference channels:
    include/utils/Common.h:11-15, src/comm/Direct.cpp:28-30), bounded by the config's max_timeout: peer 1 joins
    and never calls the allreduce; peer 0's allreduce raises fmi.Timeout after ≈ 1 s, not a hang."""
    import time

    import fmi_amd.fmi as fmi

    with tempfile.TemporaryDirectory() as d:
        cfg = os.path.join(d, "fmi.json")
        json.dump({"backends": {"Local": {"enabled": True, "rendezvous_dir": d, "max_timeout": 1000}}}, open(cfg, "w"))
        out, errors = {}, []
        joined = threading.Event()

        def absent():
            try:
                comm = fmi.Communicator(1, 2, cfg, "timeout", 512)
                joined.set()
                time.sleep(4.0)
                comm.finalize()
            except BaseException as e:  # noqa: BLE001
                errors.append(e)

        t = threading.Thread(target=absent)
        t.start()
        comm = fmi.Communicator(0, 2, cfg, "timeout", 512)
        assert joined.wait(60)
        t0 = time.monotonic()
        with pytest.raises(fmi.Timeout):
            comm.allreduce([1.5, 2.5], fmi.func(fmi.op.sum), fmi.types(fmi.datatypes.double_list, 2))
        out["waited"] = time.monotonic() - t0
        comm.finalize()
        t.join(timeout=60)
        assert not errors, errors
        assert 0.9 <= out["waited"] < 20, out
