"""The C++ FMI::Communicator surface (fmi_amd/cpp/include/fmi) through its test program
(fmi_amd/cpp/tests/test_communicator.cpp): the reference's own known-answer suites, evaluation order
against the kernels' schedules, errors and policy (CPU); device buckets and host offload (GPU); and
every peer's result of allreduce / reduce / scan checked bit-exactly against the oracle."""
import os
import subprocess
import tempfile

import numpy as np
import pytest

from oracle import fmi_oracle as orc
from oracle import fmi_ref as ref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "build", "cpp", "test_communicator")


@pytest.fixture(scope="module")
def exe():
    if not os.path.exists(EXE):
        subprocess.run(["make", "-C", os.path.join(ROOT, "fmi_amd", "cpp")], check=True)
    return EXE


def _dump(exe, kind, P, n, mode="host"):
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        path = f.name
    try:
        cmd = [exe, "--dump", kind, str(P), str(n), path] + ([f"--{mode}"] if mode != "host" else [])
        subprocess.run(cmd, check=True, timeout=300)
        raw = np.fromfile(path, dtype=np.float32)
    finally:
        os.unlink(path)
    raw = raw.reshape(2, P, n)
    return raw[0], raw[1]


def _expected(kind, P, n):
    xs = [orc.synthetic(np.float32, n, 42, p) for p in range(P)]
    ordered = kind.endswith("_ltr")
    base = kind[:-4] if ordered else kind
    flags = dict(commutative=not ordered, associative=not ordered)
    if base == "allreduce":
        res, sends = orc.allreduce(xs, orc.op_sum, **flags)
    elif base == "scan":
        res, sends = orc.scan(xs, orc.op_sum, **flags)
    else:
        root_res, sends = orc.reduce(xs, orc.op_sum, root=0, **flags)
        res = [root_res] + [None] * (P - 1)
    return res, sends


def _check(kind, P, n, recv, send):
    res, sends = _expected(kind, P, n)
    for p in range(P):
        if res[p] is not None:
            assert np.array_equal(recv[p].view(np.uint32), res[p].view(np.uint32)), f"{kind} P={P} peer {p}"
        assert np.array_equal(send[p].view(np.uint32), sends[p].view(np.uint32)), f"{kind} P={P} sendbuf {p}"


def _reference(kind, P, n):
    """The reference itself (oracle/_ref: its src/comm/PeerToPeer.cpp) on the dump's inputs: (recv, send) per
    peer, recv None where the reference leaves it undefined (reduce: non-roots)."""
    xs = [orc.synthetic(np.float32, n, 42, p) for p in range(P)]
    ordered = kind.endswith("_ltr")
    base = kind[:-4] if ordered else kind
    recv, send, _ = ref.run(base, "sum", xs, root=0, ordered=ordered)
    res = list(recv) if base != "reduce" else [recv[0]] + [None] * (P - 1)
    return res, list(send)


def _check_against_reference(kind, P, recv, send):
    res, sends = _reference(kind, P, recv.shape[1])
    for p in range(P):
        if res[p] is not None:
            assert np.array_equal(recv[p].view(np.uint32), res[p].view(np.uint32)), f"{kind} P={P} peer {p}"
        assert np.array_equal(send[p].view(np.uint32), sends[p].view(np.uint32)), f"{kind} P={P} sendbuf {p}"


live = pytest.mark.skipif(not ref.available(), reason="oracle/_ref not built (needs /root/reference)")


@live
@pytest.mark.parametrize("kind", ["allreduce", "reduce", "scan", "allreduce_ltr", "reduce_ltr", "scan_ltr"])
@pytest.mark.parametrize("P", [1, 2, 3, 5, 6, 8, 13, 16])
def test_cpp_host_path_matches_the_reference(exe, kind, P):
    """The C++ surface's channel algorithms (fmi_amd/cpp/include/fmi/comm/PeerToPeer.h) against the
    reference's own PeerToPeer.cpp on the same float buckets: every peer's recvbuf and sendbuf."""
    recv, send = _dump(exe, kind, P, 515)
    _check_against_reference(kind, P, recv, send)


@live
@pytest.mark.parametrize("kind", ["bcast", "gather", "scatter"])
@pytest.mark.parametrize("P", [1, 2, 3, 5, 8, 13])
def test_cpp_data_movement_matches_the_reference(exe, kind, P):
    """bcast / gather / scatter of the C++ surface (host buckets, Loopback channel) against the reference's own
    PeerToPeer code on the same buckets, at a root that is not 0 (transformed ids, gather's and scatter's
    wraparound copies): every peer's buffer bit for bit."""
    n = 37
    for root in sorted({0, P // 2, P - 1}):
        with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
            path = f.name
        try:
            subprocess.run([exe, "--dump-move", kind, str(P), str(n), str(root), path], check=True, timeout=120)
            raw = np.fromfile(path, dtype=np.float32)
        finally:
            os.unlink(path)
        if kind == "scatter":
            xs = [orc.synthetic(np.float32, P * n, 42, p) for p in range(P)]
            recv, _, _ = ref.run("scatter", "sum", xs, root=root)
            got = raw.reshape(P, n)
            for p in range(P):
                assert np.array_equal(got[p].view(np.uint32), recv[p].view(np.uint32)), (kind, P, root, p)
            continue
        xs = [orc.synthetic(np.float32, n, 42, p) for p in range(P)]
        recv, send, _ = ref.run(kind, "sum", xs, root=root)
        if kind == "bcast":
            got = raw.reshape(P, n)
            for p in range(P):
                assert np.array_equal(got[p].view(np.uint32), send[p].view(np.uint32)), (kind, P, root, p)
        else:
            got = raw.reshape(P, P * n)
            assert np.array_equal(got[root].view(np.uint32), recv[root].view(np.uint32)), (kind, P, root)


def test_cpp_suite_host(exe):
    out = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-4000:]
    assert "0 failed checks" in out.stderr


@pytest.mark.parametrize("kind", ["allreduce", "reduce", "scan", "allreduce_ltr", "reduce_ltr", "scan_ltr"])
@pytest.mark.parametrize("P", [2, 3, 5, 8])
def test_cpp_host_path_matches_oracle(exe, kind, P):
    n = 1027
    recv, send = _dump(exe, kind, P, n)
    _check(kind, P, n, recv, send)


@pytest.mark.gpu
def test_cpp_suite_gpu(exe):
    out = subprocess.run([exe, "--gpu"], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-4000:]
    assert "0 failed checks" in out.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("P", [2, 3, 4])
def test_cpp_rccl_channel_across_processes(exe, P):
    """FMI::Comm::Rccl over the PROC transport: P fork()ed peers on one GPU, device-bucket collectives
    bit-identical to the host-bucket collectives over the socket channel."""
    out = subprocess.run([exe, "--proc-channel", str(P)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-4000:]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["device", "offload"])
@pytest.mark.parametrize("kind", ["allreduce", "reduce", "scan", "allreduce_ltr", "scan_ltr"])
def test_cpp_device_path_matches_oracle(exe, mode, kind):
    P, n = 8, (1 << 16) + 5
    recv, send = _dump(exe, kind, P, n, mode)
    _check(kind, P, n, recv, send)
    if ref.available():  # the prebuilt checker travels with the tree
        _check_against_reference(kind, P, recv, send)


def test_c1_host_bench_runs(exe):
    """Config C1 (2-peer f32 sum-allreduce, forked peers over socketpairs): the host benchmark that bench.py
    reports beside the CPU baseline runs, and its three combine paths (reference adapter, built-in in place,
    built-in overlapped with the transfer in 2 MiB pieces) give identical bits. 8 MiB buckets, so the
    overlapped path really cuts the transfer."""
    import json

    out = subprocess.run([os.path.join(ROOT, "build", "cpp", "c1_bench"), "--reps", "3", "--mib", "8"], check=True,
                         capture_output=True, text=True, timeout=120)
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["config"] == "C1" and r["peers"] == 2 and r["bucket_mib"] == 8
    assert r["lambda_adapter_ms"] > 0 and r["builtin_inplace_ms"] > 0 and r["builtin_overlap_ms"] > 0
    assert r["paths_bit_identical"] is True


@pytest.mark.gpu
@pytest.mark.parametrize("peers", [2, 3])
def test_c1_overlapped_offload_bit_identical(exe, peers):
    """Host buckets over a socket channel with the combine on the GPU (use_device): the transfer cut into
    pieces, each piece combined by fmi_host_reduce_pair while the next moves — identical bits to the
    serial path and to the reference adapter."""
    import json

    out = subprocess.run([os.path.join(ROOT, "build", "cpp", "c1_bench"), "--reps", "3", "--mib", "16", "--peers",
                          str(peers), "--device", "0"], check=True, capture_output=True, text=True, timeout=120)
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["combine_on"].startswith("gpu") and r["paths_bit_identical"] is True
