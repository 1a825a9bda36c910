"""Multi-process tests (torch.distributed gloo on CPU, world size 2 and 4) of the sharded allreduce in
fmi_amd/collectives.py — the N>1 path bench.py runs over RCCL on MI355X nodes.

Checks: with two peers per process and N a power of two, path "tree" reproduces the reference's
2N-peer recursive-doubling allreduce bit for bit on every rank (including ragged sizes that need shard
padding); path "rccl" (reduce-scatter) stays within the stated float tolerance; integer ops are exact
on both paths; the first local bucket is clobbered like the reference's sendbuf.
"""
import os
import socket
import tempfile

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.multiprocessing as mp  # noqa: E402

from oracle import fmi_oracle as orc  # noqa: E402
from tests import _dist_worker  # noqa: E402

OPS = {0: "sum", 1: "prod", 2: "max", 3: "min"}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, n, dtype, op, path, peers_per_gpu=2):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_dist_worker.run, args=(world, _free_port(), n, dtype, op, path, peers_per_gpu, d), nprocs=world,
                 join=True)
        outs = [np.load(os.path.join(d, f"out{r}.npy")) for r in range(world)]
        sends = [np.load(os.path.join(d, f"send{r}.npy")) for r in range(world)]
    dt = np.dtype(dtype.split(":")[0])
    xs = [orc.synthetic(dt, n, 42, p) for p in range(peers_per_gpu * world)]
    if dtype.endswith(":edges"):
        xs = [_dist_worker.with_edges(x, p) for p, x in enumerate(xs)]
    return outs, sends, xs


def _bits_equal(a, b):
    u = {4: np.uint32, 8: np.uint64}[a.dtype.itemsize]
    return np.array_equal(a.view(u), b.view(u))


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("n", [4096, 1000003])
def test_tree_path_bit_exact_vs_reference_allreduce(world, n):
    outs, sends, xs = _run(world, n, "float32", 0, "tree")
    want, _ = orc.allreduce(xs, orc.op_sum)
    for r in range(world):
        # GPU r hosts peers 2r, 2r+1 and ends with the value peer 2r holds in the reference
        assert _bits_equal(outs[r], want[2 * r]), f"rank {r}"
        # sendbuf clobbered with the local partial (reference PeerToPeer.cpp:103,119)
        assert _bits_equal(sends[r], xs[2 * r] + xs[2 * r + 1])


@pytest.mark.parametrize("op", [1, 2, 3])
def test_tree_path_other_ops_int64(op):
    with np.errstate(over="ignore"):
        outs, _, xs = _run(2, 2053, "int64", op, "tree")
        want, _ = orc.allreduce(xs, orc.OPS[OPS[op]])
    for r in range(2):
        assert np.array_equal(outs[r], want[2 * r])


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("op", [2, 3])
def test_tree_path_float_max_min_each_rank_keeps_its_operand_order(world, op):
    """Float max / min on ±0 ties and NaNs: the reference's peers end with different bits. Every GPU must
    hold its own peer's (2g) bits, not rank 0's: per-rank shard versions delivered by an all-to-all."""
    n = 4099
    outs, _, xs = _run(world, n, "float32:edges", op, "tree")
    want, _ = orc.allreduce(xs, orc.OPS[OPS[op]])
    assert any(not _bits_equal(want[0], want[2 * r]) for r in range(1, world)), "data must tell the ranks apart"
    for r in range(world):
        assert _bits_equal(outs[r], want[2 * r]), f"rank {r}"


def test_rccl_path_within_tolerance():
    world, n = 4, 65536 + 7
    outs, _, xs = _run(world, n, "float32", 0, "rccl")
    want, _ = orc.allreduce(xs, orc.op_sum)
    P = len(xs)
    bound = (P - 1) * 2.0 ** -24 * np.sum(np.abs(np.stack(xs).astype(np.float64)), axis=0)
    for r in range(world):
        err = np.abs(outs[r].astype(np.float64) - want[0].astype(np.float64))
        assert np.all(err <= bound), f"rank {r}: max err {err.max()}"
    assert all(_bits_equal(outs[0], o) for o in outs[1:])  # every rank gets the same bits


def test_rccl_path_exact_for_integers():
    outs, _, xs = _run(2, 4099, "int64", 2, "rccl")
    want, _ = orc.allreduce(xs, orc.op_max)
    for r in range(2):
        assert np.array_equal(outs[r], want[0])


def test_single_peer_per_gpu():
    world, n = 2, 1031
    outs, sends, xs = _run(world, n, "float32", 0, "tree", peers_per_gpu=1)
    want, _ = orc.allreduce(xs, orc.op_sum)
    for r in range(world):
        assert _bits_equal(outs[r], want[r])


def test_four_peers_per_gpu_bit_exact():
    """2^k local peers fold as the 2^k-peer allreduce program (recursive doubling's local rounds), so the
    sharded result is still the reference's bracketing: here 8 peers on 2 processes."""
    world, n = 2, 2053
    outs, _, xs = _run(world, n, "float32", 0, "tree", peers_per_gpu=4)
    want, _ = orc.allreduce(xs, orc.op_sum)
    for r in range(world):
        assert _bits_equal(outs[r], want[4 * r]), f"rank {r}"


def test_non_power_of_two_local_peers_rejected():
    from fmi_amd import collectives

    class _Stub(collectives.ShardedAllreduce):
        def __init__(self):  # no process group needed: the check precedes any exchange
            pass

    x = [torch.zeros(8) for _ in range(3)]
    with pytest.raises(ValueError, match="power-of-two"):
        _Stub().allreduce(0, x, torch.zeros(8))


@pytest.mark.parametrize("path", ["tree", "rccl"])
def test_bench_loop_runs_multi_process(path):
    import json

    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_dist_worker.run_bench, args=(world, _free_port(), 8192, path, d), nprocs=world, join=True)
        res = [json.load(open(os.path.join(d, f"bench{r}.json"))) for r in range(world)]
    # step time is the max over ranks: identical on every rank
    assert res[0]["step_ms"] == res[1]["step_ms"] > 0
    assert len(res[0]["kernel_ms"]) == 3
    assert res[0]["extra"]["exchange"] == path and res[0]["extra"]["kernel_algo_bytes"] == 3 * 8192 * 4


def test_topology_verdict():
    """bench.py's N > 1 topology check (fmi_amd.collectives.judge_topology, host logic): RCCL must see every
    rank at its own index on its own GPU; PROC ranks may share one (labelled)."""
    from fmi_amd.collectives import judge_topology

    def rep(r, count=4, trank=None, pci=None):
        return {"rank": r, "transport_count": count, "transport_rank": r if trank is None else trank,
                "transport_device": r, "torch_device": r, "pci_bus_id": pci or f"0000:{0x10 + r:02x}:00.0"}

    good = [rep(r) for r in range(4)]
    v = judge_topology(good, 4, "rccl")
    assert v["ok"] and v["rccl_ranks"] == 4 and v["distinct_gpus"]
    shared = [rep(r, pci="0000:11:00.0") for r in range(4)]
    assert not judge_topology(shared, 4, "rccl")["ok"]  # two ranks on one GPU over RCCL: refused
    v = judge_topology(shared, 4, "proc")
    assert v["ok"] and v["rccl_ranks"] is None and v["transport_ranks"] == 4 and "by design" in v["note"]
    assert not judge_topology([rep(r, count=3) for r in range(4)], 4, "rccl")["ok"]  # RCCL saw 3 ranks
    assert judge_topology([rep(r, count=3) for r in range(4)], 4, "rccl")["rccl_ranks"] == 3
    swapped = [rep(0, trank=1), rep(1, trank=0), rep(2), rep(3)]
    assert not judge_topology(swapped, 4, "rccl")["ok"]
    assert judge_topology([rep(0, count=1)], 1, "rccl")["ok"]
    # the librccl and visibility environment travel with the verdict: rank 0's, and any rank that differs
    rt = {"rccl_version": 22703, "rccl_path": "/opt/rocm/lib/librccl.so.1.0", "HIP_VISIBLE_DEVICES": None}
    v = judge_topology([dict(rep(r), runtime=rt) for r in range(4)], 4, "rccl")
    assert v["runtime"] == rt and "runtime_differs" not in v
    odd = dict(rt, HIP_VISIBLE_DEVICES="3")
    v = judge_topology([dict(rep(r), runtime=odd if r == 2 else rt) for r in range(4)], 4, "rccl")
    assert v["runtime"] == rt and v["runtime_differs"] == {2: odd}


def test_runtime_info_names_the_rccl_and_never_raises(monkeypatch):
    """fmi_amd.comm.runtime_info (config.topology.runtime and every N > 1 error line): the librccl the RCCL
    transport maps (fmi_comm_rccl_info: ncclGetVersion, real path) and the visibility environment; on a host
    where librccl cannot be loaded it reports the error instead of raising."""
    from fmi_amd.comm import runtime_info

    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1")
    info = runtime_info()
    assert info["HIP_VISIBLE_DEVICES"] == "0,1"
    if "rccl_error" not in info:
        assert info["rccl_version"] > 0 and "librccl" in info["rccl_path"] and os.path.isabs(info["rccl_path"])


@pytest.mark.parametrize("failing_rank", [-1, 0, 1])
def test_bench_exchange_fallback_agreement_world2(failing_rank):
    """bench.py's N > 1 exchange fallback (bench._fall_back), world size 2 over gloo: when one rank's communicator
    step raised, BOTH ranks fall back (destroying their communicator, naming the reason: their own error or
    "failed on another rank"); when none did, neither does."""
    import json

    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_dist_worker.run_fall_back, args=(world, _free_port(), failing_rank, d), nprocs=world, join=True)
        res = [json.load(open(os.path.join(d, f"fall{r}.json"))) for r in range(world)]
    for r, x in enumerate(res):
        assert x["fell"] == (failing_rank >= 0) and x["destroyed"] == (failing_rank >= 0), (r, x)
        if failing_rank < 0:
            assert x["calls"] == []
        elif r == failing_rank:
            assert x["calls"] == [f"RuntimeError: rank {r} broke"]
        else:
            assert x["calls"] == ["the fmi_comm allreduce failed on another rank"]
