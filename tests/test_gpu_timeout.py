"""Timeout semantics of the device communicator (include/fmi_dev.h FMI_ERR_TIMEOUT): a peer that does not
arrive surfaces as the reference's FMI::Utils::Timeout (reference include/utils/Common.h:11-15, thrown by its
channels when a peer stays away, src/comm/Direct.cpp:28-30,40-42) — fmi_amd.comm.Timeout / fmi.Timeout in
Python, Utils::Timeout in C++ (tests/test_cpp_communicator.py runs rccl_channel_absent_peer_raises_timeout) —
instead of a hang, and the communicator is aborted (later calls fail) but destroys cleanly.

- LOCAL: two ranks as threads, one never calls the collective.
- PROC: three processes, one exits after the first allreduce (or in the middle of its next exchange); the other
  two must time out in their second allreduce.
- RCCL: rank 0 alone initialising a 2-rank communicator (non-blocking init + ncclCommAbort)."""
import json
import os
import subprocess
import sys
import threading
import time

import numpy as np
import pytest

import fmi_amd
from fmi_amd import Bucket, Op, fmi
from fmi_amd.comm import Comm, Timeout, Transport, unique_id

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_timeout_is_the_reference_exception_type():
    assert fmi.Timeout is Timeout and issubclass(Timeout, fmi_amd.FmiError)


def test_local_absent_rank_times_out(device):
    uid = unique_id(Transport.LOCAL)
    res = {}

    def absent():
        c = Comm(uid, 2, 1, timeout_s=1.0)
        res["joined"] = True
        time.sleep(3.0)  # present, but never calls the collective
        c.destroy()

    t = threading.Thread(target=absent)
    c0 = Comm(uid, 2, 0, timeout_s=1.0)
    t.start()
    x, o = Bucket.from_numpy(np.ones(4099, np.float32)), Bucket(4099, np.float32)
    t0 = time.monotonic()
    with pytest.raises(Timeout, match="Timeout was reached"):
        c0.allreduce(Op.SUM, x, o)
    waited = time.monotonic() - t0
    assert 0.9 <= waited < 20, waited
    with pytest.raises(fmi_amd.FmiError, match="aborted"):
        c0.allreduce(Op.SUM, x, o)
    c0.destroy()
    t.join(timeout=30)
    assert res.get("joined")


@pytest.mark.parametrize("call", ["barrier", "allreduce"])
def test_local_late_rank_after_a_timeout_times_out_too(device, call):
    """ranks 0 and 1 time out waiting for rank 2 and return (their published buckets may
    then be freed); rank 2 arrives afterwards. Rank 2 must get Timeout too — never a barrier that releases on
    the departed ranks' stale arrivals and then reads their buckets."""
    uid = unique_id(Transport.LOCAL)
    n = 4099
    outcome = {}

    def rank(r, delay):
        c = Comm(uid, 3, r, timeout_s=1.0)
        x, o = Bucket.from_numpy(np.full(n, r + 1, np.float32)), Bucket(n, np.float32)
        time.sleep(delay)
        try:
            if call == "barrier":
                c.barrier()
            else:
                c.allreduce(Op.SUM, x, o)
                fmi_amd.sync()
            outcome[r] = "completed"
        except Timeout:
            outcome[r] = "timeout"
        except fmi_amd.FmiError as e:
            outcome[r] = f"error: {e}"
        x.free()
        o.free()
        c.destroy()

    threads = [threading.Thread(target=rank, args=(r, 2.5 if r == 2 else 0.0)) for r in range(3)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=60)
    assert outcome == {0: "timeout", 1: "timeout", 2: "timeout"}, outcome


def _run(cmd, timeout):
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout,
                       env=dict(os.environ, OMP_NUM_THREADS="1"))
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    return r, (json.loads(lines[-1]) if lines else None)


@pytest.mark.parametrize("when", ["before", "during"])
def test_proc_rank_exit_makes_the_others_time_out(device, when):
    N, die, limit = 3, 2, 4.0
    uid = unique_id(Transport.PROC).hex()
    procs = [subprocess.Popen([sys.executable, "-u", "-m", "tests._timeout_worker", "proc", uid, str(N), str(r),
                               str(limit), str(die), when], cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True, env=dict(os.environ, OMP_NUM_THREADS="1"))
             for r in range(N)]
    outs = []
    for p in procs:
        try:
            out, err = p.communicate(timeout=180)
        except subprocess.TimeoutExpired:
            p.kill()
            out, err = p.communicate()
        outs.append((p.returncode, out, err))
    assert outs[die][0] == 17, outs[die]
    for r in range(N):
        if r == die:
            continue
        code, out, err = outs[r]
        assert code == 0, (r, code, err[-2000:])
        got = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
        assert got["first_ok"], got
        assert got["outcome"] == "timeout", got
        assert got["waited_s"] < limit + 20, got
        assert got["unusable"], got


def test_rccl_rank_alone_init_times_out(device):
    """Rank 0 of a 2-rank RCCL communicator whose rank 1 never starts: Timeout within the deadline (not a
    hang in ncclCommInitRank), and the process exits normally afterwards."""
    limit = 5.0
    r, got = _run([sys.executable, "-u", "-m", "tests._timeout_worker", "rccl_alone", str(limit)], timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    assert got is not None and got["outcome"] == "timeout", (got, r.stderr[-2000:])
    assert limit - 0.5 <= got["waited_s"] < limit + 30, got
