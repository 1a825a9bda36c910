"""One process of the communicator timeout tests (tests/test_gpu_timeout.py):

    python -m tests._timeout_worker proc <uid hex> <nranks> <rank> <timeout_s> <die_rank> [before|during]
        a PROC-transport rank: one allreduce with every rank, then rank `die_rank` exits (os._exit) — before
        its second allreduce, or 20 ms into a loop of them (inside an exchange) — while the others run a
        second allreduce of a 64 MiB bucket (two 32 MiB staging pieces per exchange), which must end in
        fmi_amd.comm.Timeout within about timeout_s.
    python -m tests._timeout_worker rccl_alone <timeout_s>
        rank 0 of a 2-rank RCCL communicator whose rank 1 never starts: fmi_comm_init must raise Timeout
        within about timeout_s (non-blocking ncclCommInitRankConfig, then ncclCommAbort), and the process
        must exit normally.

Prints one JSON line: {"outcome": "timeout" | "ok" | "error: ...", "waited_s": ...}."""
import json
import os
import sys
import time


def proc(uid_hex, N, r, timeout_s, die, when="before"):
    import numpy as np

    import fmi_amd
    from fmi_amd import Bucket, Op
    from fmi_amd.comm import Comm, Timeout

    fmi_amd.init(0)
    c = Comm(bytes.fromhex(uid_hex), N, r, timeout_s=timeout_s)
    x = Bucket.from_numpy(np.full(1027, r + 1, np.float32))
    o = Bucket(1027, np.float32)
    c.allreduce(Op.SUM, x, o)
    c.sync()
    first_ok = bool((o.numpy() == N * (N + 1) / 2).all())
    n = 16 << 20
    if r == die:
        if when == "during":  # dies inside the exchange: another thread ends the process mid-allreduce
            import threading

            threading.Timer(0.02, os._exit, args=(17,)).start()
            big, out = Bucket(n, np.float32), Bucket(n, np.float32)
            big.fill_synthetic(5, r)
            for _ in range(1000):
                c.allreduce(Op.SUM, big, out)
                c.sync()
        os._exit(17)  # a peer that disappears after joining: no destroy, no goodbye
    big, out = Bucket(n, np.float32), Bucket(n, np.float32)
    big.fill_synthetic(5, r)
    outcome = "ok"
    # "during": keep allreducing with the dying rank until it is gone (its exit lands inside one of them)
    for _ in range(1 if when == "before" else 1000):
        t0 = time.monotonic()
        try:
            c.allreduce(Op.SUM, big, out)
            c.sync()
        except Timeout:
            outcome = "timeout"
        except Exception as e:  # noqa: BLE001 - reported to the parent
            outcome = f"error: {type(e).__name__}: {e}"
        waited = time.monotonic() - t0
        if outcome != "ok":
            break
    unusable = False
    try:
        c.allreduce(Op.SUM, x, o)
    except Exception:  # noqa: BLE001 - the aborted communicator must refuse work
        unusable = True
    c.destroy()
    print(json.dumps({"outcome": outcome, "waited_s": waited, "first_ok": first_ok, "unusable": unusable}),
          flush=True)


def rccl_alone(timeout_s):
    import torch  # noqa: F401 - the product runs RCCL from torch's runtime (fmi_amd/collectives.py)

    import fmi_amd
    from fmi_amd.comm import Comm, Timeout, Transport, unique_id

    fmi_amd.init(0)
    uid = unique_id(Transport.RCCL)
    t0 = time.monotonic()
    outcome = "ok"
    try:
        Comm(uid, 2, 0, timeout_s=timeout_s)
    except Timeout:
        outcome = "timeout"
    except Exception as e:  # noqa: BLE001
        outcome = f"error: {type(e).__name__}: {e}"
    print(json.dumps({"outcome": outcome, "waited_s": time.monotonic() - t0}), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "proc":
        proc(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), float(sys.argv[5]), int(sys.argv[6]),
             sys.argv[7] if len(sys.argv) > 7 else "before")
    else:
        rccl_alone(float(sys.argv[2]))
