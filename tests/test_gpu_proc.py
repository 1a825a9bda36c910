"""The C-ABI communicator over the PROC transport: N ranks are separate processes (children of this
one, all on the one MI355X) exchanging through a page-locked shared-memory segment, with path DIRECT's
windows mapped across processes by HIP IPC — the process boundary the RCCL transport crosses between
GPUs, exercised on a single GPU. Each rank's results (tests/_proc_worker.py) are compared bit for bit with
the oracle's simulation of the reference collective over the same buckets."""
import os
import subprocess
import sys

import numpy as np
import pytest

from fmi_amd.comm import Transport, unique_id
from oracle import fmi_oracle as orc
from tests._proc_worker import ALLREDUCE_CASES
from tests.test_gpu_parity import OPNAME, assert_bit_equal, inputs

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def launch(N, tmp_path):
    uid = unique_id(Transport.PROC).hex()
    paths = [str(tmp_path / f"rank{r}.npz") for r in range(N)]
    procs = [subprocess.Popen([sys.executable, "-m", "tests._proc_worker", uid, str(N), str(r), paths[r]], cwd=ROOT,
                              env=dict(os.environ, FMI_PROC_TIMEOUT_S="90"))
             for r in range(N)]
    codes = []
    for p in procs:
        try:
            codes.append(p.wait(timeout=240))
        except subprocess.TimeoutExpired:
            p.kill()
            codes.append(p.wait())
    assert codes == [0] * N, f"rank exit codes {codes}"
    return [dict(np.load(p)) for p in paths]


@pytest.mark.parametrize("N", [2, 3, 4])
def test_proc_transport_collectives(device, N, tmp_path):
    res = launch(N, tmp_path)
    with np.errstate(all="ignore"):
        for name, dtype, op, n in ALLREDUCE_CASES:
            want, _ = orc.allreduce([inputs(dtype, n, r, seed=31) for r in range(N)], orc.OPS[OPNAME[op]])
            for r in range(N):
                assert_bit_equal(res[r]["allreduce_" + name], want[r], f"allreduce {name} rank {r}")
        want, _ = orc.allreduce([inputs(np.float32, 4099, r, seed=32) for r in range(N)], orc.op_sum,
                                commutative=False, associative=False)
        for r in range(N):
            assert_bit_equal(res[r]["ordered"], want[r], f"ordered rank {r}")
        xs = [inputs(np.float32, 2053, r, seed=33) for r in range(N)]
        for root in range(N):
            want, _ = orc.reduce(xs, orc.op_sum, root=root)
            assert_bit_equal(res[root]["reduce"], want, f"reduce root {root}")
        for dtype, op in ((np.float32, "sum"), (np.int64, "max")):
            want, _ = orc.scan([inputs(dtype, 65536 + 129, r, seed=34) for r in range(N)], orc.OPS[op])
            for r in range(N):
                assert_bit_equal(res[r]["scan_" + np.dtype(dtype).name], want[r], f"scan {op} rank {r}")
        want, _ = orc.allreduce([inputs(np.float64, 3 * 4099 + 17, r, seed=36) for r in range(N)], orc.op_sum)
        for r in range(N):
            assert_bit_equal(res[r]["host_f64"], want[r], f"host allreduce rank {r}")
        for dtype, op, n in ((np.float32, "sum", 3 * 65536 + 5), (np.int32, "min", 1027)):
            want, _ = orc.allreduce([inputs(dtype, n, r, seed=35) for r in range(N)], orc.OPS[op])
            for r in range(N):
                assert_bit_equal(res[r]["direct_" + np.dtype(dtype).name], want[r], f"direct {op} rank {r}")
        want, _ = orc.allreduce([inputs(np.float32, 3 * 65536 + 5, r, seed=37) for r in range(N)], orc.op_sum)
        for r in range(N):
            assert_bit_equal(res[r]["direct_stream_free"], want[r], f"direct on a user stream, rank {r}")
    assert np.array_equal(res[0]["gather"], np.concatenate([np.arange(1000) + 1000 * j for j in range(N)]))
    for r in range(N):
        assert res[r]["bcast_ok"][0] and res[r]["ring_ok"][0], f"rank {r}"
        assert np.array_equal(res[r]["scatter"], np.arange(r * 1000, (r + 1) * 1000))
