"""bench.py's N>1 driver code run multi-process on one GPU: ranks are processes bootstrapped over
torch.distributed (gloo), the C-ABI communicator runs over the PROC transport (shared-memory staging, HIP IPC
windows) — the same code path the driver's 8-GPU run takes over RCCL, minus RCCL itself (which refuses two
ranks on one GPU).

- test_comm_allreduce_gloo_world2: CommAllreduce (bench loop, self-check, path DIRECT check, host buckets,
  shard kernel) in 2 processes; the allreduce result is compared bit for bit with the oracle's simulation of
  the reference's 2-peer allreduce (src/comm/PeerToPeer.cpp:96-130), and the self-check must reject a result
  checked against the wrong buckets.
- test_bench_py_proc_transport[world 2, 3, 4, 8]: bench.py itself under torch.distributed.run; its JSON line must
  carry a passing self_check (headline and C4 TREE) and a correct C5 result.
"""
import json
import os
import socket
import subprocess
import sys
import tempfile

import numpy as np
import pytest

from oracle import fmi_oracle as orc

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_comm_allreduce_gloo_world2():
    world, n = 2, 1_000_003
    with tempfile.TemporaryDirectory() as d:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "-m", "tests._gloo_comm_worker", d]
        r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240,
                           env=dict(os.environ, FMI_PROC_TIMEOUT_S="90", OMP_NUM_THREADS="1"))
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        res = [dict(np.load(os.path.join(d, f"rank{r}.npz"))) for r in range(world)]
    seed = int(res[0]["tree_seed"][0])
    want, _ = orc.allreduce([orc.synthetic(np.float32, n, seed, p) for p in range(world)], orc.op_sum)
    for r in range(world):
        assert np.array_equal(res[r]["tree"].view(np.uint32), want[r].view(np.uint32)), f"rank {r}"
        assert res[r]["self_check_ok"][0], f"rank {r}"
        assert not res[r]["self_check_wrong_seed_ok"][0], "the self-check accepted a wrong result"
        assert res[r]["direct_ok"][0] and res[r]["host_ok"][0], f"rank {r}"
        assert res[r]["kernel_bytes"][0] == (world + 1) * 32768 * 4
    assert res[0]["step_ms"][0] == res[1]["step_ms"][0] > 0  # max over ranks


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_bench_py_proc_transport(world):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", str(world),
           "--transport", "proc", "--steps", "4", "--warmup", "1", "--dist-sets", "2", "--bucket-mib", "8",
           "--c4-mib", "16", "--c5-mib", "8", "--diag-deadline", "150"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, FMI_PROC_TIMEOUT_S="90", OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == world and line["value"] > 0 and line["ms_per_step"] > 0
    assert "incomplete" not in line, line
    assert line["self_check"]["ok"] and line["self_check"]["elements_checked_per_rank"] > 0
    assert line["c4"]["tree"]["self_check"]["ok"]
    assert line["c5"]["result_ok"]
    assert line["roofline"]["algorithmic_bytes_per_launch"] > 0
    assert "every shard-kernel launch of the K timed allreduces" in line["roofline"]["kernel_avg_source"]
    assert line["config"]["peers"] == world and line["config"]["transport"] == "proc"
    assert "replicated_pairs" in line["diagnostics"]
