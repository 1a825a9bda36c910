"""bench.py's N>1 driver code run multi-process on one GPU: ranks are processes bootstrapped over
torch.distributed (gloo), the C-ABI communicator runs over the PROC transport (shared-memory staging, HIP IPC
windows) — the same code path the driver's 8-GPU run takes over RCCL, minus RCCL itself (which refuses two
ranks on one GPU).

- test_comm_allreduce_gloo_world2: CommAllreduce (bench loop, self-check, path DIRECT check, host buckets,
  shard kernel) in 2 processes; the allreduce result is compared bit for bit with the oracle's simulation of
  the reference's 2-peer allreduce (src/comm/PeerToPeer.cpp:96-130), and the self-check must reject a result
  checked against the wrong buckets.
- test_bench_py_proc_transport[world 2, 3, 4, 8]: bench.py itself under torch.distributed.run; its JSON line must
  carry a passing self_check (headline and C4 TREE), a correct C5 result, the topology every rank reported
  (PROC: shared GPU, labelled) and the single-GPU anchor `local_equivalent`.
- test_bench_py_launches_its_own_ranks: `python bench.py --gpus 2 …` with no launcher starts its ranks itself
  and prints the same one self-checked line.
- test_bench_py_force_dist_rccl_world1: the RCCL transport's own rank count (ncclCommCount) in the line.
Every N > 1 line must name its workload (`sharded_allreduce`) and the librccl version and path plus the
visibility environment it ran under (`config.topology.runtime`); the N = 1 line says `local_combine`.
- test_bench_py_error_line_names_the_runtime: ranks that fail before `value` leave one line with the error,
  the phase and the same runtime fields.
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
    _check_topology_and_anchor(line, world, "proc")


def _check_topology_and_anchor(line, world, transport):
    assert line["workload"] == "sharded_allreduce", line.get("workload")
    assert line["exchange"] == "fmi_comm", line.get("exchange")  # whose exchange `value` measured
    topo = line["config"]["topology"]
    assert topo["ok"] and topo["transport"] == transport and len(topo["ranks"]) == world, topo
    rt = topo["runtime"]  # the librccl and visibility environment the run used
    assert rt["rccl_version"] > 0 and "librccl" in rt["rccl_path"] and os.path.isabs(rt["rccl_path"]), rt
    assert "HIP_VISIBLE_DEVICES" in rt and "GPU_MAX_HW_QUEUES" in rt and "runtime_differs" not in topo, topo
    assert [r["transport_rank"] for r in topo["ranks"]] == list(range(world)), topo
    assert all(r["pci_bus_id"] for r in topo["ranks"]), topo
    if transport == "proc":
        assert topo["transport_ranks"] == world and topo["rccl_ranks"] is None
        assert world == 1 or (not topo["distinct_gpus"] and "share GPUs by design" in topo["note"]), topo
    else:
        assert topo["rccl_ranks"] == world and topo["distinct_gpus"], topo
    le = line["local_equivalent"]
    assert le["ms"] > 0 and le["GiB_s_reduced_buckets"] > 0 and le["value_over_local"] > 0, le
    assert f"{world} peers" in le["workload"]


def test_bench_py_launches_its_own_ranks():
    """No torch.distributed.run: bench.py starts the 2 ranks itself (a child launcher, never exec) and relays
    rank 0's one line; the line is the same self-checked N > 1 line as the torchrun form."""
    env = dict(os.environ, FMI_PROC_TIMEOUT_S="90", OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "FMI_BENCH_LAUNCHED"):
        env.pop(k, None)
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--transport", "proc", "--steps", "4", "--warmup", "1",
           "--dist-sets", "2", "--bucket-mib", "8", "--c4-mib", "16", "--c5-mib", "8", "--diag-deadline", "150",
           "--no-diagnostics"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["value"] > 0 and line["self_check"]["ok"]
    assert "without a launcher: starting" in r.stderr
    _check_topology_and_anchor(line, 2, "proc")


def test_bench_py_force_dist_rccl_world1():
    """The N > 1 code path over the RCCL transport at world size 1 (the only RCCL world a 1-GPU box has):
    the line carries RCCL's own rank count and the 1-GPU anchor."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--force-dist",
           "--steps", "4", "--warmup", "1", "--dist-sets", "2", "--bucket-mib", "8", "--c4-mib", "16",
           "--c5-mib", "8", "--no-diagnostics"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1, r.stdout  # RCCL's version banner goes to stderr (bench.claim_stdout)
    line = json.loads(lines[0])
    assert line["config"]["topology"]["rccl_ranks"] == 1
    assert "one_rank_exchange" in line["config"] and line["self_check"]["ok"] and line["c4"]["tree"]["self_check"]["ok"]
    assert line["c4"]["rccl"]["self_check"]["ok"]  # ncclReduceScatter + ncclAllGather with one rank
    _check_topology_and_anchor(line, 1, "rccl")


def test_bench_py_n1_line_self_checks_the_timed_combines():
    """N = 1 (config C2): the line carries a passing self_check — every set's bucket after its warm-up, timed and
    probe launches equals numpy's float32 a + b repeated that many times, bit for bit, on three windows per set —
    and is the only stdout line."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "FMI_BENCH_LAUNCHED"):
        env.pop(k, None)
    cmd = [sys.executable, "bench.py", "--steps", "10", "--warmup", "3", "--sets", "4", "--no-cpu-baseline",
           "--no-c3", "--no-c5"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    chk = line["self_check"]
    assert line["n_gpus"] == 1 and line["value"] > 0 and chk["ok"] and chk["mismatches"] == 0
    assert line["workload"] == "local_combine"
    assert chk["elements_checked"] == 4 * 3 * 4096


def test_bench_py_error_line_names_the_runtime():
    """A failed N > 1 run is diagnosable from its one line: every rank fails in the phase right after the
    communicator bootstrap (FMI_BENCH_TEST_RAISE_IN, bench._PhaseWatch.enter), and rank 0's line must carry the
    error, the phase and the runtime (librccl version and path, visibility environment)."""
    env = dict(os.environ, FMI_PROC_TIMEOUT_S="60", OMP_NUM_THREADS="1", FMI_BENCH_TEST_RAISE_IN="topology check")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--transport", "proc", "--steps", "2", "--warmup", "1", "--bucket-mib", "1", "--no-c5",
           "--no-diagnostics"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode != 0
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout + r.stderr[-3000:]
    line = json.loads(lines[0])
    assert line["value"] is None and line["workload"] == "sharded_allreduce", line
    assert line["exchange"] == "fmi_comm", line
    assert line["phase"] == "topology check" and "injected failure" in line["error"], line
    rt = line["runtime"]
    assert rt["rccl_version"] > 0 and "librccl" in rt["rccl_path"] and "HIP_VISIBLE_DEVICES" in rt, rt


@pytest.mark.parametrize("phase,allow", [("fmi_comm init", False), ("warm-up and timed allreduces", True)])
def test_bench_py_falls_back_to_torch_exchange_when_fmi_comm_fails(phase, allow):
    """If the product communicator cannot be built over RCCL, or fails in its first allreduces
    (FMI_BENCH_TEST_RAISE_IN injects the failure in that phase, on every rank), bench.py still measures the same
    sharded allreduce — the fused tree kernel of libfmi_dev.so on every shard, the two exchanges through
    torch.distributed's own RCCL group — self-checks it bit-exact, and names the reason in config.exchange_fallback
    and `exchange: torch_fallback` at top level. By default the product failed, so `value` is null, the rate is
    `fallback_value` and the run exits 1; --allow-exchange-fallback reports it as `value` and exits 0.
    World size 1 with --force-dist: the exchange runs with itself."""
    env = dict(os.environ, OMP_NUM_THREADS="1", FMI_BENCH_TEST_RAISE_IN=phase)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--force-dist",
           "--steps", "4", "--warmup", "1", "--dist-sets", "2", "--bucket-mib", "8", "--no-diagnostics"]
    if allow:
        cmd.append("--allow-exchange-fallback")
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
    assert (r.returncode == 0) == allow, r.stdout[-3000:] + r.stderr[-3000:]
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["exchange"] == "torch_fallback", line
    if allow:
        assert line["value"] > 0 and "fallback_value" not in line, line
    else:
        assert line["value"] is None and line["fallback_value"] > 0, line
    assert line["workload"] == "sharded_allreduce", line
    fb = line["config"]["exchange_fallback"]
    assert "injected failure" in fb["reason"] and "torch.distributed" in fb["exchange"], fb
    chk = line["self_check"]
    assert chk["ok"] and chk["mismatches"] == 0 and chk["elements_checked_per_rank"] > 0, chk
    assert line["roofline"]["kernel_avg_us"] > 0 and line["config"]["topology"]["ok"], line
    assert line["local_equivalent"]["GiB_s_reduced_buckets"] > 0, line
    assert "falling back to torch.distributed" in r.stderr
