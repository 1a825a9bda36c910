"""The communicator's point-to-point exchange plans (fmi_amd/csrc/fmi_exchange_plan.h) on the host.

The RCCL transport posts these plans between GPUs as grouped ncclSend / ncclRecv; a receive whose length
differs from the matching send, or a send nobody receives, hangs RCCL. The one-GPU test box cannot run
RCCL with two ranks, so tests/exchange_plan_check.cpp simulates every plan for N = 1…40, 64, 100 and 257
ranks on tagged host buffers, pairing per ordered pair of ranks as RCCL does, and checks pairing, bounds,
single writes and the exchange's definition byte by byte (fixed-size all-to-all / all-gather / gather /
scatter, and the ragged all-to-all, all-gather, gather and all-to-all-back used for buckets whose last
shards are short). The LOCAL transport executes the same plans in the GPU tests (tests/test_gpu_comm*.py).
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("plan") / "exchange_plan_check")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "fmi_amd", "csrc"),
                    "-o", exe, os.path.join(ROOT, "tests", "exchange_plan_check.cpp")], check=True)
    return exe


def test_exchange_plans_pair_and_deliver(checker):
    r = subprocess.run([checker, "40"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok:"), r.stdout
