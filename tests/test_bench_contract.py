"""bench.py's host-side contract (CPU): the JSON line is printed exactly once, and the per-rank deadline
over the after-`value` section (C4, C5 and the diagnostics) prints the measured line, marked "incomplete" at
top level, and exits when that section hangs."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_emitter_prints_once(capsys):
    e = bench._Emitter({"metric": "m", "value": 1.0, "config": {}}, rank=0)
    e.emit()
    e.emit()
    out = capsys.readouterr().out.strip().splitlines()
    assert len(out) == 1 and json.loads(out[0])["value"] == 1.0


def test_emitter_silent_on_other_ranks(capsys):
    bench._Emitter({"metric": "m", "value": 1.0, "config": {}}, rank=3).emit()
    assert capsys.readouterr().out == ""


def test_deadline_prints_measured_line_and_exits():
    code = textwrap.dedent(f"""
        import sys, threading, time
        sys.path.insert(0, {ROOT!r})
        import bench
        line = {{"metric": "m", "value": 2.5, "config": {{}}}}
        state = line["c4"] = {{}}
        e = bench._Emitter(line, 0)
        t = threading.Timer(0.2, e.deadline, args=(state,))
        t.daemon = True
        t.start()
        time.sleep(30)  # a hung diagnostic
        print("not reached")
    """)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=20)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1
    got = json.loads(lines[0])
    assert got["value"] == 2.5 and "incomplete" in got and "incomplete" in got["c4"]


def test_defaults_are_the_contract(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert a.gpus == 1 and a.bucket_mib == 256 and a.steps > 0 and a.warmup > 0 and a.path == "tree"
    assert a.c4_mib == 1024 and a.transport == "rccl"  # C4: 1 GiB per peer, one process per GPU over RCCL


def test_roofline_traffic_is_the_launched_kernels():
    """roofline.traffic comes from the committed PMC summary of exactly the launch the line measures: C2's
    default pair_tile<OpSum, float, 4, 3> at 256 MiB (not another pair_tile instantiation, e.g. C3's i64
    max), and the N>1 shard kernel per world size at its shard size; PMC bytes within 1 % of the algorithmic
    bytes. A key matching several instantiations reports nothing rather than a wrong kernel's bytes."""
    import fmi_amd

    fmi_amd.load()
    key = bench.c2_kernel_signature()
    assert key == "pair_tile<fmi::dev::OpSum, float, 4, 3>"
    algo = 3 * 256 * (1 << 20)
    traffic, src = bench.pmc_traffic(key, algo)
    assert traffic is not None and abs(traffic / algo - 1) < 0.01, (traffic, src)
    assert bench.pmc_traffic("pair_tile", 3 * 64 * (1 << 20)) != (None, None)  # only C3's i64 max is 64 MiB
    assert bench.pmc_traffic("tree_kernel", 9 * 32 * (1 << 20)) != (None, None)
    assert bench.pmc_traffic("synth_kernel", 64 * (1 << 20)) == (None, None)  # ambiguous: f32 and i64
    for world, shard_mib in ((2, 128), (4, 64), (8, 32)):
        shard_algo = (world + 1) * shard_mib * (1 << 20)
        t, _ = bench.pmc_traffic(f"tree_kernel<fmi::dev::OpSum, float, 0, {world}, false>", shard_algo)
        assert t is not None and abs(t / shard_algo - 1) < 0.01, (world, t)


def test_same_instantiation_at_another_shape_is_not_returned():
    """The 8-way tree is profiled at two shapes (N = 8's 32 MiB shards, C3's 64 MiB buckets): each lookup gets
    its own shape's bytes, and a shape with no profile (e.g. --bucket-mib 64 at N = 8: 8 MiB shards) gets
    nothing, never the other shape's bytes."""
    key = "tree_kernel<fmi::dev::OpSum, float, 0, 8, false>"
    t32, _ = bench.pmc_traffic(key, 9 * 32 * (1 << 20))
    t64, _ = bench.pmc_traffic(key, 9 * 64 * (1 << 20))
    assert t32 is not None and t64 is not None and abs(t64 / t32 - 2) < 0.01
    assert bench.pmc_traffic(key, 9 * 8 * (1 << 20)) == (None, None)
    r = bench._roofline("pair_tile", 3 * 64 * (1 << 20), 0.05, "test",
                        pmc_key="pair_tile<fmi::dev::OpSum, float, 4, 3>")  # C2's kernel at a non-default size
    assert r["traffic"] is None and r["traffic_source"].startswith("not reported")


def test_pmc_merge_keeps_both_shapes(tmp_path):
    """tools/pmc_summarize.py: a merge replaces an entry only by a profile of the same instantiation AND shape."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from pmc_summarize import algorithmic_bytes, same_launch

    name = "void fmi::dev::tree_kernel<fmi::dev::OpSum, float, 0, 8, false>(fmi::dev::PeerPtrs, unsigned long, int, int)"
    a = {"kernel": name, "algorithmic_bytes_per_launch": algorithmic_bytes(name, 32 * (1 << 20) + 128)}
    b = {"kernel": name, "algorithmic_bytes_per_launch": algorithmic_bytes(name, 64 * (1 << 20))}
    assert a["algorithmic_bytes_per_launch"] == 9 * 32 * (1 << 20)
    assert not same_launch(a, b) and same_launch(a, dict(a))
    assert algorithmic_bytes("void fmi::dev::scan_kernel<fmi::dev::OpSum, float, 3, 8>(x)", 512 << 20) == 1 << 30
    assert algorithmic_bytes("void fmi::dev::pair_tile<fmi::dev::OpMax, long, 4, 3>(x)", 64 << 20) == 192 << 20


def test_measure_deadline_names_the_phase_and_exits_nonzero():
    """N > 1: a rank stuck before `value` reports its phase on stderr and exits with status 3 (run in a child
    process: the watch ends the process)."""
    code = ("import bench, time\n"
            "w = bench._PhaseWatch(0.2, 5)\n"
            "w.enter('warm-up and timed allreduces')\n"
            "time.sleep(5)\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=60)
    assert r.returncode == 3
    assert "rank 5 still in phase 'warm-up and timed allreduces'" in r.stderr
    assert r.stdout.strip() == ""  # only rank 0 prints the line
    code0 = code.replace("_PhaseWatch(0.2, 5)", "_PhaseWatch(0.2, 0)")
    r = subprocess.run([sys.executable, "-c", code0], cwd=ROOT, capture_output=True, text=True, timeout=60)
    assert r.returncode == 3
    line = json.loads(r.stdout.strip())
    assert line["value"] is None and line["phase"] == "warm-up and timed allreduces"


def test_relay_keeps_one_stdout_line_and_the_exit_status(capsys):
    """bench.relay: the child's JSON line reaches stdout, its other output goes to stderr, and a failing
    child's status comes back unchanged."""
    code = "import sys; print('rank 1 log'); print('{\"metric\": \"m\", \"value\": 1}'); sys.exit(5)"
    rc = bench.relay([sys.executable, "-c", code])
    cap = capsys.readouterr()
    assert rc == 5
    assert cap.out.strip().splitlines() == ['{"metric": "m", "value": 1}']
    assert "rank 1 log" in cap.err


def test_gpus_n_without_launcher_starts_ranks_and_fails_loudly():
    """`python bench.py --gpus 2` with no WORLD_SIZE starts 2 ranks under torch.distributed.run itself (a child
    process, no exec). Here one rank is made to fail before it touches anything (FMI_BENCH_TEST_FAIL_RANK):
    the launcher must return non-zero and print no line."""
    env = dict(os.environ, FMI_BENCH_TEST_FAIL_RANK="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "FMI_BENCH_LAUNCHED"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--transport", "proc",
                        "--bucket-mib", "1"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert r.stdout.strip() == ""
    assert "without a launcher: starting" in r.stderr and "torch.distributed.run" in r.stderr
    assert "FMI_BENCH_TEST_FAIL_RANK" in r.stderr


def test_library_stdout_noise_cannot_reach_the_line():
    """claim_stdout(): after it, anything written to fd 1 (RCCL's version banner, C printf) lands on stderr
    and the JSON line alone on the original stdout."""
    code = ("import os, sys, json\n"
            f"sys.path.insert(0, {ROOT!r})\n"
            "import bench\n"
            "bench.claim_stdout()\n"
            "os.write(1, b'RCCL version : banner\\n')\n"
            "print('python noise')\n"
            "print(json.dumps({'metric': 'm', 'value': 1}), file=bench.json_out(), flush=True)\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().splitlines() == ['{"metric": "m", "value": 1}']
    assert "RCCL version" in r.stderr and "python noise" in r.stderr


def test_pmc_summary_splits_one_kernel_by_launch_shape(tmp_path):
    """tools/pmc_summarize.py groups launches by (kernel, grid size): copy_tile launched at 256 MiB and at
    64 MiB in one run gives two entries with their own PMC bytes and trace durations, never a median across
    shapes (what round 3's first C2 profile would otherwise have reported for the copy kernel)."""
    import csv

    name = "void fmi::dev::copy_tile<4>(char*, char const*, unsigned long)"
    big, small = 16384, 4096  # workgroups: 256 MiB and 64 MiB in 16-KiB tiles (grid size = threads)
    for sub, counter, per in (("f", "FETCH_SIZE", lambda g: g * 8.0), ("w", "WRITE_SIZE", lambda g: g * 16.0)):
        d = tmp_path / sub
        d.mkdir()
        with open(d / "run_counter_collection.csv", "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Grid_Size", "Kernel_Name", "Counter_Name", "Counter_Value"])
            for g, k in ((big, 3), (small, 5)):
                for _ in range(k):  # KiB: fetch is half the bytes on gfx950 (x2 correction), write exact
                    w.writerow([g * 256, name, counter, per(g)])
    t = tmp_path / "t"
    t.mkdir()
    with open(t / "run_kernel_trace.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"])
        for g, ns, k in ((big, 84000, 3), (small, 24000, 5)):
            for i in range(k):
                w.writerow([name, 1000 * i, 1000 * i + ns, g * 256, 1, 1])
    out = tmp_path / "out"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summarize.py"), "--trace", str(t),
                        "--fetch", str(tmp_path / "f"), "--write", str(tmp_path / "w"), "--tag", "t", "--command", "x",
                        "--no-default", "--out", str(out)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    entries = {e["grid_size"]: e for e in json.load(open(out / "t_pmc_summary.json"))["kernels"]}
    assert set(entries) == {big * 256, small * 256}
    for g, mib, ns in ((big, 256, 84000), (small, 64, 24000)):
        e = entries[g * 256]
        assert e["algorithmic_bytes_per_launch"] == 2 * mib << 20
        assert e["hbm_bytes_per_launch"] == 2 * mib << 20  # 2 x fetch KiB + write KiB = 2 x bucket
        assert e["trace"]["avg_ns"] == ns and e["trace"]["calls"] == (3 if g == big else 5)


def test_c2_self_check_counts_every_launch_and_catches_one_flipped_bit():
    """bench.py's N = 1 self_check (c2_self_check) on host stand-ins for the buckets: after each set's a was
    combined in place with b as many times as `launches` says, the check passes bit for bit; one wrong element
    in one window (or a miscounted launch) fails it."""
    import numpy as np

    import bench

    class Host:
        def __init__(self, arr):
            self.arr = arr

        def view(self, o, n):
            return Host(self.arr[o:o + n])

        def numpy(self):
            return self.arr.copy()

    rng = np.random.default_rng(3)
    n, win = 1 << 14, 4096
    offs = [0, (n // 2) // 64 * 64, n - win]
    sets = [(Host(rng.random(n, dtype=np.float32)), Host(rng.random(n, dtype=np.float32))) for _ in range(3)]
    before = [[(a.view(o, win).numpy(), b.view(o, win).numpy()) for o in offs] for a, b in sets]
    launches = [5, 4, 4]
    for (a, b), k in zip(sets, launches):
        for _ in range(k):
            a.arr[:] = a.arr + b.arr
    ok = bench.c2_self_check(sets, offs, win, before, launches)
    assert ok["ok"] and ok["mismatches"] == 0 and ok["elements_checked"] == 3 * 3 * win
    assert not bench.c2_self_check(sets, offs, win, before, [4, 4, 4])["ok"]  # a miscounted launch
    sets[1][0].arr[n // 2 + 7] = np.nextafter(sets[1][0].arr[n // 2 + 7], np.float32(2))
    bad = bench.c2_self_check(sets, offs, win, before, launches)
    assert not bad["ok"] and bad["mismatches"] == 1


def test_failed_n_gt_1_run_leaves_one_error_line(monkeypatch, capsys):
    """A rank-0 failure inside the N > 1 path (here: the communicator bootstrap raising) prints one JSON line
    naming the error and the phase, then fails; with the line already out, nothing more is printed."""
    import json

    import bench

    def boom(args, world, rank, local_rank):
        bench._WATCH = type("W", (), {"phase": "fmi_comm init (communicator id broadcast, RCCL init)"})()
        raise RuntimeError("ncclCommInitRankConfig: unhandled system error")

    monkeypatch.setattr(bench, "run_dist", boom)
    monkeypatch.setattr(bench, "_LINE_PRINTED", False)
    monkeypatch.setattr(bench, "_JSON_OUT", None)
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("LOCAL_RANK", "0")
    monkeypatch.setattr("sys.argv", ["bench.py", "--gpus", "2"])
    with pytest.raises(RuntimeError):
        bench.main()
    out = capsys.readouterr().out.strip().splitlines()
    assert len(out) == 1
    line = json.loads(out[0])
    assert line["value"] is None and line["n_gpus"] == 2 and "unhandled system error" in line["error"]
    assert line["phase"].startswith("fmi_comm init")
    monkeypatch.setattr(bench, "_LINE_PRINTED", True)  # the measured line was already printed: no second line
    with pytest.raises(RuntimeError):
        bench.main()
    assert capsys.readouterr().out.strip() == ""


def test_scan_self_check_bracketing_evaluator_equals_the_oracle():
    """bench.py's C3 scan self-check evaluates each peer's program bracketing (fmi_schedule_expr) in numpy: for
    order-sensitive f32 buckets it must give the oracle's scan bit for bit (and a plain left fold must not)."""
    import numpy as np

    import bench
    import fmi_amd
    from oracle import fmi_oracle as orc

    rng = np.random.default_rng(11)
    for P in (1, 2, 3, 5, 8, 13):
        xs = [(rng.standard_normal(257) * 2.0 ** (7 * p % 13 - 6)).astype(np.float32) for p in range(P)]
        want, _ = orc.scan(xs, orc.op_sum)
        for r in range(P):
            got = bench.eval_bracketing(fmi_amd.schedule_expr(fmi_amd.Alg.SCAN, P, r), xs)
            assert np.array_equal(got.view(np.uint32), want[r].view(np.uint32)), (P, r)


def test_every_line_names_its_workload_and_failed_lines_name_the_runtime(monkeypatch):
    """The 1/2/4/8 curve spans two workloads, so every line says at top level which one `value` measures
    (local_combine at N = 1, sharded_allreduce at N > 1), and an N > 1 error line carries the librccl version and
    path and the device-visibility environment it failed under."""
    import argparse

    args = argparse.Namespace(gpus=1, force_dist=False, steps=1, warmup=1, bucket_mib=256, sets=16)
    assert bench._headline(args, 1.0, 1.0, "w", "p", 4, {})["workload"] == bench.WORKLOAD_N1 == "local_combine"
    args.gpus = 8
    assert bench._headline(args, 1.0, 1.0, "w", "p", 4, {})["workload"] == bench.WORKLOAD_DIST == "sharded_allreduce"
    args.gpus, args.force_dist = 1, True
    assert bench._headline(args, 1.0, 1.0, "w", "p", 4, {})["workload"] == "sharded_allreduce"
    assert "workload" in bench._HEADLINE_KEYS
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1,2,3")
    line = bench._error_line(4, "RuntimeError: boom", "topology check", topology={"ok": False})
    assert line["value"] is None and line["workload"] == "sharded_allreduce" and line["phase"] == "topology check"
    assert line["runtime"]["HIP_VISIBLE_DEVICES"] == "0,1,2,3" and line["topology"] == {"ok": False}
    assert "rccl_version" in line["runtime"] or "rccl_error" in line["runtime"] or "error" in line["runtime"]


def test_failed_checks_fail_the_n1_run():
    """a wrong C3 or P = 1 result, or a wrong C5 block, makes bench.py exit 1 like a wrong C2; a block
    that raised is reported in the line, not counted as a wrong result."""
    ok = {"self_check": {"ok": True}}
    line = {"self_check": {"ok": True}, "allreduce_1peer": {"result_ok": True},
            "c3": {"i64_max_pair_64MiB": dict(ok), "f32_scan_P8_64MiB": dict(ok)},
            "c4_one_gpu": dict(ok),
            "c5": {"p1_copy": dict(ok), "host_pair_reduce": dict(ok), "local_peers": {"error": "MemoryError"}}}
    assert bench.failed_checks(line) == []
    line["c4_one_gpu"] = "failed: MemoryError: out of memory"  # raised: reported, not a wrong result
    assert bench.failed_checks(line) == []
    line["c3"]["f32_scan_P8_64MiB"] = {"self_check": {"ok": False}}
    line["allreduce_1peer"]["result_ok"] = False
    line["c4_one_gpu"] = {"self_check": {"ok": False}}
    line["c5"]["host_pair_reduce"] = {"self_check": {"ok": False}}
    assert bench.failed_checks(line) == ["allreduce_1peer", "c3 f32_scan_P8_64MiB", "c4_one_gpu",
                                         "c5 host_pair_reduce"]
    line["self_check"]["ok"] = False
    assert bench.failed_checks(line)[0] == "c2"


def test_c5_size_follows_mem_available():
    """C5's 8-peer block runs 8 x 1 GiB page-locked send + recv buckets (16 GiB) when MemAvailable holds them
    with C5_HEADROOM to spare, and halves the bucket until it fits otherwise."""
    G = bench.GIB
    assert bench.c5_size_mib(8, 1024, None) == 1024
    assert bench.c5_size_mib(8, 1024, 64 * G) == 1024
    assert bench.c5_size_mib(8, 1024, 32 * G) == 1024  # 16 + 16 fits exactly
    assert bench.c5_size_mib(8, 1024, 31 * G) == 512
    assert bench.c5_size_mib(8, 1024, 20 * G) == 256


def _light_cpu_baseline(monkeypatch):
    for name in ("c1_host", "c1_reference", "c3_cpu", "c4_reference"):
        monkeypatch.setattr(bench, name, lambda *a, **k: None)
    monkeypatch.setattr(bench, "c2_reference", lambda *a, **k: None)
    import argparse

    return argparse.Namespace(bucket_mib=4, cpu_reps=3)


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "oracle", "build", "cpu_baseline")),
                    reason="oracle/build/cpu_baseline not built (__graft_entry__.build())")
def test_cpu_baseline_value_is_the_reference_combine(monkeypatch):
    """the stated CPU baseline is the reference's own adapter combine (oracle/_ref), the
    port beside it as port_value; value = bucket / reference ms."""
    from oracle import fmi_ref

    if not fmi_ref.available():
        pytest.skip("oracle/_ref not built")
    got = bench.cpu_baseline(_light_cpu_baseline(monkeypatch))
    assert got["kind"] == "reference" and got["cores"] == 1 and got["unit"] == "GiB/s"
    assert got["value"] == pytest.approx(4 / 1024 / (got["reference_combine_ms"] * 1e-3), rel=1e-3)
    assert got["port_value"] > 0 and got["port_combine_ms"] > 0
    assert got["reference_over_port"] == pytest.approx(got["reference_combine_ms"] / got["port_combine_ms"], rel=1e-2)
    assert "reference's own adapter combine" in got["sample"]


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "oracle", "build", "cpu_baseline")),
                    reason="oracle/build/cpu_baseline not built (__graft_entry__.build())")
def test_cpu_baseline_falls_back_to_the_port_only_without_oracle_ref(monkeypatch):
    monkeypatch.setattr(bench, "reference_combine_ms", lambda n, reps: (None, "oracle/_ref not built"))
    got = bench.cpu_baseline(_light_cpu_baseline(monkeypatch))
    assert got["kind"] == "port" and got["value"] == got["port_value"] and got["reference_combine_ms"] is None
    assert got["reference_error"] == "oracle/_ref not built"


def test_line_names_the_bucket_placement():
    """The N = 1 / N > 1 line's config.placement says how the device buckets were placed: plain
    hipMallocs by default (the pair's buckets), the allocator's rotating 4 KiB slots when FMI_TUNE_ALLOC_SLOTS = 1."""
    import fmi_amd

    old = fmi_amd.tune_get(fmi_amd.Tune.ALLOC_SLOTS)
    try:
        assert old == 0 and "plain hipMalloc" in bench.placement()
        fmi_amd.tune_set(fmi_amd.Tune.ALLOC_SLOTS, 1)
        assert "FMI_TUNE_ALLOC_SLOTS = 1" in bench.placement()
        with pytest.raises(fmi_amd.FmiError):
            fmi_amd.tune_set(fmi_amd.Tune.ALLOC_SLOTS, 3)
    finally:
        fmi_amd.tune_set(fmi_amd.Tune.ALLOC_SLOTS, old)


def _emulated_allocator(monkeypatch, rotating):
    """The C-ABI's documented placement rules (include/fmi_dev.h) on fake 2 MiB-aligned bases, no device:
    fmi_dev_alloc puts buckets of >= 1 MiB in slot g++ mod 16 (rotating) or at the base (plain);
    fmi_dev_alloc_group puts bucket j in slot j mod 16."""
    from fmi_amd import _lib

    state = {"base": 1 << 40, "g": 0}

    def base():
        state["base"] += 1 << 30
        return state["base"]

    def call(name, *args):
        if name == "fmi_dev_alloc":
            slot = (state["g"] % 16) if rotating and args[1] >= 1 << 20 else 0
            state["g"] += 1 if rotating and args[1] >= 1 << 20 else 0
            args[0]._obj.value = base() + slot * 4096
        elif name == "fmi_dev_alloc_group":
            for j in range(args[1]):
                args[0][j] = base() + (j % 16) * 4096 * (args[2] >= 1 << 20)
        else:
            raise AssertionError(f"unexpected call {name}")

    monkeypatch.setattr(_lib, "call", call)


@pytest.mark.parametrize("rotating", [0, 1])
def test_c3_scan_sets_give_every_launch_16_distinct_slots(monkeypatch, rotating):
    """whatever was allocated before and whatever FMI_TUNE_ALLOC_SLOTS says, every C3 scan set's
    8 inputs and 8 outputs sit in 16 distinct 4 KiB slots mod 64 KiB (bench.scan_sets allocates each set as one
    group). The order bench.py used in round 5 — every set's inputs, then every set's outputs, one fmi_dev_alloc each
    — gives set s's input p and output p the same slot, the collision the group removes."""
    import numpy as np

    from fmi_amd import Bucket

    _emulated_allocator(monkeypatch, rotating)
    P, S, n = 8, 8, 64 * (1 << 20) // 4
    [Bucket(n, np.float32) for _ in range(5)]  # unrelated allocations before
    ins, outs = bench.scan_sets(S, P, n)
    for s in range(S):
        assert len({(b.ptr % 65536) // 4096 for b in ins[s] + outs[s]}) == 16, s
    old_ins = [[Bucket(n, np.float32) for _ in range(P)] for _ in range(S)]
    old_outs = [[Bucket(n, np.float32) for _ in range(P)] for _ in range(S)]
    for s in range(S):
        assert len({(b.ptr % 65536) // 4096 for b in old_ins[s] + old_outs[s]}) == (8 if rotating else 1)
    for b in [b for g in ins + outs + old_ins + old_outs for b in g]:
        b._owns = False
