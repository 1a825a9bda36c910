"""bench.py's host-side contract (CPU): the JSON line is printed exactly once, and the per-rank deadline
over the after-`value` section (C4, C5 and the diagnostics) prints the measured line, marked "incomplete" at
top level, and exits when that section hangs."""
import json
import os
import subprocess
import sys
import textwrap

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
