"""CPU-side checks of the C-ABI boundary: the library loads, exports every symbol include/fmi_dev.h
declares, reports errors through status codes + fmi_last_error, and its host-only logic (schedules,
tuning validation) is right. No compute call is made here (no GPU in this container)."""
import ctypes
import os
import re

import pytest

import fmi_amd
from fmi_amd import _lib
from fmi_amd.device import Alg
from oracle import fmi_oracle as orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    text = open(os.path.join(ROOT, "include", "fmi_dev.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(fmi_\w+)\s*\(", text, flags=re.M)))


def test_header_declares_expected_surface():
    syms = _declared_symbols()
    for must in ["fmi_dev_reduce_pair", "fmi_dev_reduce_tree", "fmi_dev_scan_peers", "fmi_host_reduce_pair",
                 "fmi_dev_init", "fmi_last_error", "fmi_dev_fill_synthetic", "fmi_schedule_expr"]:
        assert must in syms
    assert len(syms) >= 30


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    missing = [s for s in _declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    # and the ctypes signature table covers all of them
    assert sorted(_lib.SIGNATURES) == _declared_symbols()


def test_abi_version():
    assert _lib.load().fmi_abi_version() == 1


def test_calls_without_device_fail_loudly():
    lib = _lib.load()
    c = ctypes.c_int(-1)
    assert lib.fmi_dev_count(ctypes.byref(c)) == 0
    if c.value > 0:
        pytest.skip("a device is visible; this test is for GPU-less hosts")
    assert lib.fmi_dev_init(0) == _lib.FMI_ERR_NO_DEVICE
    assert "no HIP device" in _lib.last_error()
    # compute entry points refuse without an initialised gfx950 device (no CPU fallback)
    assert lib.fmi_dev_reduce_pair(0, 0, None, None, 16, None) == _lib.FMI_ERR_NO_DEVICE
    with pytest.raises(fmi_amd.FmiError):
        fmi_amd.init(0)


def test_argument_validation_is_host_side():
    lib = _lib.load()
    assert lib.fmi_dev_reduce_tree(9, 0, 0, None, None, 2, 0, 8, None) == _lib.FMI_ERR_INVALID
    assert "unknown op" in _lib.last_error()
    assert lib.fmi_dev_reduce_tree(0, 7, 0, None, None, 2, 0, 8, None) == _lib.FMI_ERR_INVALID
    assert lib.fmi_dev_reduce_tree(0, 0, 0, None, None, 0, 0, 8, None) == _lib.FMI_ERR_INVALID
    assert lib.fmi_dev_reduce_tree(0, 0, 3, None, None, 2, 0, 8, None) == _lib.FMI_ERR_INVALID
    assert lib.fmi_dev_scan_peers(0, 0, 0, None, None, 2, 8, None) == _lib.FMI_ERR_INVALID
    assert lib.fmi_host_reduce_pair(0, 0, None, None, 0) == 0  # empty bucket is a no-op


def test_comm_host_side_without_device():
    """Communicator ids and LOCAL-transport joins are host logic; collectives refuse without a device."""
    from fmi_amd.comm import Comm, Transport, unique_id

    a, b = unique_id(Transport.LOCAL), unique_id(Transport.LOCAL)
    assert len(a) == 128 and a != b and a[:8] == b"FMILOCAL"
    c0, c1 = Comm(a, 2, 0), Comm(a, 2, 1)
    lib = _lib.load()
    c = ctypes.c_int(-1)
    lib.fmi_dev_count(ctypes.byref(c))
    if c.value == 0:
        assert lib.fmi_comm_barrier(ctypes.c_void_p(c0.handle), None) == _lib.FMI_ERR_NO_DEVICE
    assert lib.fmi_comm_allreduce(ctypes.c_void_p(c0.handle), 9, 0, 0, 0, None, None, 8, None) == _lib.FMI_ERR_INVALID
    with pytest.raises(fmi_amd.FmiError):
        Comm(a, 3, 0)  # joining a 2-rank communicator as a 3-rank one
    with pytest.raises(fmi_amd.FmiError):
        Comm(a, 2, 2)  # rank out of range
    Comm(unique_id(Transport.LOCAL), 1000, 0).destroy()  # no rank cap (reference: any num_peers)
    c0.destroy()
    c1.destroy()


_PROC_JOIN = """
import sys
from fmi_amd.comm import Comm
c = Comm(bytes.fromhex(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]))
c.destroy()
"""


def test_proc_transport_join_and_timeout():
    """PROC ids carry their magic; N processes join one shared-memory segment (a host barrier) and the
    name is unlinked once all hold it; a rank whose peers never arrive raises the reference's Timeout
    (FMI_ERR_TIMEOUT -> fmi_amd.Timeout, include/utils/Common.h:11-15), not a hang."""
    import subprocess
    import sys

    from fmi_amd.comm import Transport, unique_id

    a, b = unique_id(Transport.PROC), unique_id(Transport.PROC)
    assert a[:8] == b"FMIPROC\0" and a != b
    shm = "/dev/shm/fmi_proc_%016x" % int.from_bytes(a[8:16], "little")
    env = dict(os.environ, FMI_PROC_TIMEOUT_S="20")
    procs = [subprocess.Popen([sys.executable, "-c", _PROC_JOIN, a.hex(), "3", str(r)], cwd=ROOT, env=env)
             for r in range(3)]
    assert [p.wait(timeout=120) for p in procs] == [0, 0, 0]
    assert not os.path.exists(shm)
    env["FMI_PROC_TIMEOUT_S"] = "1"
    lone = subprocess.run([sys.executable, "-c", _PROC_JOIN, b.hex(), "2", "0"], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=120)
    assert lone.returncode != 0 and "Timeout was reached" in lone.stderr, lone.stderr
    assert "fmi_amd._lib.Timeout: FMI_ERR_TIMEOUT" in lone.stderr and "waiting for peers (join)" in lone.stderr
    assert not os.path.exists("/dev/shm/fmi_proc_%016x" % int.from_bytes(b[8:16], "little"))


def test_tuning_knobs_validate():
    fmi_amd.tune_set(fmi_amd.Tune.PAIR_UNROLL, 8)
    assert fmi_amd.tune_get(fmi_amd.Tune.PAIR_UNROLL) == 8
    fmi_amd.tune_set(fmi_amd.Tune.PAIR_UNROLL, 4)
    with pytest.raises(fmi_amd.FmiError):
        fmi_amd.tune_set(fmi_amd.Tune.PAIR_UNROLL, 3)
    with pytest.raises(fmi_amd.FmiError):
        fmi_amd.tune_set(fmi_amd.Tune.BLOCK, 100)
    assert fmi_amd.tune_get(fmi_amd.Tune.FUSED_INFLIGHT_KIB) == 64  # default (tools/ab_fused_cap.py)
    fmi_amd.tune_set(fmi_amd.Tune.FUSED_INFLIGHT_KIB, 0)
    assert fmi_amd.tune_get(fmi_amd.Tune.FUSED_INFLIGHT_KIB) == 0
    fmi_amd.tune_set(fmi_amd.Tune.FUSED_INFLIGHT_KIB, 64)
    with pytest.raises(fmi_amd.FmiError):
        fmi_amd.tune_set(fmi_amd.Tune.FUSED_INFLIGHT_KIB, -1)
    assert fmi_amd.tune_get(fmi_amd.Tune.BLOCKS_ONE_PASS) == 1  # default: one pass over every input
    fmi_amd.tune_set(fmi_amd.Tune.BLOCKS_ONE_PASS, 0)
    assert fmi_amd.tune_get(fmi_amd.Tune.BLOCKS_ONE_PASS) == 0
    fmi_amd.tune_set(fmi_amd.Tune.BLOCKS_ONE_PASS, 1)
    with pytest.raises(fmi_amd.FmiError):
        fmi_amd.tune_set(fmi_amd.Tune.BLOCKS_ONE_PASS, 2)
    assert fmi_amd.tune_get(fmi_amd.Tune.FUSED_POLICY) == 1  # default: per kernel (tools/ab_fused_policy.py)
    for v in (0, 2, 1):
        fmi_amd.tune_set(fmi_amd.Tune.FUSED_POLICY, v)
        assert fmi_amd.tune_get(fmi_amd.Tune.FUSED_POLICY) == v
    with pytest.raises(fmi_amd.FmiError):
        fmi_amd.tune_set(fmi_amd.Tune.FUSED_POLICY, 3)
    assert fmi_amd.tune_get(fmi_amd.Tune.PAIR_SC1_OF_8) == 1  # default (tools/ab_pair_sc1.py)
    for v in (0, 8, 1):
        fmi_amd.tune_set(fmi_amd.Tune.PAIR_SC1_OF_8, v)
        assert fmi_amd.tune_get(fmi_amd.Tune.PAIR_SC1_OF_8) == v
    for bad in (-1, 9):
        with pytest.raises(fmi_amd.FmiError):
            fmi_amd.tune_set(fmi_amd.Tune.PAIR_SC1_OF_8, bad)
    for key in (fmi_amd.Tune.COMM_A2A, fmi_amd.Tune.COMM_GATHER, fmi_amd.Tune.COMM_ONE_RANK_EXCHANGE):
        assert fmi_amd.tune_get(key) == 0
        fmi_amd.tune_set(key, 1)
        assert fmi_amd.tune_get(key) == 1
        fmi_amd.tune_set(key, 0)
        with pytest.raises(fmi_amd.FmiError):
            fmi_amd.tune_set(key, 2)


@pytest.mark.parametrize("P", list(range(1, 34)) + [48, 64, 100, 129, 256])
def test_kernel_schedules_match_oracle(P):
    """The programs the fused kernels execute (fmi_schedule.h, round-synchronous) against the oracle's
    event-driven message simulation of the reference algorithms — for every rank and root."""
    for r in range(P):
        assert fmi_amd.schedule_expr(Alg.ALLREDUCE, P, r) == orc.expr("allreduce", P, rank=r)
        assert fmi_amd.schedule_expr(Alg.SCAN, P, r) == orc.expr("scan", P, rank=r)
        assert fmi_amd.schedule_expr(Alg.SCAN_LTR, P, r) == orc.expr("scan", P, rank=r, ordered=True)
        assert fmi_amd.schedule_expr(Alg.REDUCE_LTR, P, r) == orc.expr("reduce", P, root=r, ordered=True)
        # reduce programs are in transformed ids (root -> 0); map back to real ids
        t = fmi_amd.schedule_expr(Alg.REDUCE, P, 0)
        real = re.sub(r"x(\d+)", lambda m: "x%d" % ((int(m.group(1)) + r) % P), t)
        assert real == orc.expr("reduce", P, root=r)
        if P > 16:
            break  # larger P: one rank is enough, the oracle simulation is O(P^2 log P) per call


def test_allreduce_power_of_two_is_xor_symmetric():
    """For P = 2^k the value peer r holds is rank 0's expression over inputs x[p ^ r], operand order
    included: what lets fmi_fused_allreduce.hip run the rank-0 kernel over permuted pointers."""
    for P in (2, 4, 8, 16, 32, 64, 128, 256):
        e0 = fmi_amd.schedule_expr(Alg.ALLREDUCE, P, 0)
        for r in range(P):
            want = re.sub(r"x(\d+)", lambda m: "x%d" % (int(m.group(1)) ^ r), e0)
            assert fmi_amd.schedule_expr(Alg.ALLREDUCE, P, r) == want, (P, r)


@pytest.mark.parametrize("P", [257, 300, 512, 1000])
def test_schedules_beyond_256_peers_match_oracle(P):
    """No peer cap: the run-time-sized host programs (fmi_schedule.h HostProgram) for P > 256 against the
    oracle's message simulation — a few ranks / roots per algorithm."""
    for r in (0, 1, P // 2 + 1, P - 1):
        assert fmi_amd.schedule_expr(Alg.ALLREDUCE, P, r) == orc.expr("allreduce", P, rank=r)
        assert fmi_amd.schedule_expr(Alg.SCAN, P, r) == orc.expr("scan", P, rank=r)
        assert fmi_amd.schedule_expr(Alg.SCAN_LTR, P, r) == orc.expr("scan", P, rank=r, ordered=True)
        assert fmi_amd.schedule_expr(Alg.REDUCE_LTR, P, r) == orc.expr("reduce", P, root=r, ordered=True)
        t = fmi_amd.schedule_expr(Alg.REDUCE, P, 0)
        real = re.sub(r"x(\d+)", lambda m: "x%d" % ((int(m.group(1)) + r) % P), t)
        assert real == orc.expr("reduce", P, root=r)


def test_schedule_expr_rejects_bad_args():
    with pytest.raises(fmi_amd.FmiError):
        fmi_amd.schedule_expr(Alg.ALLREDUCE, 0, 0)
    with pytest.raises(fmi_amd.FmiError):
        fmi_amd.schedule_expr(Alg.ALLREDUCE, 4, 4)


def _offload_bundles(data: bytes):
    """The offload bundles of a .hip_fatbin section, one per translation unit: compressed ("CCOB" header,
    version 2/3: the bundle's total size at byte 8, 32- or 64-bit; the library is built with
    --offload-compress) or plain ("__CLANG_OFFLOAD_BUNDLE__", running to the next magic)."""
    import struct

    plain = b"__CLANG_OFFLOAD_BUNDLE__"
    pos, out = 0, []
    while True:
        c, p = data.find(b"CCOB", pos), data.find(plain, pos)
        starts = [x for x in (c, p) if x >= 0]
        if not starts:
            return out
        pos = min(starts)
        if pos == c:
            version = struct.unpack_from("<H", data, pos + 4)[0]
            total = struct.unpack_from("<Q" if version >= 3 else "<I", data, pos + 8)[0]
            out.append(data[pos:pos + total])
            pos += total
        else:
            nxt = [x for x in (data.find(b"CCOB", pos + 1), data.find(plain, pos + 1)) if x >= 0]
            end = min(nxt) if nxt else len(data)
            out.append(data[pos:end])
            pos = end


def test_no_kernel_spills_to_scratch(tmp_path):
    """Every gfx950 kernel in libfmi_dev.so keeps its values in registers: .private_segment_fixed_size is 0
    for all of them (fused programs index their value arrays with constants only; a select chain over
    that array, or a per-byte loop, once put it in scratch)."""
    import subprocess

    llvm = "/opt/rocm/lib/llvm/bin"
    if not os.path.exists(os.path.join(llvm, "clang-offload-bundler")):
        pytest.skip("ROCm LLVM tools not installed")
    fat = tmp_path / "fatbin"
    subprocess.run([os.path.join(llvm, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", _lib.LIB_PATH,
                    str(tmp_path / "lib.so")], check=True)
    data = fat.read_bytes()
    kernels = spilled = 0
    for k, bundle in enumerate(_offload_bundles(data)):
        b, elf = tmp_path / f"b{k}", tmp_path / f"b{k}.elf"
        b.write_bytes(bundle)
        subprocess.run([os.path.join(llvm, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={b}",
                        f"--output={elf}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"], check=True)
        notes = subprocess.run([os.path.join(llvm, "llvm-readelf"), "--notes", str(elf)], check=True,
                               capture_output=True, text=True).stdout
        sizes = re.findall(r"private_segment_fixed_size:\s+(\d+)", notes)
        kernels += len(sizes)
        spilled += sum(1 for v in sizes if v != "0")
    assert kernels > 2000 and spilled == 0, f"{spilled} of {kernels} kernels use scratch"


def test_header_contract_matches_the_tests():
    """The C-ABI header states the contract the GPU tests assert (it once said 'rank 0's
    operand order' while the tests assert each rank's own order): each rank keeps its own operand order;
    `send` is left untouched by allreduce / reduce / scan (tests/test_gpu_comm.py "send bucket untouched"),
    and fmi_comm_reduce_sendbuf reproduces the reference's sendbuf partials
    (test_comm_reduce_sendbuf_partials)."""
    hdr = open(os.path.join(ROOT, "include", "fmi_dev.h")).read()
    rccl = open(os.path.join(ROOT, "fmi_amd", "cpp", "include", "fmi", "comm", "Rccl.h")).read()
    flat = " ".join(re.sub(r"^\s*\*\s?", "", hdr, flags=re.M).split())
    assert "rank 0's operand order" not in hdr and "rank 0's operand order" not in rccl
    assert "each rank with its OWN operand order" in flat
    assert "`send` is never modified by allreduce, reduce or scan" in flat
    assert "fmi_comm_reduce_sendbuf" in hdr and "fmi_comm_reduce_sendbuf" in rccl
    gpu_tests = open(os.path.join(ROOT, "tests", "test_gpu_comm.py")).read()
    assert "send bucket untouched" in gpu_tests and "plain reduce leaves send untouched" in gpu_tests


@pytest.mark.parametrize("seed", range(4))
def test_programs_combine_every_input_exactly_once(seed):
    """Structure of the run-time-sized programs at random P up to 2,000 (no peer cap): every reduce /
    allreduce result combines each of the P inputs exactly once, and scan output k exactly the inputs 0..k
    (the reference's semantics, whatever the bracketing), for random ranks / roots."""
    import collections
    import random

    rng = random.Random(seed)
    for _ in range(6):
        P = rng.randint(1, 2000)
        r = rng.randrange(P)
        for alg in (Alg.ALLREDUCE, Alg.REDUCE_LTR):
            leaves = collections.Counter(int(x) for x in re.findall(r"x(\d+)", fmi_amd.schedule_expr(alg, P, r)))
            assert leaves == collections.Counter(range(P)), (alg, P, r)
        # reduce works on transformed ids: id 0 (the root) ends with every input; id t > 0 with its binomial
        # subtree t .. t + 2^(trailing zeros of t) - 1 (the partial it forwarded, PeerToPeer.cpp:72)
        t = r
        span = P if t == 0 else (t & -t)
        leaves = collections.Counter(int(x) for x in re.findall(r"x(\d+)", fmi_amd.schedule_expr(Alg.REDUCE, P, t)))
        assert leaves == collections.Counter(range(t, min(P, t + span))), (P, t)
        for alg in (Alg.SCAN, Alg.SCAN_LTR):
            leaves = collections.Counter(int(x) for x in re.findall(r"x(\d+)", fmi_amd.schedule_expr(alg, P, r)))
            assert leaves == collections.Counter(range(r + 1)), (alg, P, r)


def test_python_enums_match_the_header():
    """Every enumerator the C-ABI header defines has the same value in the Python binding (a binding that
    drifts from include/fmi_dev.h would pass wrong ops, dtypes or tuning keys through ctypes silently)."""
    import re

    from fmi_amd.comm import Path, Transport

    text = open(os.path.join(ROOT, "include", "fmi_dev.h")).read()
    consts = {m.group(1): int(m.group(2)) for m in re.finditer(r"\b(FMI_[A-Z0-9_]+)\s*=\s*(\d+)", text)}
    groups = [(fmi_amd.Op, "FMI_OP_"), (fmi_amd.DType, "FMI_"), (fmi_amd.Alg, "FMI_ALG_"), (Transport, "FMI_TRANSPORT_"),
              (Path, "FMI_PATH_"), (fmi_amd.Tune, "FMI_TUNE_")]
    for enum_cls, prefix in groups:
        for member in enum_cls:
            name = prefix + member.name
            assert name in consts, f"{name} missing from include/fmi_dev.h"
            assert consts[name] == int(member), f"{name}: header {consts[name]}, Python {int(member)}"
        declared = {k for k in consts if k.startswith(prefix)}
        if prefix not in ("FMI_",):  # every header enumerator of the group is bound in Python
            assert declared == {prefix + m.name for m in enum_cls}, (prefix, declared ^ {prefix + m.name for m in enum_cls})


def test_host_out_of_memory_is_a_status_not_a_crash():
    """No C++ exception crosses the C-ABI (include/fmi_dev.h entry points run under a guard): building a
    16,777,216-peer allreduce program under a 3 GiB address-space limit throws std::bad_alloc inside the
    library, which must come back as FMI_ERR_ALLOC with a message instead of std::terminate killing the caller.
    Not under AddressSanitizer (tools/sanitize_lib.sh): its shadow memory cannot live in a 3 GiB address space."""
    import subprocess
    import sys

    if "asan" in os.environ.get("LD_PRELOAD", ""):
        pytest.skip("AddressSanitizer's shadow memory does not fit an RLIMIT_AS of 3 GiB")

    code = (f"import resource, ctypes, sys\nsys.path.insert(0, {ROOT!r})\n"
            "from fmi_amd import _lib\nlib = _lib.load()\n"
            "resource.setrlimit(resource.RLIMIT_AS, (3 << 30, 3 << 30))\n"
            "buf = ctypes.create_string_buffer(64)\n"
            "rc = lib.fmi_schedule_expr(0, 1 << 24, 0, buf, 64)\n"
            "print(rc, _lib.last_error())\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.split()[0] == str(_lib.FMI_ERR_ALLOC) and "out of host memory" in r.stdout


def test_pci_bus_id_and_comm_query_host_side():
    """fmi_dev_pci_bus_id refuses a device that is not there (FMI_ERR_NO_DEVICE, no crash); fmi_comm_query on a
    LOCAL communicator reports its own size and rank (host logic); both refuse null arguments."""
    from fmi_amd.comm import Comm, Transport, unique_id

    lib = _lib.load()
    buf = ctypes.create_string_buffer(64)
    assert lib.fmi_dev_pci_bus_id(4096, buf, 64) == _lib.FMI_ERR_NO_DEVICE
    assert lib.fmi_dev_pci_bus_id(0, None, 64) == _lib.FMI_ERR_INVALID
    uid = unique_id(Transport.LOCAL)
    c0, c1 = Comm(uid, 2, 0), Comm(uid, 2, 1)
    cnt, rk, dev = ctypes.c_int(-1), ctypes.c_int(-1), ctypes.c_int(-1)
    assert lib.fmi_comm_query(ctypes.c_void_p(c1.handle), None, ctypes.byref(rk), ctypes.byref(dev)) == _lib.FMI_ERR_INVALID
    rc = lib.fmi_comm_query(ctypes.c_void_p(c1.handle), ctypes.byref(cnt), ctypes.byref(rk), ctypes.byref(dev))
    c = ctypes.c_int(0)
    lib.fmi_dev_count(ctypes.byref(c))
    if c.value == 0:  # no device: hipGetDevice fails after the size and rank are known
        assert rc in (_lib.FMI_OK, _lib.FMI_ERR_HIP)
    else:
        assert rc == _lib.FMI_OK
    assert (cnt.value, rk.value) == (2, 1)
    assert lib.fmi_comm_sync(ctypes.c_void_p(c0.handle), None) in (_lib.FMI_OK, _lib.FMI_ERR_NO_DEVICE)
    c0.destroy()
    c1.destroy()
