"""The reference-side binding mechanics, on the CPU: oracle/_ref runs the REFERENCE's
own src/comm/PeerToPeer.cpp with f.f bound to a C-ABI whose entry points are passed in by address
(oracle/ref_harness.cpp fmi_ref_run_bound). Here the bound entry points are numpy callbacks with the
reference's element semantics, so the test checks the harness mode itself — every recvbuf and sendbuf equal to
the same reference code with its own std functors (fmi_ref_run) — and that the device entry point is refused
for the reference's pageable temporaries instead of being handed a pointer no GPU may read. The same mode bound
to libfmi_dev.so on MI355X is tests/test_gpu_ref_binding.py.
"""
import ctypes

import numpy as np
import pytest

from oracle import fmi_ref as ref

pytestmark = pytest.mark.skipif(not ref.available(), reason="oracle/_ref not built (make -C oracle)")

NP = {0: np.float32, 1: np.float64, 2: np.int32, 3: np.int64, 4: np.uint32, 5: np.uint64}
CT = {0: ctypes.c_float, 1: ctypes.c_double, 2: ctypes.c_int32, 3: ctypes.c_int64, 4: ctypes.c_uint32,
      5: ctypes.c_uint64}


def _combine(op, dtype, a, b, n):
    """a = op(a, b) with the reference's built-ins: std::plus / multiplies, std::max = (a < b) ? b : a,
    std::min = (b < a) ? b : a (python/PythonCommunicator.h:131-149)."""
    if n == 0:
        return 0
    x = np.ctypeslib.as_array(ctypes.cast(a, ctypes.POINTER(CT[dtype])), shape=(n,))
    y = np.ctypeslib.as_array(ctypes.cast(b, ctypes.POINTER(CT[dtype])), shape=(n,))
    with np.errstate(all="ignore"):
        if op == 0:
            x[:] = x + y
        elif op == 1:
            x[:] = x * y
        elif op == 2:
            x[:] = np.where(x < y, y, x)
        else:
            x[:] = np.where(y < x, y, x)
    return 0


CALLS = {"host": 0, "dev": 0}


@ref.HOST_PAIR
def _host_pair(op, dtype, a, b, n):
    CALLS["host"] += 1
    return _combine(op, dtype, a, b, n)


@ref.DEV_PAIR
def _dev_pair(op, dtype, a, b, n, stream):
    CALLS["dev"] += 1
    return _combine(op, dtype, a, b, n)


@ref.STREAM_SYNC
def _sync(stream):
    return 0


_MSG = ctypes.create_string_buffer(b"numpy binding")


@ref.LAST_ERROR
def _last_error():
    return ctypes.addressof(_MSG)


def _binding(device_entry=False):
    addr = lambda f: ctypes.cast(f, ctypes.c_void_p).value  # noqa: E731
    return ref.Binding(addr(_host_pair), addr(_dev_pair) if device_entry else None, addr(_sync), addr(_last_error))


def _inputs(dtype, P, n, seed):
    rng = np.random.default_rng(seed)
    if np.issubdtype(dtype, np.floating):
        xs = rng.standard_normal((P, n)).astype(dtype) * rng.choice([1e-3, 1.0, 1e3], size=(P, 1)).astype(dtype)
        xs[:, :4] = np.array([0.0, -0.0, np.inf, np.nan], dtype)[None, :] if n >= 4 else xs[:, :4]
        return xs
    return rng.integers(np.iinfo(dtype).min, np.iinfo(dtype).max, size=(P, n), dtype=dtype, endpoint=True)


def _eq(got, want, what):
    u = {4: np.uint32, 8: np.uint64}[got.dtype.itemsize]
    same = got.view(u) == want.view(u)
    if np.issubdtype(got.dtype, np.floating):
        same |= np.isnan(got) & np.isnan(want)
    assert same.all(), f"{what}: {np.count_nonzero(~same)} elements differ"


@pytest.mark.parametrize("P", [1, 2, 3, 5, 8, 13])
@pytest.mark.parametrize("dt", [0, 1, 3])
def test_bound_host_entry_equals_reference_functors(P, dt):
    dtype = NP[dt]
    xs = _inputs(dtype, P, 37, seed=P * 10 + dt)
    b = _binding()
    for op in ("sum", "prod", "max", "min"):
        for ordered in (False, True):
            for coll, roots in (("allreduce", [0]), ("scan", [0]), ("reduce", range(P))):
                for root in roots:
                    want_r, want_s, _ = ref.run(coll, op, xs, root=root, ordered=ordered)
                    got_r, got_s = ref.run_bound(coll, op, xs, b, root=root, ordered=ordered)
                    what = f"{coll} {op} P={P} ordered={ordered} root={root}"
                    _eq(got_r, want_r, what + " recvbufs")
                    _eq(got_s, want_s, what + " sendbufs")


def test_bound_combine_is_called_at_every_reference_site():
    """The bound entry point is the combine: the reference's 8-peer allreduce makes 3 combines per peer
    (recursive doubling, PeerToPeer.cpp:119), its reduce 7 (binomial tree, :72), scan_ltr 7 (:147)."""
    xs = _inputs(np.float32, 8, 16, seed=1)
    b = _binding()
    for coll, ordered, calls in (("allreduce", False, 24), ("reduce", False, 7), ("scan", True, 7)):
        CALLS["host"] = 0
        ref.run_bound(coll, "sum", xs, b, ordered=ordered)
        assert CALLS["host"] == calls, (coll, CALLS["host"])


def test_device_entry_on_caller_buckets_and_refused_on_reference_temporaries():
    """Device entry point: the caller's buckets only. allreduce (commutative) and scan combine only the caller's
    sendbuf / recvbuf (PeerToPeer.cpp:103,119,147,160,179) and match; reduce combines into the reference's own
    `new char[]` temporaries (:47,63), which the harness refuses to hand to a device entry point."""
    P, n = 5, 33
    xs = _inputs(np.float64, P, n, seed=3)
    bufs = [np.zeros(n, np.float64) for _ in range(2 * P)]
    addrs = [a.ctypes.data for a in bufs]
    b = _binding(device_entry=True)
    for coll, ordered in (("allreduce", False), ("scan", False), ("scan", True)):
        CALLS["dev"] = CALLS["host"] = 0
        want_r, want_s, _ = ref.run(coll, "sum", xs, ordered=ordered)
        got_r, got_s = ref.run_bound(coll, "sum", xs, b, ordered=ordered, bufs=addrs)
        _eq(got_r, want_r, f"{coll} ordered={ordered} recvbufs")
        _eq(got_s, want_s, f"{coll} ordered={ordered} sendbufs")
        assert CALLS["dev"] > 0 and CALLS["host"] == 0
    for coll, ordered in (("reduce", False), ("reduce", True), ("allreduce", True)):
        with pytest.raises(ref.RefError, match="not a device-mapped bucket"):
            ref.run_bound(coll, "sum", xs, b, ordered=ordered, bufs=addrs)
    with pytest.raises(ref.RefError, match="invalid argument"):  # the device entry point needs caller buckets
        ref.run_bound("allreduce", "sum", xs, b)


def test_bound_failure_surfaces_the_library_message():
    @ref.HOST_PAIR
    def failing(op, dtype, a, b, n):
        return -2

    addr = lambda f: ctypes.cast(f, ctypes.c_void_p).value  # noqa: E731
    b = ref.Binding(addr(failing), None, addr(_sync), addr(_last_error))
    with pytest.raises(ref.RefError, match=r"bound combine failed \(-2\): numpy binding"):
        ref.run_bound("allreduce", "sum", _inputs(np.float32, 2, 8, seed=0), b)


def test_bound_timing_runs():
    ms = ref.time_allreduce_bound(2, 1024, 3, _binding())
    assert ms > 0
