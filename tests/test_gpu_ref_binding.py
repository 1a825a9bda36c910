"""The REFERENCE's own collective code driving the HIP combine through the C-ABI.

oracle/_ref runs /root/reference/src/comm/PeerToPeer.cpp, compiled unmodified, over an in-memory transport;
its mode fmi_ref_run_bound makes every f.f(a, b) at the reference's combine sites (PeerToPeer.cpp:51,72,103,
119,147,160,179) the raw_func §B.2 builds (include/Communicator.h:180-189 replaced): a call, by address, of
the product's exported entry point —
  * host entry point: fmi_host_reduce_pair on whatever the reference hands the combine (the peers' pageable
    buckets and the reference's own `new char[]` temporaries: the staged H2D / kernel / D2H path; page-locked
    caller buckets: the zero-copy kernel over PCIe);
  * device entry point: fmi_dev_reduce_pair on the library stream + fmi_stream_sync, on page-locked, mapped
    caller buckets the GPU addresses directly (the collectives whose combines touch only the caller's buckets:
    commutative allreduce, scan; the reference's reduce combines into its own pageable temporaries, which the
    harness refuses to hand to a device entry point — tests/test_ref_binding.py).
The library is libfmi_dev.so as the product loads it (fmi_amd._lib); oracle/_ref links nothing of it and the
product never loads oracle/_ref. Bar: every peer's recvbuf AND sendbuf bit-identical to the same reference code
with its CPU combine (std functors, fmi_ref_run); a NaN matches any NaN (tests/test_gpu_parity.assert_bit_equal).
"""
import ctypes

import numpy as np
import pytest

import fmi_amd
from fmi_amd import PinnedArray, _lib
from oracle import fmi_ref as ref
from tests.test_gpu_parity import assert_bit_equal, inputs

pytestmark = pytest.mark.gpu

OPS = ("sum", "prod", "max", "min")
PEERS = (2, 3, 5, 8, 13)
DTYPES = (np.float32, np.float64, np.int64)
N = 1031  # ragged: no multiple of the kernels' 16-B vectors


@pytest.fixture(scope="module")
def binding(device):
    assert ref.available(), "oracle/_ref/libfmi_ref.so must travel with the tree (make -C oracle)"
    return ref.Binding.from_library(_lib.load())


@pytest.fixture(scope="module")
def device_binding(device):
    return ref.Binding.from_library(_lib.load(), device_entry=True)


def _peers(dtype, P, n, seed=0):
    return np.stack([inputs(dtype, n, peer=p, seed=seed + 17) for p in range(P)])


def _check(got, want, what):
    for p in range(got[0].shape[0]):
        assert_bit_equal(got[0][p], want[0][p], f"{what}: recvbuf of peer {p}")
        assert_bit_equal(got[1][p], want[1][p], f"{what}: sendbuf of peer {p}")


@pytest.mark.parametrize("P", PEERS)
@pytest.mark.parametrize("dtype", DTYPES, ids=lambda d: np.dtype(d).name)
def test_reference_collectives_through_host_entry(binding, P, dtype):
    """Reference allreduce / reduce (every root) / scan, commutative and left-to-right, 4 ops: f.f is
    fmi_host_reduce_pair on the reference's pageable buckets and temporaries."""
    xs = _peers(dtype, P, N, seed=P)
    for op in OPS:
        for ordered in (False, True):
            for coll, roots in (("allreduce", [0]), ("scan", [0]), ("reduce", range(P))):
                for root in roots:
                    want = ref.run(coll, op, xs, root=root, ordered=ordered)[:2]
                    got = ref.run_bound(coll, op, xs, binding, root=root, ordered=ordered)
                    _check(got, want, f"{coll} {op} P={P} ordered={ordered} root={root}")


def _pinned_buckets(P, n, dtype):
    bufs = [PinnedArray(n, dtype) for _ in range(2 * P)]
    return bufs, [b.ptr for b in bufs]


def _assert_device_addressable(ptrs, nbytes):
    """The device entry point hands the caller's host pointers to a kernel: each must be the address the GPU
    maps the page-locked bucket at (fmi_host_device_ptr), checked before any launch."""
    for p in ptrs:
        dp = ctypes.c_void_p()
        _lib.call("fmi_host_device_ptr", p, nbytes, ctypes.byref(dp))
        assert dp.value == p, "page-locked bucket is mapped at another device address"


@pytest.mark.parametrize("P", PEERS)
def test_reference_collectives_on_pinned_buckets(binding, device_binding, P):
    """Page-locked caller buckets: the host entry point takes its zero-copy kernel path where both operands
    are the caller's (and stages the reference's temporaries); the device entry point (fmi_dev_reduce_pair +
    fmi_stream_sync) runs the commutative allreduce and both scans on them directly."""
    for dtype in DTYPES:
        xs = _peers(dtype, P, N, seed=100 + P)
        bufs, ptrs = _pinned_buckets(P, N, dtype)
        try:
            _assert_device_addressable(ptrs, N * np.dtype(dtype).itemsize)
            for op in OPS:
                for ordered in (False, True):
                    for coll, roots in (("allreduce", [0]), ("scan", [0]), ("reduce", range(P))):
                        for root in roots:
                            want = ref.run(coll, op, xs, root=root, ordered=ordered)[:2]
                            what = f"{np.dtype(dtype).name} {coll} {op} P={P} ordered={ordered} root={root}"
                            got = ref.run_bound(coll, op, xs, binding, root=root, ordered=ordered, bufs=ptrs)
                            _check(got, want, "host entry, pinned: " + what)
                            if coll == "reduce" or (coll == "allreduce" and ordered):
                                continue  # combines into the reference's pageable temporaries
                            got = ref.run_bound(coll, op, xs, device_binding, ordered=ordered, bufs=ptrs)
                            _check(got, want, "device entry, pinned: " + what)
        finally:
            for b in bufs:
                b.free()


def test_c1_shape_through_both_entries(binding, device_binding):
    """Config C1's shape: the reference's 2-peer f32 sum-allreduce of 1 MiB buckets, its combine on the GPU."""
    n = (1 << 20) // 4
    xs = _peers(np.float32, 2, n, seed=7)
    want = ref.run("allreduce", "sum", xs)[:2]
    _check(ref.run_bound("allreduce", "sum", xs, binding), want, "C1 host entry, pageable")
    bufs, ptrs = _pinned_buckets(2, n, np.float32)
    try:
        _assert_device_addressable(ptrs, n * 4)
        _check(ref.run_bound("allreduce", "sum", xs, binding, bufs=ptrs), want, "C1 host entry, pinned")
        _check(ref.run_bound("allreduce", "sum", xs, device_binding, bufs=ptrs), want, "C1 device entry, pinned")
    finally:
        for b in bufs:
            b.free()
    ms = ref.time_allreduce_bound(2, n, 5, binding)
    assert ms > 0


def test_library_errors_reach_the_reference_caller(binding):
    """A failing combine surfaces as the reference collective's failure, carrying the library's message. The
    harness validates op ids itself, so the bad op is injected below it: an entry point that forwards to
    fmi_host_reduce_pair with op 9."""
    host = ctypes.cast(binding.host_pair, ref.HOST_PAIR)

    @ref.HOST_PAIR
    def bad_op(op, dtype, a, b, n):
        return host(9, dtype, a, b, n)

    b = ref.Binding(ctypes.cast(bad_op, ctypes.c_void_p).value, None, binding.stream_sync, binding.last_error)
    with pytest.raises(ref.RefError, match="unknown op 9"):
        ref.run_bound("allreduce", "sum", _peers(np.float32, 2, 64), b)


def test_host_device_ptr(device):
    """fmi_host_device_ptr: the device address of a page-locked range (the same address for fmi_host_pin_alloc
    memory on MI355X); a pageable range is refused."""
    a = PinnedArray(1024, np.float32)
    try:
        dp = ctypes.c_void_p()
        _lib.call("fmi_host_device_ptr", a.ptr + 64, 512, ctypes.byref(dp))
        assert dp.value == a.ptr + 64
        pageable = np.zeros(1024, np.float32)
        with pytest.raises(fmi_amd.FmiError, match="page-locked"):
            _lib.call("fmi_host_device_ptr", pageable.ctypes.data, 64, ctypes.byref(dp))
    finally:
        a.free()
