"""ORACLE — TEST INFRASTRUCTURE ONLY. ctypes access to oracle/_ref/libfmi_ref.so: the REFERENCE's own
src/comm/PeerToPeer.cpp (compiled unmodified from /root/reference by oracle/Makefile) running over an in-memory
PeerToPeer transport (oracle/ref_harness.cpp). Imported only by tests/, tests/golden/make_ref_vectors.py and
bench.py's cpu_baseline leg (configs C1 and C2 through the reference's code, `time_allreduce`; C1 with the
combine bound to the product's C-ABI, `time_allreduce_bound`). `run_bound` runs the reference's collectives
with f.f bound to a C-ABI's entry points passed by address.

The library exists where oracle/Makefile could build it: in the build container (the reference is there) and
on a GPU box that received the prebuilt file with the tree. `available()` says whether it is loadable; the
committed fixtures (tests/golden/ref_vectors.npz, tests/golden/ref_expr.json) carry its outputs everywhere else.

Same conventions as oracle/fmi_oracle.py: `allreduce(xs, op)` etc. return (recvbufs, sendbufs-after-call) per
peer, `expr(kind, P, rank, root, ordered)` the bracketing string, left operand = arg 0 of f.f.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence, Tuple

import numpy as np

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_ref", "libfmi_ref.so")

COLL = {"allreduce": 0, "reduce": 1, "scan": 2, "bcast": 3, "gather": 4, "scatter": 5, "barrier": 6}
OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3, "sub": 4}
DTYPES = {np.dtype(np.float32): 0, np.dtype(np.float64): 1, np.dtype(np.int32): 2, np.dtype(np.int64): 3,
          np.dtype(np.uint32): 4, np.dtype(np.uint64): 5}

_lib: Optional[ctypes.CDLL] = None


def available() -> bool:
    return os.path.exists(LIB_PATH)


def _load() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not available():
            raise FileNotFoundError(f"{LIB_PATH} is not built (make -C oracle; needs /root/reference)")
        lib = ctypes.CDLL(LIB_PATH)
        lib.fmi_ref_run.restype = ctypes.c_int
        lib.fmi_ref_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t),
                                    ctypes.c_char_p, ctypes.c_size_t]
        lib.fmi_ref_expr.restype = ctypes.c_long
        lib.fmi_ref_expr.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                     ctypes.c_size_t]
        _lib = lib
    return _lib


class RefError(RuntimeError):
    pass


def run(coll: str, op: str, xs: Sequence[np.ndarray], root: int = 0, ordered: bool = False,
        recv_init: Optional[Sequence[np.ndarray]] = None) -> Tuple[np.ndarray, np.ndarray, int]:
    """One collective of the reference over len(xs) peers. Returns (recv[P, ...], send_after[P, ...],
    sends_dropped): the recvbuf and the sendbuf of every peer after the call, and how many messages went to a
    peer id >= P (the reference's scan_ltr at P = 1 sends to peer 1)."""
    lib = _load()
    ins = np.ascontiguousarray(np.stack([np.asarray(x) for x in xs]))
    P = ins.shape[0]
    dt = DTYPES[ins.dtype]
    n = ins[0].size if coll != "scatter" else ins[0].size // P
    recv_shape = (P, P * n) if coll == "gather" else (P, n)
    recv = np.zeros(recv_shape, ins.dtype)
    init = None
    if recv_init is not None:
        init = np.ascontiguousarray(np.stack([np.asarray(r, ins.dtype) for r in recv_init]).reshape(recv_shape))
    send = np.zeros_like(ins)
    dropped = ctypes.c_size_t(0)
    err = ctypes.create_string_buffer(512)
    rc = lib.fmi_ref_run(COLL[coll], OPS[op], dt, int(ordered), P, root, n, ins.ctypes.data,
                         None if init is None else init.ctypes.data, recv.ctypes.data, send.ctypes.data,
                         ctypes.byref(dropped), err, len(err))
    if rc != 0:
        raise RefError(err.value.decode())
    return recv, send, dropped.value


def allreduce(xs, op: str, ordered: bool = False):
    recv, send, _ = run("allreduce", op, xs, ordered=ordered)
    return list(recv), list(send)


def reduce(xs, op: str, root: int = 0, ordered: bool = False):
    """(root's recvbuf, every peer's sendbuf after the call)."""
    recv, send, _ = run("reduce", op, xs, root=root, ordered=ordered)
    return recv[root], list(send)


def scan(xs, op: str, ordered: bool = False):
    recv, send, _ = run("scan", op, xs, ordered=ordered)
    return list(recv), list(send)


def expr(kind: str, P: int, rank: int = 0, root: int = 0, ordered: bool = False, which: str = "recv") -> str:
    """The expression the reference leaves in peer `rank`'s recvbuf (reduce: the root's), or with
    which="send" in its sendbuf, after `kind` over P peers x0 .. x{P-1}."""
    lib = _load()
    err = ctypes.create_string_buffer(512)
    size = 4096
    while True:
        buf = ctypes.create_string_buffer(size)
        k = lib.fmi_ref_expr(COLL[kind], int(ordered), P, rank, root, 1 if which == "send" else 0, buf, size,
                             err, len(err))
        if k < 0:
            raise RefError(err.value.decode())
        if k < size:
            return buf.value.decode()
        size = k + 1


def exprs(kind: str, P: int, ordered: bool = False) -> List[str]:
    """Every rank's expression (reduce: every root's)."""
    if kind == "reduce":
        return [expr(kind, P, root=r, ordered=ordered) for r in range(P)]
    return [expr(kind, P, rank=r, ordered=ordered) for r in range(P)]


HOST_PAIR = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_size_t)
DEV_PAIR = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                            ctypes.c_size_t, ctypes.c_void_p)
STREAM_SYNC = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)
LAST_ERROR = ctypes.CFUNCTYPE(ctypes.c_void_p)  # const char* (an address: ctypes leaks a c_char_p result)


class Binding(ctypes.Structure):
    """struct RefBinding (oracle/ref_harness.cpp): the entry points of a bucket-reduction C-ABI, by address —
    fmi_host_reduce_pair, fmi_dev_reduce_pair, fmi_stream_sync, fmi_last_error (include/fmi_dev.h). A null
    dev_pair selects the host entry point."""
    _fields_ = [("host_pair", ctypes.c_void_p), ("dev_pair", ctypes.c_void_p), ("stream_sync", ctypes.c_void_p),
                ("last_error", ctypes.c_void_p)]

    @classmethod
    def from_library(cls, lib: ctypes.CDLL, device_entry: bool = False) -> "Binding":
        """The binding INTEGRATION.md §B.2 makes, with the addresses of `lib`'s exported entry points."""
        addr = lambda name: ctypes.cast(getattr(lib, name), ctypes.c_void_p).value  # noqa: E731
        return cls(addr("fmi_host_reduce_pair"), addr("fmi_dev_reduce_pair") if device_entry else None,
                   addr("fmi_stream_sync"), addr("fmi_last_error"))


def run_bound(coll: str, op: str, xs: Sequence[np.ndarray], binding: Binding, root: int = 0, ordered: bool = False,
              recv_init: Optional[Sequence[np.ndarray]] = None,
              bufs: Optional[Sequence[int]] = None) -> Tuple[np.ndarray, np.ndarray]:
    """`run` with the reference's combine bound to `binding` (allreduce / reduce / scan). bufs: None (the
    harness's pageable buckets) or 2P addresses of caller-owned host-addressable buckets of n elements —
    peers' sendbufs, then their recvbufs (required, page-locked and mapped, for the device entry point)."""
    lib = _load()
    f = lib.fmi_ref_run_bound
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                  ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                  ctypes.POINTER(Binding), ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
    ins = np.ascontiguousarray(np.stack([np.asarray(x) for x in xs]))
    P, n = ins.shape[0], ins[0].size
    init = None
    if recv_init is not None:
        init = np.ascontiguousarray(np.stack([np.asarray(r, ins.dtype) for r in recv_init]).reshape(P, n))
    recv, send = np.zeros((P, n), ins.dtype), np.zeros_like(ins)
    ptrs = None
    if bufs is not None:
        if len(bufs) != 2 * P:
            raise ValueError("bufs must hold 2 * P bucket addresses")
        ptrs = (ctypes.c_void_p * (2 * P))(*bufs)
    err = ctypes.create_string_buffer(1024)
    rc = f(COLL[coll], OPS[op], DTYPES[ins.dtype], int(ordered), P, root, n, ins.ctypes.data,
           None if init is None else init.ctypes.data, recv.ctypes.data, send.ctypes.data, ctypes.byref(binding),
           None if ptrs is None else ctypes.cast(ptrs, ctypes.c_void_p), err, len(err))
    if rc != 0:
        raise RefError(err.value.decode())
    return recv, send


def time_allreduce_bound(P: int, n: int, reps: int, binding: Binding) -> float:
    """Median ms of the reference's own f32 sum-allreduce with every f.f through binding.host_pair."""
    lib = _load()
    f = lib.fmi_ref_time_allreduce_bound
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(Binding),
                  ctypes.POINTER(ctypes.c_double), ctypes.c_char_p, ctypes.c_size_t]
    ms = ctypes.c_double(0.0)
    err = ctypes.create_string_buffer(1024)
    if f(P, n, reps, ctypes.byref(binding), ctypes.byref(ms), err, len(err)) != 0:
        raise RefError(err.value.decode())
    return ms.value


def time_combine(threads: int, n: int, reps: int, adapter: bool) -> float:
    """Median ms of the f32 sum combine alone (adapter=True: the reference's vector adapter; False: std::transform
    in place) applied by `threads` threads at once, each to its own pair of n-element buckets (slowest thread)."""
    lib = _load()
    f = lib.fmi_ref_time_combine
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                  ctypes.c_char_p, ctypes.c_size_t]
    ms = ctypes.c_double(0.0)
    err = ctypes.create_string_buffer(512)
    if f(threads, n, reps, int(bool(adapter)), ctypes.byref(ms), err, len(err)) != 0:
        raise RefError(err.value.decode())
    return ms.value


def time_allreduce(P: int, n: int, reps: int, adapter) -> float:
    """Median ms of the reference's own f32 sum-allreduce (PeerToPeer::allreduce) over P peer threads and the
    in-memory transport; adapter=True combines through the reference's vector adapter (include/Communicator.h
    :180-189, restated in oracle/ref_harness.cpp), False through std::transform in place, "nop" through the
    reference's no-op combine (PeerToPeer.cpp:30): the transport and copies of the collective alone."""
    adapter = 2 if adapter == "nop" else int(bool(adapter))
    lib = _load()
    f = lib.fmi_ref_time_allreduce
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                  ctypes.c_char_p, ctypes.c_size_t]
    ms = ctypes.c_double(0.0)
    err = ctypes.create_string_buffer(512)
    if f(P, n, reps, adapter, ctypes.byref(ms), err, len(err)) != 0:
        raise RefError(err.value.decode())
    return ms.value


def time_scan(P: int, n: int, reps: int, adapter: bool) -> float:
    """Median ms of the reference's own f32 sum-scan (PeerToPeer::scan -> scan_no_order) over P peer threads and
    the in-memory transport; adapter as for time_allreduce (True: the vector adapter, False: in place)."""
    lib = _load()
    f = lib.fmi_ref_time_scan
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                  ctypes.c_char_p, ctypes.c_size_t]
    ms = ctypes.c_double(0.0)
    err = ctypes.create_string_buffer(512)
    if f(P, n, reps, int(bool(adapter)), ctypes.byref(ms), err, len(err)) != 0:
        raise RefError(err.value.decode())
    return ms.value
