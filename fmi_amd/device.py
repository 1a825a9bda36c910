"""Host-side handle to the gfx950 bucket-reduction engine (thin layer over include/fmi_dev.h).

Names follow FMI's vocabulary: a *bucket* is one peer's contiguous buffer (reference
include/comm/Data.h:50-73, `Data<std::vector<A>>`), an *op* is one of the reference's built-in
reduction functions (reference python/PythonCommunicator.h:131-149), and the P-way entry points
reproduce the combine order of a reference collective (reference src/comm/PeerToPeer.cpp).
"""
from __future__ import annotations

import ctypes
import enum
from typing import Optional, Sequence

import numpy as np

from . import _lib


class Op(enum.IntEnum):
    """Reference Python op enum SUM/PROD/MAX/MIN (reference python/PythonCommunicator.h:13-15)."""
    SUM = 0
    PROD = 1
    MAX = 2
    MIN = 3


class DType(enum.IntEnum):
    """fmi_dtype_t. F32 / F64 / I32 / I64 run every kernel; the other integer widths run the pairwise
    kernel, and their P-way programs run as pairwise passes."""
    F32 = 0
    F64 = 1
    I32 = 2
    I64 = 3
    U32 = 4
    U64 = 5
    I8 = 6
    U8 = 7
    I16 = 8
    U16 = 9


class Alg(enum.IntEnum):
    """Evaluation orders of the reference collectives (src/comm/PeerToPeer.cpp)."""
    ALLREDUCE = 0   # allreduce_no_order  :96-130
    REDUCE = 1      # reduce_no_order     :59-84
    REDUCE_LTR = 2  # reduce_ltr          :44-57
    SCAN = 3        # scan_no_order       :154-184
    SCAN_LTR = 4    # scan_ltr            :141-152


class Tune(enum.IntEnum):
    PAIR_VARIANT = 0
    PAIR_UNROLL = 1
    BLOCK = 2
    GRID_PER_CU = 3
    HOST_CHUNK = 4
    HOST_ZERO_COPY = 5
    FUSED_INFLIGHT_KIB = 6
    BLOCKS_ONE_PASS = 7
    COMM_A2A = 8
    COMM_GATHER = 9
    COMM_PIPELINE = 10
    FUSED_POLICY = 11
    PAIR_SC1_OF_8 = 12
    COMM_ONE_RANK_EXCHANGE = 13
    ALLOC_SLOTS = 14
    COMM_SHARD_SKEW = 15


NP_DTYPE = {DType.F32: np.float32, DType.F64: np.float64, DType.I32: np.int32, DType.I64: np.int64,
            DType.U32: np.uint32, DType.U64: np.uint64, DType.I8: np.int8, DType.U8: np.uint8, DType.I16: np.int16,
            DType.U16: np.uint16}


def dtype_of(arr_or_dtype) -> DType:
    if isinstance(arr_or_dtype, np.ndarray):
        dt = arr_or_dtype.dtype
    else:
        dt = np.dtype(arr_or_dtype)
    for k, v in NP_DTYPE.items():
        if np.dtype(v) == dt:
            return k
    raise TypeError(f"unsupported bucket dtype {dt}; FMI device buckets are f32, f64 or 8/16/32/64-bit integers")


def _ptr(x) -> Optional[int]:
    if x is None:
        return None
    if isinstance(x, Bucket):
        return x.ptr
    if isinstance(x, int):
        return x
    raise TypeError(f"expected a Bucket or a raw device pointer, got {type(x)}")


def _sptr(stream) -> Optional[int]:
    if stream is None:
        return None
    return stream.handle if isinstance(stream, Stream) else int(stream)


# ----------------------------------------------------------------------------------------------------
# device / memory
# ----------------------------------------------------------------------------------------------------
def device_count() -> int:
    c = ctypes.c_int(0)
    _lib.call("fmi_dev_count", ctypes.byref(c))
    return c.value


def init(device: int = 0) -> None:
    _lib.call("fmi_dev_init", device)


def finalize() -> None:
    _lib.call("fmi_dev_finalize")


def sync() -> None:
    _lib.call("fmi_dev_sync")


def describe() -> str:
    buf = ctypes.create_string_buffer(512)
    _lib.call("fmi_dev_describe", buf, len(buf))
    return buf.value.decode()


def pci_bus_id(device: int) -> str:
    """PCI bus id of a visible device ("dddd:bb:dd.f")."""
    buf = ctypes.create_string_buffer(64)
    _lib.call("fmi_dev_pci_bus_id", int(device), buf, len(buf))
    return buf.value.decode()


class Bucket:
    """A device-resident bucket of `n` elements of `dtype` (owns its HBM allocation unless `view`)."""

    def __init__(self, n: int, dtype, ptr: Optional[int] = None, owner: Optional["Bucket"] = None):
        self.dtype = dtype_of(dtype) if not isinstance(dtype, DType) else dtype
        self.n = int(n)
        self.itemsize = np.dtype(NP_DTYPE[self.dtype]).itemsize
        self._owner = owner
        if ptr is None:
            p = ctypes.c_void_p()
            _lib.call("fmi_dev_alloc", ctypes.byref(p), self.nbytes)
            self.ptr = p.value
            self._owns = True
        else:
            self.ptr = ptr
            self._owns = False

    @property
    def nbytes(self) -> int:
        return self.n * self.itemsize

    @classmethod
    def group(cls, count: int, n: int, dtype) -> list:
        """`count` buckets that one kernel streams together (a fused kernel's peers and outputs, a pair's two
        operands): fmi_dev_alloc_group puts bucket j in 4 KiB slot j mod 16, whatever was allocated before
        (DESIGN §4)."""
        dt = dtype_of(dtype) if not isinstance(dtype, DType) else dtype
        nbytes = int(n) * np.dtype(NP_DTYPE[dt]).itemsize
        ptrs = (ctypes.c_void_p * max(int(count), 1))()
        _lib.call("fmi_dev_alloc_group", ptrs, int(count), nbytes)
        out = []
        for j in range(int(count)):
            b = cls(n, dt, ptr=ptrs[j])
            b._owns = True
            out.append(b)
        return out

    @classmethod
    def from_numpy(cls, arr: np.ndarray, stream=None) -> "Bucket":
        arr = np.ascontiguousarray(arr)
        b = cls(arr.size, dtype_of(arr))
        b.upload(arr, stream)
        return b

    def view(self, offset: int, n: int) -> "Bucket":
        """Sub-bucket starting `offset` elements in (used to exercise unaligned buckets)."""
        if offset < 0 or offset + n > self.n:
            raise ValueError("view out of range")
        return Bucket(n, self.dtype, ptr=self.ptr + offset * self.itemsize, owner=self)

    def upload(self, arr: np.ndarray, stream=None) -> None:
        arr = np.ascontiguousarray(arr, dtype=NP_DTYPE[self.dtype])
        if arr.size != self.n:
            raise ValueError(f"size mismatch: bucket has {self.n} elements, array {arr.size}")
        _lib.call("fmi_dev_h2d_async", self.ptr, arr.ctypes.data, self.nbytes, _sptr(stream))
        _lib.call("fmi_stream_sync", _sptr(stream))

    def numpy(self, stream=None) -> np.ndarray:
        out = np.empty(self.n, dtype=NP_DTYPE[self.dtype])
        _lib.call("fmi_dev_d2h_async", out.ctypes.data, self.ptr, self.nbytes, _sptr(stream))
        _lib.call("fmi_stream_sync", _sptr(stream))
        return out

    def fill_synthetic(self, seed: int, peer: int, stream=None, first: int = 0) -> "Bucket":
        """Elements [first, first + n) of peer `peer`'s synthetic bucket (SURVEY.md §8d generator)."""
        _lib.call("fmi_dev_fill_synthetic_at", int(self.dtype), self.ptr, self.n, seed, peer, int(first),
                  _sptr(stream))
        return self

    def copy_from(self, other: "Bucket", stream=None) -> None:
        if other.nbytes != self.nbytes:
            raise ValueError("size mismatch")
        _lib.call("fmi_dev_d2d_async", self.ptr, other.ptr, self.nbytes, _sptr(stream))

    def free(self) -> None:
        if self._owns and self.ptr:
            _lib.call("fmi_dev_free", self.ptr)
        self.ptr = 0
        self._owns = False

    def __del__(self):
        try:
            if getattr(self, "_owns", False) and self.ptr:
                _lib.load().fmi_dev_free(self.ptr)
        except Exception:
            pass


class Stream:
    def __init__(self):
        h = ctypes.c_void_p()
        _lib.call("fmi_stream_create", ctypes.byref(h))
        self.handle = h.value

    def sync(self) -> None:
        _lib.call("fmi_stream_sync", self.handle)

    def destroy(self) -> None:
        if self.handle:
            _lib.call("fmi_stream_destroy", self.handle)
            self.handle = None


class Graph:
    """A launch sequence recorded once and replayed as one submission (fmi_graph_*): many small bucket
    combines, where launch cost rather than HBM is the limit.

        g = Graph.capture(stream, lambda: [reduce_pair(Op.SUM, a, b, stream=stream) for a, b in pairs])
        g.launch(stream)   # every combine again, same buckets
    """

    def __init__(self, handle: int):
        self.handle = handle

    @classmethod
    def capture(cls, stream: "Stream", record) -> "Graph":
        _lib.call("fmi_graph_capture_begin", stream.handle)
        h = ctypes.c_void_p()
        try:
            record()
        finally:  # always end the capture, so a failure inside `record` leaves the stream usable
            end_rc = _lib.load().fmi_graph_capture_end(stream.handle, ctypes.byref(h))
        if end_rc != 0:
            raise _lib.FmiError(end_rc, _lib.last_error())
        return cls(h.value)

    def launch(self, stream=None) -> None:
        _lib.call("fmi_graph_launch", self.handle, _sptr(stream))

    def destroy(self) -> None:
        if self.handle:
            _lib.call("fmi_graph_destroy", self.handle)
            self.handle = None


class Event:
    def __init__(self):
        h = ctypes.c_void_p()
        _lib.call("fmi_event_create", ctypes.byref(h))
        self.handle = h.value

    def record(self, stream=None) -> "Event":
        _lib.call("fmi_event_record", self.handle, _sptr(stream))
        return self

    def sync(self) -> None:
        _lib.call("fmi_event_sync", self.handle)

    def wait_on(self, stream=None) -> None:
        """Make later work on `stream` (None = library stream) wait for this event."""
        _lib.call("fmi_stream_wait_event", _sptr(stream), self.handle)

    def elapsed_ms(self, end: "Event") -> float:
        ms = ctypes.c_float()
        _lib.call("fmi_event_elapsed_ms", ctypes.byref(ms), self.handle, end.handle)
        return float(ms.value)

    def destroy(self) -> None:
        if self.handle:
            _lib.call("fmi_event_destroy", self.handle)
            self.handle = None


# ----------------------------------------------------------------------------------------------------
# hot path
# ----------------------------------------------------------------------------------------------------
def reduce_pair(op: Op, inout: Bucket, src: Bucket, n: Optional[int] = None, stream=None) -> None:
    """inout = op(inout, src) elementwise — one reference `f.f(a, b)` (include/Communicator.h:180-189)."""
    n = inout.n if n is None else n
    if src.dtype != inout.dtype or src.n < n or inout.n < n:
        raise ValueError("reduce_pair: buckets must share dtype and hold n elements")
    _lib.call("fmi_dev_reduce_pair", int(op), int(inout.dtype), inout.ptr, src.ptr, n, _sptr(stream))


class _PairDesc(ctypes.Structure):
    _fields_ = [("inout", ctypes.c_void_p), ("in_", ctypes.c_void_p), ("n", ctypes.c_size_t)]


def reduce_pair_batch(op: Op, pairs: Sequence, stream=None) -> None:
    """inout = op(inout, in) for every (inout, in) bucket pair, batched into as few launches as possible
    (fmi_dev_reduce_pair_batch): for many small buckets. All buckets share one dtype."""
    if not pairs:
        return
    dtype = pairs[0][0].dtype
    for a, b in pairs:
        if a.dtype != dtype or b.dtype != dtype or b.n < a.n:
            raise ValueError("reduce_pair_batch: one dtype for every bucket, and each `in` at least as long as its inout")
    descs = (_PairDesc * len(pairs))(*[_PairDesc(a.ptr, b.ptr, a.n) for a, b in pairs])
    _lib.call("fmi_dev_reduce_pair_batch", int(op), int(dtype), ctypes.cast(descs, ctypes.c_void_p), len(pairs),
              _sptr(stream))


def combine(op: Op, out: Bucket, a: Bucket, b: Bucket, stream=None) -> None:
    if not (out.dtype == a.dtype == b.dtype) or not (out.n == a.n == b.n):
        raise ValueError("combine: buckets must share dtype and length")
    _lib.call("fmi_dev_combine", int(op), int(out.dtype), out.ptr, a.ptr, b.ptr, out.n, _sptr(stream))


def _ptr_array(buckets: Sequence[Bucket]):
    arr = (ctypes.c_void_p * len(buckets))()
    for i, b in enumerate(buckets):
        arr[i] = b.ptr
    return arr


def reduce_tree(op: Op, alg: Alg, out: Bucket, ins: Sequence[Bucket], rank: int = 0, stream=None) -> None:
    """P-way reduction with a reference collective's bracketing (see include/fmi_dev.h)."""
    _check_peers(out, ins)
    _lib.call("fmi_dev_reduce_tree", int(op), int(out.dtype), int(alg), out.ptr, _ptr_array(ins), len(ins), rank,
              out.n, _sptr(stream))


def scan_peers(op: Op, alg: Alg, outs: Sequence[Bucket], ins: Sequence[Bucket], stream=None) -> None:
    """Peer-axis inclusive scan with the bracketing of reference scan_no_order / scan_ltr."""
    if len(outs) != len(ins):
        raise ValueError("scan_peers: one output bucket per peer")
    _check_peers(outs[0], ins)  # O(P): every bucket, in or out, against the first output
    _check_peers(outs[0], outs)
    _lib.call("fmi_dev_scan_peers", int(op), int(outs[0].dtype), int(alg), _ptr_array(outs), _ptr_array(ins),
              len(ins), outs[0].n, _sptr(stream))


def host_reduce_pair(op: Op, inout: np.ndarray, src: np.ndarray) -> None:
    """inout = op(inout, src) for host arrays, streamed through the device (H2D, kernel, D2H)."""
    if inout.dtype != src.dtype or inout.size != src.size:
        raise ValueError("host_reduce_pair: arrays must share dtype and size")
    if not (inout.flags.c_contiguous and src.flags.c_contiguous):
        raise ValueError("host_reduce_pair: arrays must be contiguous")
    _lib.call("fmi_host_reduce_pair", int(op), int(dtype_of(inout)), inout.ctypes.data, src.ctypes.data, inout.size)


class PinnedArray:
    """A numpy array over page-locked host memory (fmi_host_pin_alloc) — the recv-buffer kind the
    zero-copy host path combines in place over PCIe. Free with .free() (or on garbage collection)."""

    def __init__(self, n: int, dtype):
        self.dtype = np.dtype(dtype)
        nbytes = max(1, int(n) * self.dtype.itemsize)
        p = ctypes.c_void_p()
        _lib.call("fmi_host_pin_alloc", ctypes.byref(p), nbytes)
        self.ptr = p.value
        raw = (ctypes.c_char * nbytes).from_address(self.ptr)
        self.array = np.frombuffer(raw, dtype=self.dtype, count=int(n))

    def free(self) -> None:
        if self.ptr:
            self.array = None
            _lib.call("fmi_host_pin_free", self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            if getattr(self, "ptr", None):
                _lib.load().fmi_host_pin_free(self.ptr)
        except Exception:
            pass


class HostRegistration:
    """Page-lock an existing contiguous numpy array in place (fmi_host_register), so fmi_host_reduce_pair
    combines it zero-copy and the host pipelines move it at DMA rate. For recv buffers reused across many
    collectives: registering costs about one copy of the array. The array must outlive the registration.
    Use as a context manager, or call .close()."""

    def __init__(self, arr: np.ndarray):
        if not arr.flags.c_contiguous or arr.nbytes == 0:
            raise ValueError("HostRegistration: needs a non-empty contiguous array")
        self.array = arr
        self.ptr = arr.ctypes.data
        _lib.call("fmi_host_register", self.ptr, arr.nbytes)

    def close(self) -> None:
        if self.ptr:
            _lib.call("fmi_host_unregister", self.ptr)
            self.ptr = None
            self.array = None

    def __enter__(self) -> "HostRegistration":
        return self

    def __exit__(self, *exc) -> None:
        self.close()


def _check_peers(out: Bucket, ins: Sequence[Bucket]) -> None:
    if not ins:
        raise ValueError("need at least one peer bucket")
    for b in ins:
        if b.dtype != out.dtype or b.n != out.n:
            raise ValueError("all peer buckets must share dtype and length")


def schedule_expr(alg: Alg, P: int, rank: int) -> str:
    size = 1 << 16
    while True:
        buf = ctypes.create_string_buffer(size)
        status = _lib.load().fmi_schedule_expr(int(alg), P, rank, buf, len(buf))
        msg = _lib.last_error() if status else ""
        if status and "buffer too small" in msg:  # "(<bytes> needed)"
            size = int(msg.split("(")[1].split()[0])
            continue
        _lib.check(status)
        return buf.value.decode()


def tune_set(key: Tune, value: int) -> None:
    _lib.call("fmi_tune_set", int(key), int(value))


def tune_get(key: Tune) -> int:
    v = ctypes.c_longlong()
    _lib.call("fmi_tune_get", int(key), ctypes.byref(v))
    return v.value
