"""Python handle over the C-ABI communicator (include/fmi_dev.h, "sharded device collectives").

`Comm` wraps fmi_comm_*: sharded allreduce / reduce / scan of device buckets across ranks (one rank per
GPU over RCCL, ranks as threads of one process over the LOCAL transport, or processes of one node over
PROC), with the combine done by the
fused kernels in the reference's evaluation order (reference src/comm/PeerToPeer.cpp). Buffers are
`fmi_amd.Bucket`s or raw device pointers.
"""
from __future__ import annotations

import ctypes
import enum
import os
from typing import Optional

from . import _lib
import numpy as np

from ._lib import Timeout  # noqa: F401 - FMI_ERR_TIMEOUT, the reference's FMI::Utils::Timeout

from .device import NP_DTYPE, Alg, Bucket, Op, _sptr, dtype_of

ID_BYTES = 128


class Transport(enum.IntEnum):
    RCCL = 0
    LOCAL = 1
    PROC = 2  # ranks are processes of one node (same or different GPUs): shared-memory staging + HIP IPC windows


class Path(enum.IntEnum):
    TREE = 0  # all-to-all + fused kernel in the reference's order + all-gather (bit-exact)
    RCCL = 1  # RCCL reduce-scatter + all-gather (RCCL's order)
    DIRECT = 2  # fused kernel reading every rank's window over xGMI + direct gather (bit-exact, windows only)


def unique_id(transport: Transport = Transport.RCCL) -> bytes:
    buf = ctypes.create_string_buffer(ID_BYTES)
    _lib.call("fmi_comm_unique_id", int(transport), buf, ID_BYTES)
    return buf.raw


VISIBILITY_ENV = ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "GPU_MAX_HW_QUEUES")


def runtime_info() -> dict:
    """What a multi-GPU run needs to be diagnosable from one line: the librccl the RCCL transport runs on
    (fmi_comm_rccl_info: ncclGetVersion and the real path of the mapped object) and the device-visibility /
    hardware-queue environment of this process. Never raises: a failure is reported in the dict."""
    info = {k: os.environ.get(k) for k in VISIBILITY_ENV}
    try:
        v = ctypes.c_int(0)
        path = ctypes.create_string_buffer(4096)
        _lib.call("fmi_comm_rccl_info", ctypes.byref(v), path, len(path))
        info["rccl_version"] = v.value
        info["rccl_path"] = path.value.decode(errors="replace")
    except Exception as e:  # reported, never raised: this runs on error paths
        info["rccl_error"] = f"{type(e).__name__}: {e}"
    return info


def _p(x) -> Optional[int]:
    if x is None:
        return None
    return x.ptr if isinstance(x, Bucket) else int(x)


class Comm:
    def __init__(self, uid: bytes, nranks: int, rank: int, timeout_s: Optional[float] = None):
        """timeout_s: how long any wait for the peers may last (init rendezvous, barriers, sync); None = the
        library default (FMI_COMM_TIMEOUT_S, else 300 s). Expiry raises Timeout and aborts the communicator."""
        if len(uid) != ID_BYTES:
            raise ValueError("communicator id must be 128 bytes")
        h = ctypes.c_void_p()
        self._id = ctypes.create_string_buffer(uid, ID_BYTES)
        _lib.call("fmi_comm_init_timeout", ctypes.byref(h), self._id, nranks, rank, float(timeout_s or 0.0))
        self.handle = h.value
        self.nranks = nranks
        self.rank = rank

    def destroy(self) -> None:
        if self.handle:
            _lib.call("fmi_comm_destroy", self.handle)
            self.handle = None

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                _lib.load().fmi_comm_destroy(self.handle)
        except Exception:
            pass

    def sync(self, stream=None) -> None:
        """Wait for the collectives enqueued on `stream` (None = library stream) within the communicator's
        timeout; raises Timeout (the communicator is then aborted) or FmiError on a transport error."""
        _lib.call("fmi_comm_sync", self.handle, _sptr(stream))

    def query(self) -> dict:
        """What the transport reports about this rank: RCCL's own rank count, rank and device
        (ncclCommCount / ncclCommUserRank / ncclCommCuDevice); the communicator's for LOCAL / PROC."""
        cnt, rk, dev = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _lib.call("fmi_comm_query", self.handle, ctypes.byref(cnt), ctypes.byref(rk), ctypes.byref(dev))
        return {"count": cnt.value, "rank": rk.value, "device": dev.value}

    def timing(self, enable: bool) -> None:
        """Record an event pair around every shard-kernel launch of the collectives (fmi_comm_timing)."""
        _lib.call("fmi_comm_timing", self.handle, 1 if enable else 0)

    def timing_read(self):
        """(total shard-kernel ms, launches) since timing was enabled or last read."""
        ms, k = ctypes.c_float(), ctypes.c_int()
        _lib.call("fmi_comm_timing_read", self.handle, ctypes.byref(ms), ctypes.byref(k))
        return float(ms.value), int(k.value)

    def allreduce(self, op: Op, send: Bucket, recv: Bucket, ordered: bool = False, path: Path = Path.TREE,
                  stream=None) -> None:
        alg = Alg.REDUCE_LTR if ordered else Alg.ALLREDUCE
        _lib.call("fmi_comm_allreduce", self.handle, int(op), int(send.dtype), int(alg), int(path), _p(send), _p(recv),
                  send.n, _sptr(stream))

    def window(self, n: int, dtype) -> Bucket:
        """A symmetric window bucket for Path.DIRECT (collective: every rank, same n and dtype). Release it
        with window_free (collective) or with the communicator."""
        nbytes = int(n) * np.dtype(NP_DTYPE[dtype_of(dtype)]).itemsize
        p = ctypes.c_void_p()
        _lib.call("fmi_comm_window_alloc", self.handle, nbytes, ctypes.byref(p))
        return Bucket(n, dtype, ptr=p.value)

    def window_free(self, b: Bucket) -> None:
        _lib.call("fmi_comm_window_free", self.handle, b.ptr)
        b.ptr = 0

    def allreduce_host(self, op: Op, send: np.ndarray, recv: np.ndarray, ordered: bool = False,
                       path: Path = Path.TREE, chunk: int = 0) -> None:
        """Allreduce of HOST arrays (channel recv buffers, config C5), streamed through the GPU in
        `chunk`-element pieces (0 = FMI_TUNE_HOST_CHUNK). Page-locked arrays (PinnedArray.array) take the
        DMA path. Blocking: `recv` holds the result on return."""
        if send.dtype != recv.dtype or send.size != recv.size:
            raise ValueError("allreduce_host: arrays must share dtype and size")
        if not (send.flags.c_contiguous and recv.flags.c_contiguous):
            raise ValueError("allreduce_host: arrays must be contiguous")
        alg = Alg.REDUCE_LTR if ordered else Alg.ALLREDUCE
        _lib.call("fmi_comm_allreduce_host", self.handle, int(op), int(dtype_of(send)), int(alg), int(path),
                  send.ctypes.data, recv.ctypes.data, send.size, int(chunk))

    def reduce(self, op: Op, send: Bucket, recv: Optional[Bucket], root: int, ordered: bool = False,
               stream=None, sendbuf_partials: bool = False) -> None:
        """sendbuf_partials=True: `send` ends as the reference leaves peer `rank`'s sendbuf (the partial it
        forwarded up the binomial tree, reference src/comm/PeerToPeer.cpp:72) — fmi_comm_reduce_sendbuf."""
        alg = Alg.REDUCE_LTR if ordered else Alg.REDUCE
        fn = "fmi_comm_reduce_sendbuf" if sendbuf_partials else "fmi_comm_reduce"
        _lib.call(fn, self.handle, int(op), int(send.dtype), int(alg), _p(send), _p(recv), send.n, root, _sptr(stream))

    def scan(self, op: Op, send: Bucket, recv: Bucket, ordered: bool = False, stream=None) -> None:
        alg = Alg.SCAN_LTR if ordered else Alg.SCAN
        _lib.call("fmi_comm_scan", self.handle, int(op), int(send.dtype), int(alg), _p(send), _p(recv), send.n,
                  _sptr(stream))

    def bcast(self, buf: Bucket, root: int, stream=None) -> None:
        _lib.call("fmi_comm_bcast", self.handle, _p(buf), buf.nbytes, root, _sptr(stream))

    def gather(self, send: Bucket, recv: Optional[Bucket], root: int, stream=None) -> None:
        _lib.call("fmi_comm_gather", self.handle, _p(send), _p(recv), send.nbytes, root, _sptr(stream))

    def scatter(self, send: Optional[Bucket], recv: Bucket, root: int, stream=None) -> None:
        _lib.call("fmi_comm_scatter", self.handle, _p(send), _p(recv), recv.nbytes, root, _sptr(stream))

    def send(self, buf: Bucket, peer: int, stream=None) -> None:
        _lib.call("fmi_comm_send", self.handle, _p(buf), buf.nbytes, peer, _sptr(stream))

    def recv(self, buf: Bucket, peer: int, stream=None) -> None:
        _lib.call("fmi_comm_recv", self.handle, _p(buf), buf.nbytes, peer, _sptr(stream))

    def barrier(self, stream=None) -> None:
        _lib.call("fmi_comm_barrier", self.handle, _sptr(stream))
