"""ctypes binding of the C-ABI in include/fmi_dev.h (libfmi_dev.so, built in-tree for gfx950).

The library is the product path: nothing here falls back to a CPU implementation. If the shared
library is missing, `load()` raises; if no gfx950 device is visible, `fmi_dev_init` reports
FMI_ERR_NO_DEVICE and every device call raises FmiError.
"""
from __future__ import annotations

import ctypes
import os
import sys
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# FMI_DEV_LIB: another build of the same library (e.g. the host-sanitized one, tools/sanitize_lib.sh)
LIB_PATH = os.environ.get("FMI_DEV_LIB") or os.path.join(_HERE, "lib", "libfmi_dev.so")

FMI_OK = 0
FMI_ERR_INVALID = -1
FMI_ERR_HIP = -2
FMI_ERR_NO_DEVICE = -3
FMI_ERR_UNSUPPORTED = -4
FMI_ERR_ALLOC = -5
FMI_ERR_COMM = -6
FMI_ERR_TIMEOUT = -7

_STATUS_NAMES = {
    FMI_ERR_INVALID: "FMI_ERR_INVALID",
    FMI_ERR_HIP: "FMI_ERR_HIP",
    FMI_ERR_NO_DEVICE: "FMI_ERR_NO_DEVICE",
    FMI_ERR_UNSUPPORTED: "FMI_ERR_UNSUPPORTED",
    FMI_ERR_ALLOC: "FMI_ERR_ALLOC",
    FMI_ERR_COMM: "FMI_ERR_COMM",
    FMI_ERR_TIMEOUT: "FMI_ERR_TIMEOUT",
}


class FmiError(RuntimeError):
    """A C-ABI call returned a negative status (mirrors the std::runtime_error the C++ layer throws)."""

    def __init__(self, status: int, message: str):
        super().__init__(f"{_STATUS_NAMES.get(status, status)}: {message}")
        self.status = status


class Timeout(FmiError):
    """A peer did not arrive within the communicator's timeout (FMI_ERR_TIMEOUT): the reference's
    FMI::Utils::Timeout (include/utils/Common.h:11-15). The communicator is aborted; destroy it."""

    def __init__(self, message: str = "Timeout was reached"):
        super().__init__(FMI_ERR_TIMEOUT, message)


_c = ctypes
_vp = _c.c_void_p
_sz = _c.c_size_t
_i = _c.c_int

# name -> (restype, argtypes); kept in the order of include/fmi_dev.h
SIGNATURES = {
    "fmi_abi_version": (_i, []),
    "fmi_last_error": (_c.c_char_p, []),
    "fmi_dev_count": (_i, [_c.POINTER(_i)]),
    "fmi_dev_init": (_i, [_i]),
    "fmi_dev_finalize": (_i, []),
    "fmi_dev_sync": (_i, []),
    "fmi_dev_describe": (_i, [_c.c_char_p, _sz]),
    "fmi_dev_pci_bus_id": (_i, [_i, _c.c_char_p, _sz]),
    "fmi_dev_alloc": (_i, [_c.POINTER(_vp), _sz]),
    "fmi_dev_alloc_group": (_i, [_c.POINTER(_vp), _i, _sz]),
    "fmi_dev_free": (_i, [_vp]),
    "fmi_host_pin_alloc": (_i, [_c.POINTER(_vp), _sz]),
    "fmi_host_pin_free": (_i, [_vp]),
    "fmi_host_register": (_i, [_vp, _sz]),
    "fmi_host_unregister": (_i, [_vp]),
    "fmi_dev_h2d_async": (_i, [_vp, _vp, _sz, _vp]),
    "fmi_dev_d2h_async": (_i, [_vp, _vp, _sz, _vp]),
    "fmi_dev_d2d_async": (_i, [_vp, _vp, _sz, _vp]),
    "fmi_dev_memset_async": (_i, [_vp, _i, _sz, _vp]),
    "fmi_stream_create": (_i, [_c.POINTER(_vp)]),
    "fmi_stream_destroy": (_i, [_vp]),
    "fmi_stream_sync": (_i, [_vp]),
    "fmi_event_create": (_i, [_c.POINTER(_vp)]),
    "fmi_event_destroy": (_i, [_vp]),
    "fmi_event_record": (_i, [_vp, _vp]),
    "fmi_stream_wait_event": (_i, [_vp, _vp]),
    "fmi_event_sync": (_i, [_vp]),
    "fmi_event_elapsed_ms": (_i, [_c.POINTER(_c.c_float), _vp, _vp]),
    "fmi_graph_capture_begin": (_i, [_vp]),
    "fmi_graph_capture_end": (_i, [_vp, _c.POINTER(_vp)]),
    "fmi_graph_launch": (_i, [_vp, _vp]),
    "fmi_graph_destroy": (_i, [_vp]),
    "fmi_dev_reduce_pair": (_i, [_i, _i, _vp, _vp, _sz, _vp]),
    "fmi_dev_reduce_pair_batch": (_i, [_i, _i, _vp, _i, _vp]),
    "fmi_dev_combine": (_i, [_i, _i, _vp, _vp, _vp, _sz, _vp]),
    "fmi_dev_reduce_tree": (_i, [_i, _i, _i, _vp, _c.POINTER(_vp), _i, _i, _sz, _vp]),
    "fmi_dev_scan_peers": (_i, [_i, _i, _i, _c.POINTER(_vp), _c.POINTER(_vp), _i, _sz, _vp]),
    "fmi_host_reduce_pair": (_i, [_i, _i, _vp, _vp, _sz]),
    "fmi_host_device_ptr": (_i, [_vp, _sz, _c.POINTER(_vp)]),
    "fmi_host_page_locked": (_i, [_vp, _sz]),
    "fmi_comm_unique_id": (_i, [_i, _vp, _sz]),
    "fmi_comm_init": (_i, [_c.POINTER(_vp), _vp, _i, _i]),
    "fmi_comm_init_timeout": (_i, [_c.POINTER(_vp), _vp, _i, _i, _c.c_double]),
    "fmi_comm_destroy": (_i, [_vp]),
    "fmi_comm_size": (_i, [_vp, _c.POINTER(_i), _c.POINTER(_i)]),
    "fmi_comm_sync": (_i, [_vp, _vp]),
    "fmi_comm_query": (_i, [_vp, _c.POINTER(_i), _c.POINTER(_i), _c.POINTER(_i)]),
    "fmi_comm_rccl_info": (_i, [_c.POINTER(_i), _c.c_char_p, _sz]),
    "fmi_comm_window_alloc": (_i, [_vp, _sz, _c.POINTER(_vp)]),
    "fmi_comm_window_free": (_i, [_vp, _vp]),
    "fmi_comm_timing": (_i, [_vp, _i]),
    "fmi_comm_timing_read": (_i, [_vp, _c.POINTER(_c.c_float), _c.POINTER(_i)]),
    "fmi_comm_allreduce": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _sz, _vp]),
    "fmi_comm_allreduce_host": (_i, [_vp, _i, _i, _i, _i, _vp, _vp, _sz, _sz]),
    "fmi_comm_reduce": (_i, [_vp, _i, _i, _i, _vp, _vp, _sz, _i, _vp]),
    "fmi_comm_reduce_sendbuf": (_i, [_vp, _i, _i, _i, _vp, _vp, _sz, _i, _vp]),
    "fmi_comm_scan": (_i, [_vp, _i, _i, _i, _vp, _vp, _sz, _vp]),
    "fmi_comm_bcast": (_i, [_vp, _vp, _sz, _i, _vp]),
    "fmi_comm_gather": (_i, [_vp, _vp, _vp, _sz, _i, _vp]),
    "fmi_comm_scatter": (_i, [_vp, _vp, _vp, _sz, _i, _vp]),
    "fmi_comm_send": (_i, [_vp, _vp, _sz, _i, _vp]),
    "fmi_comm_recv": (_i, [_vp, _vp, _sz, _i, _vp]),
    "fmi_comm_barrier": (_i, [_vp, _vp]),
    "fmi_dev_fill_synthetic": (_i, [_i, _vp, _sz, _c.c_uint64, _c.c_uint32, _vp]),
    "fmi_dev_fill_synthetic_at": (_i, [_i, _vp, _sz, _c.c_uint64, _c.c_uint32, _c.c_uint64, _vp]),
    "fmi_schedule_expr": (_i, [_i, _i, _i, _c.c_char_p, _sz]),
    "fmi_tune_set": (_i, [_i, _c.c_longlong]),
    "fmi_tune_get": (_i, [_i, _c.POINTER(_c.c_longlong)]),
}

_lock = threading.Lock()
_lib = None
# Whether torch (and with it torch's bundled HIP runtime) was already loaded when libfmi_dev.so was: only
# then do torch, RCCL and our kernels share one runtime (see fmi_amd/collectives.py).
TORCH_LOADED_FIRST = False


def load() -> ctypes.CDLL:
    """Load libfmi_dev.so (once). Raises FileNotFoundError if it has not been built."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise FileNotFoundError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "or `make -C fmi_amd/csrc`. There is no CPU fallback for the device path.")
        global TORCH_LOADED_FIRST
        TORCH_LOADED_FIRST = "torch" in sys.modules
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def last_error() -> str:
    msg = load().fmi_last_error()
    return msg.decode() if msg else ""


def check(status: int) -> None:
    if status == FMI_ERR_TIMEOUT:
        raise Timeout(last_error())
    if status != FMI_OK:
        raise FmiError(status, last_error())


def call(name: str, *args) -> None:
    check(getattr(load(), name)(*args))
