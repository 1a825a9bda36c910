"""fmi_amd — MI355X-native (gfx950) engine for FMI's bucket reduction (reduce / allreduce / scan).

Layout:
  include/fmi_dev.h          C-ABI (the drop-in boundary)
  fmi_amd/csrc/              HIP kernels + C-ABI implementation → fmi_amd/lib/libfmi_dev.so
  fmi_amd/cpp/include/fmi/   C++ mirror of the FMI::Communicator surface (reference include/)
  fmi_amd/device.py          Python handle over the C-ABI (ctypes)
  fmi_amd/collectives.py     multi-GPU sharded allreduce over torch.distributed (RCCL over xGMI)
"""
from ._lib import FmiError, LIB_PATH, Timeout, load  # noqa: F401
from .device import (  # noqa: F401
    Alg, Bucket, DType, Event, Graph, HostRegistration, Op, PinnedArray, Stream, Tune, combine, describe,
    device_count, finalize, host_reduce_pair, init, pci_bus_id, reduce_pair, reduce_pair_batch, reduce_tree, scan_peers, schedule_expr, sync, tune_get, tune_set,
)

__all__ = [
    "Alg", "Bucket", "DType", "Event", "FmiError", "Graph", "HostRegistration", "LIB_PATH", "Op", "PinnedArray", "Stream",
    "Timeout", "Tune", "combine", "describe", "device_count", "finalize", "host_reduce_pair", "init", "load", "pci_bus_id", "reduce_pair", "reduce_pair_batch",
    "reduce_tree", "scan_peers", "schedule_expr", "sync", "tune_get", "tune_set",
]
