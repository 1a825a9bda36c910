"""`fmi` — the reference's Python API (reference python/fmi_python.cpp:12-54, PythonCommunicator.{h,cpp})
over the MI355X engine, so Python FMI code runs unchanged:

    import fmi_amd.fmi as fmi
    comm = fmi.Communicator(peer_id, num_peers, "config.json", "job", 512)
    comm.allreduce([1.5, 2.5], fmi.func(fmi.op.sum), fmi.types(fmi.datatypes.double_list, 2))

Built-in ops (`fmi.op.sum/prod/max/min`) on int / double / int_list / double_list run as device
collectives (fmi_comm_*: sharded exchange + the fused kernel in the reference's order, reference
python/PythonCommunicator.h:131-149 semantics). `fmi.op.custom` Python callables are evaluated on the host
in exactly the reference's bracketing (the same programs the kernels run), after gathering the peers'
values through the device transport.

Peers, transport and rendezvous:
  * one peer = one process = one GPU (transport "Rccl", device = $LOCAL_RANK or peer_id modulo the
    visible GPUs), or peers = threads of one process sharing a GPU (transport "Local");
  * config (the reference's JSON schema): {"backends": {"Rccl": {"enabled": true, "rendezvous_dir": "/tmp",
    "max_timeout": 60000}}} or "Local" instead of "Rccl"; a config without either selects Rccl with
    these defaults (the reference's Direct/Redis/S3 host transports are not part of this engine);
  * the 128-byte communicator id travels through a file `<rendezvous_dir>/fmi_amd_<comm_name>.id` that
    peer 0 writes — so, as in the reference, comm_name must be unique per concurrent communicator.
"""
from __future__ import annotations

import enum
import json
import os
import re
import time
from typing import Any, Callable, List, Optional

import numpy as np

from . import _lib
from . import device as _dev
from .comm import Comm, Transport, unique_id
from .device import Alg, Bucket, Op


# FMI::Utils::Timeout (reference include/utils/Common.h:11-15): raised when the communicator id does not
# appear in time and by every device wait the communicator bounds (FMI_ERR_TIMEOUT; "max_timeout" ms).
Timeout = _lib.Timeout


class datatypes(enum.IntEnum):  # noqa: N801 - reference spelling (python/fmi_python.cpp:28-33)
    int = 0
    double = 1
    int_list = 2
    double_list = 3


class op(enum.IntEnum):  # noqa: N801 - reference spelling (python/fmi_python.cpp:39-45)
    sum = 0
    prod = 1
    max = 2
    min = 3
    custom = 4


class hints(enum.IntEnum):  # noqa: N801
    fast = 0
    cheap = 1


class types:  # noqa: N801
    def __init__(self, type: datatypes, num_objects: int = 1):  # noqa: A002 - reference signature
        self.type = datatypes(type)
        self.num_objects = int(num_objects)


class func:  # noqa: N801
    def __init__(self, o: op, fn: Optional[Callable] = None, commutative: bool = False, associative: bool = False):
        self.op = op(o)
        self.fn = fn
        self.commutative = commutative
        self.associative = associative
        if self.op == op.custom and fn is None:
            raise ValueError("fmi.op.custom needs a Python callable")


_NP = {datatypes.int: np.int32, datatypes.double: np.float64, datatypes.int_list: np.int32,
       datatypes.double_list: np.float64}


def _is_list(t: types) -> bool:
    return t.type in (datatypes.int_list, datatypes.double_list)


def _eval_expr(expr: str, values: List[Any], fn: Callable) -> Any:
    """Evaluate a schedule expression '((x0+x1)+x2)' with `fn` as the combine (left = arg 0 of f.f)."""
    tokens = re.findall(r"\(|\)|\+|x\d+", expr)
    pos = 0

    def parse():
        nonlocal pos
        tok = tokens[pos]
        pos += 1
        if tok.startswith("x"):
            return values[int(tok[1:])]
        left = parse()
        pos += 1  # '+'
        right = parse()
        pos += 1  # ')'
        return fn(left, right)

    return parse()


class Communicator:
    def __init__(self, peer_id: int, num_peers: int, config_path: str, comm_name: str, faas_memory: int = 128):
        self.peer_id = int(peer_id)
        self.num_peers = int(num_peers)
        self.comm_name = comm_name
        self.faas_memory = faas_memory
        self._hint = hints.cheap
        transport, params = self._read_config(config_path)
        if transport == Transport.RCCL:
            ndev = _dev.device_count()
            if ndev == 0:
                raise RuntimeError("fmi: no GPU visible for the Rccl transport")
            device = int(os.environ.get("LOCAL_RANK", self.peer_id)) % ndev
        else:
            device = 0
        _dev.init(device)
        self._id_path = os.path.join(params.get("rendezvous_dir", "/tmp"), f"fmi_amd_{comm_name}.id")
        timeout_s = float(params.get("max_timeout", 60000)) / 1000.0
        uid = self._rendezvous(transport, timeout_s)
        self._comm = Comm(uid, self.num_peers, self.peer_id, timeout_s=timeout_s)

    # ---- setup ------------------------------------------------------------------------------------
    @staticmethod
    def _read_config(path: str):
        if not path or not os.path.exists(path):
            return Transport.RCCL, {}
        cfg = json.load(open(path))
        backends = cfg.get("backends", {})
        for name, transport in (("Local", Transport.LOCAL), ("Rccl", Transport.RCCL)):
            b = backends.get(name)
            if b is not None and str(b.get("enabled", True)).lower() == "true":
                return transport, b
        return Transport.RCCL, {}

    def _rendezvous(self, transport: Transport, timeout_s: float) -> bytes:
        if self.peer_id == 0:
            uid = unique_id(transport)
            tmp = f"{self._id_path}.{os.getpid()}.{id(self)}.tmp"
            with open(tmp, "wb") as f:
                f.write(uid)
            os.replace(tmp, self._id_path)
            return uid
        deadline = time.monotonic() + timeout_s
        while True:
            try:
                with open(self._id_path, "rb") as f:
                    uid = f.read()
                if len(uid) == 128:
                    return uid
            except FileNotFoundError:
                pass
            if time.monotonic() > deadline:
                raise Timeout(f"no communicator id at {self._id_path}")
            time.sleep(0.01)

    def finalize(self) -> None:
        if getattr(self, "_comm", None) is not None:
            self._comm.destroy()
            self._comm = None
            if self.peer_id == 0:
                try:
                    os.unlink(self._id_path)
                except OSError:
                    pass

    def __del__(self):
        try:
            self.finalize()
        except Exception:
            pass

    # ---- marshalling ------------------------------------------------------------------------------
    def _array(self, value, t: types) -> np.ndarray:
        dt = _NP[t.type]
        if _is_list(t):
            a = np.asarray(list(value), dtype=dt)
        else:
            a = np.asarray([value], dtype=dt)
        return a

    @staticmethod
    def _py(a: np.ndarray, t: types):
        return a.tolist() if _is_list(t) else a[0].item()

    def _count(self, t: types) -> int:
        return t.num_objects if _is_list(t) else 1

    # ---- point to point / data movement ------------------------------------------------------------
    def send(self, data, dest: int, t: types) -> None:
        self._comm.send(Bucket.from_numpy(self._array(data, t)), dest)
        self._comm.sync()

    def recv(self, src: int, t: types):
        b = Bucket(self._count(t), _NP[t.type])
        self._comm.recv(b, src)
        self._comm.sync()
        return self._py(b.numpy(), t)

    def bcast(self, data, root: int, t: types):
        if self.peer_id == root:
            b = Bucket.from_numpy(self._array(data, t))
        else:
            b = Bucket(self._count(t), _NP[t.type])
        self._comm.bcast(b, root)
        self._comm.sync()
        return self._py(b.numpy(), t)

    def barrier(self) -> None:
        self._comm.barrier()

    def gather(self, data, root: int, t: types):
        mine = self._array(data, t)
        send = Bucket.from_numpy(mine)
        recv = Bucket(mine.size * self.num_peers, mine.dtype) if self.peer_id == root else None
        self._comm.gather(send, recv, root)
        self._comm.sync()
        return recv.numpy().tolist() if recv is not None else []

    def scatter(self, data, root: int, t: types):
        if t.num_objects % self.num_peers != 0:
            raise RuntimeError("List length not divisible by number of peers")
        if not _is_list(t):
            raise RuntimeError("Cannot scatter atomic types")
        per = t.num_objects // self.num_peers
        send = Bucket.from_numpy(self._array(data, t)) if self.peer_id == root else None
        recv = Bucket(per, _NP[t.type])
        self._comm.scatter(send, recv, root)
        self._comm.sync()
        return recv.numpy().tolist()

    # ---- reductions (reference python/PythonCommunicator.cpp:173-278) -----------------------------
    def _flags(self, f: func, t: types):
        if f.op != op.custom:
            return True, True
        if _is_list(t):  # the reference registers custom list functions as commutative + associative
            return True, True
        return f.commutative, f.associative

    def _custom_values(self, mine: np.ndarray) -> List[np.ndarray]:
        """Every peer's bucket on every peer (gather to 0 + bcast), for host evaluation of custom ops."""
        n = mine.size
        send = Bucket.from_numpy(mine)
        allb = Bucket(n * self.num_peers, mine.dtype)
        self._comm.gather(send, allb if self.peer_id == 0 else None, 0)
        self._comm.bcast(allb, 0)
        self._comm.sync()
        flat = allb.numpy()
        return [flat[p * n:(p + 1) * n] for p in range(self.num_peers)]

    def _custom(self, f: func, t: types, values: List[np.ndarray], expr: str):
        if _is_list(t):
            elems = [[v[i].item() for v in values] for i in range(values[0].size)]
            out = [_eval_expr(expr, e, f.fn) for e in elems]
            return [_NP[t.type](x).item() for x in out]
        res = _eval_expr(expr, [v[0].item() for v in values], f.fn)
        return _NP[t.type](res).item()

    def reduce(self, data, root: int, f: func, t: types):
        mine = self._array(data, t)
        comm_, assoc = self._flags(f, t)
        ordered = not (comm_ and assoc)
        if f.op == op.custom:
            values = self._custom_values(mine)
            if self.peer_id != root:  # the reference returns its untouched recvbuf off-root
                return self._py(np.zeros_like(mine), t)
            if ordered:
                expr = _dev.schedule_expr(Alg.REDUCE_LTR, self.num_peers, 0)
            else:  # reduce programs are in transformed ids (root -> 0)
                expr = re.sub(r"x(\d+)", lambda m: "x%d" % ((int(m.group(1)) + root) % self.num_peers),
                              _dev.schedule_expr(Alg.REDUCE, self.num_peers, 0))
            return self._custom(f, t, values, expr)
        send = Bucket.from_numpy(mine)
        recv = Bucket(mine.size, mine.dtype) if self.peer_id == root else None
        self._comm.reduce(Op(int(f.op)), send, recv, root, ordered=ordered)
        self._comm.sync()
        return self._py(recv.numpy(), t) if recv is not None else self._py(np.zeros_like(mine), t)

    def allreduce(self, data, f: func, t: types):
        mine = self._array(data, t)
        comm_, assoc = self._flags(f, t)
        ordered = not (comm_ and assoc)
        if f.op == op.custom:
            values = self._custom_values(mine)
            alg = Alg.REDUCE_LTR if ordered else Alg.ALLREDUCE
            return self._custom(f, t, values, _dev.schedule_expr(alg, self.num_peers, self.peer_id))
        # host buckets straight through the host-ingress pipeline (fmi_comm_allreduce_host)
        recv = np.empty_like(mine)
        self._comm.allreduce_host(Op(int(f.op)), np.ascontiguousarray(mine), recv, ordered=ordered)
        return self._py(recv, t)

    def scan(self, data, f: func, t: types):
        mine = self._array(data, t)
        comm_, assoc = self._flags(f, t)
        ordered = not (comm_ and assoc)
        if f.op == op.custom:
            values = self._custom_values(mine)
            alg = Alg.SCAN_LTR if ordered else Alg.SCAN
            return self._custom(f, t, values, _dev.schedule_expr(alg, self.num_peers, self.peer_id))
        send, recv = Bucket.from_numpy(mine), Bucket(mine.size, mine.dtype)
        self._comm.scan(Op(int(f.op)), send, recv, ordered=ordered)
        self._comm.sync()
        return self._py(recv.numpy(), t)

    def hint(self, h: hints) -> None:
        self._hint = hints(h)


__all__ = ["Communicator", "Timeout", "datatypes", "func", "hints", "op", "types"]
_ = _lib  # the C-ABI is loaded through fmi_amd.device
