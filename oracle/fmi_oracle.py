"""ORACLE — TEST INFRASTRUCTURE ONLY. Never imported by the product (fmi_amd/), only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg, and there only as the checker.

A CPU restatement of the reference's bucket-reduction path (spcl/fmi @ v1):
  * element ops: the reference built-ins, reference python/PythonCommunicator.h:116-149
    (std::plus / std::multiplies / std::max = (a<b)?b:a / std::min = (b<a)?b:a);
  * the collectives: every peer runs the reference algorithm of src/comm/PeerToPeer.cpp step by step
    (send / recv / local combine `f.f(mine, received)`), peers exchange copies through FIFO mailboxes,
    exactly like the reference's per-pair TCP channels (src/comm/Direct.cpp:25-45). This is an
    event-driven simulation, independent of the round-synchronous programs the kernels are built from
    (fmi_amd/csrc/fmi_schedule.h), so the two restatements check each other.
  * the side effects: commutative reduce/allreduce/scan overwrite the caller's sendbuf
    (reference src/comm/PeerToPeer.cpp:72,103,119,160,179); the simulation returns both buffers.

Pinning. Since round 3 this restatement is pinned by the REFERENCE ITSELF, floats included:
oracle/_ref/libfmi_ref.so (oracle/Makefile) is the reference's own src/comm/PeerToPeer.cpp, compiled unmodified
from /root/reference, run over an in-memory PeerToPeer transport (oracle/ref_harness.cpp; oracle/fmi_ref.py).
Only src/comm/Channel.cpp (the S3 / Redis / Direct factory: aws-sdk-cpp, hiredis, TCPunch) and
include/Communicator.h (boost::property_tree) stay unbuilt; neither is on the evaluation-order path. Checked by
  (1) the reference's own known-answer tests (reference tests/communicator.cpp:94-254,
      tests/channels.cpp:419-690) — tests/golden/reference_kats.json, tests/test_oracle.py;
  (2) the reference's float outputs and exact bracketing — tests/golden/ref_vectors.npz / ref_expr.json
      (tests/golden/make_ref_vectors.py) and live runs of oracle/_ref — tests/test_ref_pinning.py: every
      collective, commutative and left-to-right, every rank / root, sendbuf side effects, bit-exact.
(SURVEY.md Appendix B's table, tests/golden/bracketing.json, came from a survey build with stand-ins and is
kept only as a cross-check.)

Floating point: numpy float32/float64 arithmetic is IEEE round-to-nearest-even with denormals kept,
the same as the reference's libstdc++ loop compiled without fast-math. Integer arrays wrap modulo 2^bits
like the reference's two's-complement int arithmetic.
"""
from __future__ import annotations

from collections import deque
from typing import Callable, Dict, List, Sequence, Tuple

import numpy as np

# ------------------------------------------------------------------------------------------------
# Element ops (reference python/PythonCommunicator.h:131-149)
# ------------------------------------------------------------------------------------------------


def op_sum(a, b):
    return a + b


def op_prod(a, b):
    return a * b


def op_max(a, b):  # std::max(a, b): (a < b) ? b : a
    return np.where(a < b, b, a).astype(np.asarray(a).dtype, copy=False)


def op_min(a, b):  # std::min(a, b): (b < a) ? b : a
    return np.where(b < a, b, a).astype(np.asarray(a).dtype, copy=False)


OPS: Dict[str, Callable] = {"sum": op_sum, "prod": op_prod, "max": op_max, "min": op_min}
OP_IDS = {"sum": 0, "prod": 1, "max": 2, "min": 3}


def sym_combine(a: str, b: str) -> str:
    """Symbolic combine: records the bracketing, left operand = arg 0 of f.f."""
    return f"({a}+{b})"


# ------------------------------------------------------------------------------------------------
# Synthetic buckets: h = splitmix64(seed ^ (peer << 40) ^ i)
# ------------------------------------------------------------------------------------------------
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def synthetic(dtype, n: int, seed: int, peer: int, start: int = 0) -> np.ndarray:
    """Counter-based bucket: element i of peer `peer` (identical to fmi_dev_fill_synthetic)."""
    return synthetic_at(dtype, np.arange(start, start + n, dtype=np.uint64), seed, peer)


def synthetic_at(dtype, idx: np.ndarray, seed: int, peer: int) -> np.ndarray:
    """The synthetic bucket's elements at arbitrary indices (sampled checks of full-size buckets)."""
    dtype = np.dtype(dtype)
    key = np.uint64((seed ^ (peer << 40)) & 0xFFFFFFFFFFFFFFFF)
    h = splitmix64(key ^ np.asarray(idx, dtype=np.uint64))
    if dtype == np.float32:
        u = (h >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)
        return u * np.float32(2.0) - np.float32(1.0)
    if dtype == np.float64:
        u = (h >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)
        return u * 2.0 - 1.0
    if dtype.kind in "iu":  # the top 8·itemsize bits of h (i32 = h >> 32, i64 = h)
        bits = 8 * dtype.itemsize
        top = (h >> np.uint64(64 - bits)) if bits < 64 else h
        return top.astype(np.dtype(f"u{dtype.itemsize}")).view(dtype)
    raise TypeError(f"unsupported dtype {dtype}")


# ------------------------------------------------------------------------------------------------
# Peer simulation: generators yield ("send", dst, value) or ("recv", src) and get the received value.
# ------------------------------------------------------------------------------------------------
class Deadlock(RuntimeError):
    pass


def _copy(v):
    if isinstance(v, np.ndarray):
        return v.copy()
    if isinstance(v, dict):
        return {k: _copy(x) for k, x in v.items()}
    return v


def _run(programs: List) -> List:
    """Drive one generator per peer until all return. Sends are buffered (never block), receives block
    until the matching FIFO mailbox holds a message — the reference's per-peer-pair stream semantics."""
    P = len(programs)
    mail: Dict[Tuple[int, int], deque] = {}
    results = [None] * P
    pending = [None] * P  # value to send into the generator on its next step
    waiting = [None] * P  # src peer a generator is blocked on
    done = [False] * P
    started = [False] * P
    remaining = P
    while remaining:
        progressed = False
        for p in range(P):
            if done[p]:
                continue
            if waiting[p] is not None:
                box = mail.get((waiting[p], p))
                if not box:
                    continue
                pending[p] = box.popleft()
                waiting[p] = None
            while True:
                try:
                    if not started[p]:
                        started[p] = True
                        req = next(programs[p])
                    else:
                        req, pending[p] = programs[p].send(pending[p]), None
                except StopIteration as stop:
                    results[p] = stop.value
                    done[p] = True
                    remaining -= 1
                    progressed = True
                    break
                progressed = True
                if req[0] == "send":
                    _, dst, value = req
                    if not 0 <= dst < P:
                        raise ValueError(f"peer {p} sends to invalid peer {dst}")
                    mail.setdefault((p, dst), deque()).append(_copy(value))
                    pending[p] = None
                    continue
                _, src = req
                if not 0 <= src < P:
                    raise ValueError(f"peer {p} receives from invalid peer {src}")
                box = mail.get((src, p))
                if box:
                    pending[p] = box.popleft()
                    continue
                waiting[p] = src
                break
        if not progressed:
            raise Deadlock(f"peers {[p for p in range(P) if not done[p]]} blocked")
    leftover = {k: len(v) for k, v in mail.items() if v}
    if leftover:
        raise RuntimeError(f"unconsumed messages {leftover}")
    return results


def _ceil_log2(v: int) -> int:
    r = 0
    while (1 << r) < v:
        r += 1
    return r


def _floor_log2(v: int) -> int:
    r = 0
    while (2 << r) <= v:
        r += 1
    return r


def _fwd(me: int, root: int, P: int) -> int:  # transform_peer_id forward, PeerToPeer.cpp:287-293
    return (me + P - root) % P


def _back(t: int, root: int, P: int) -> int:  # transform_peer_id backward
    return (t + root) % P


def _bcast(me, P, buf, root):
    """Binomial broadcast, reference src/comm/PeerToPeer.cpp:14-27."""
    t = _fwd(me, root, P)
    for i in reversed(range(_ceil_log2(P))):
        step = 1 << i
        if t % (2 * step) == 0 and t + step < P:
            yield ("send", _back(t + step, root, P), buf)
        elif t % step == 0 and t % (2 * step) != 0:
            buf = yield ("recv", _back(t - step, root, P))
    return buf


def _gather(me, P, send, root):
    """Binomial gather, reference src/comm/PeerToPeer.cpp:186-239. A peer's message carries the buckets
    of the transformed ids it is responsible for; the root lays them out by real peer id (with the
    wraparound copy of :213-222), so the result is indexed by real id."""
    t = _fwd(me, root, P)
    held = {t: send}
    for i in range(_ceil_log2(P)):
        step = 1 << i
        if t % (2 * step) == 0 and t + step < P:
            responsible = min(step, P - (t + step))
            chunk = yield ("recv", _back(t + step, root, P))
            if len(chunk) != responsible:
                raise RuntimeError("gather: unexpected chunk size")
            held.update(chunk)
        elif t % step == 0 and t % (2 * step) != 0:
            yield ("send", _back(t - step, root, P), dict(held))
    if me == root:
        return [held[_fwd(r, root, P)] for r in range(P)]
    return None


def _reduce_ltr(me, P, send, root, f):
    """Reference src/comm/PeerToPeer.cpp:44-57: gather, then ((x0 f x1) f x2) ... at the root."""
    gathered = yield from _gather(me, P, send, root)
    if me != root:
        return None, send
    acc = gathered[0]
    for i in range(1, P):
        acc = f(acc, gathered[i])
    return acc, send


def _reduce_no_order(me, P, send, root, f):
    """Reference src/comm/PeerToPeer.cpp:59-84: binomial tree on transformed ids, f(own, received)."""
    t = _fwd(me, root, P)
    for i in range(_ceil_log2(P)):
        step = 1 << i
        if t % (2 * step) == 0 and t + step < P:
            got = yield ("recv", _back(t + step, root, P))
            send = f(send, got)
        elif t % step == 0 and t % (2 * step) != 0:
            yield ("send", _back(t - step, root, P), send)
    return (send if me == root else None), send


def _allreduce_no_order(me, P, send, f):
    """Reference src/comm/PeerToPeer.cpp:96-130: fold of the peers above 2^floor(log2 P), recursive
    doubling, result handed back to the folded peers; recvbuf = sendbuf at the end (:129)."""
    rounds = _floor_log2(P)
    pow2 = 1 << rounds
    if P > pow2:
        if me < pow2 and me + pow2 < P:
            got = yield ("recv", me + pow2)
            send = f(send, got)
        elif me >= pow2:
            yield ("send", me - pow2, send)
    if me < pow2:
        for i in range(rounds):
            peer = me ^ (1 << i)
            if peer < me:
                yield ("send", peer, send)
                got = yield ("recv", peer)
            else:
                got = yield ("recv", peer)
                yield ("send", peer, send)
            send = f(send, got)
    if P > pow2:
        if me < pow2 and me + pow2 < P:
            yield ("send", me + pow2, send)
        elif me >= pow2:
            send = yield ("recv", me - pow2)
    return send, send


def _scan_ltr(me, P, send, f):
    """Reference src/comm/PeerToPeer.cpp:141-152: chain; recv prefix, f(prefix, own), pass on."""
    if me == 0:
        if P > 1:
            yield ("send", 1, send)
        return send, send
    prefix = yield ("recv", me - 1)
    prefix = f(prefix, send)
    if me < P - 1:
        yield ("send", me + 1, prefix)
    return prefix, send


def _scan_no_order(me, P, send, f):
    """Reference src/comm/PeerToPeer.cpp:154-184: binomial up-sweep then down-sweep, f(own, received)."""
    rounds = _floor_log2(P)
    for i in range(rounds):
        full = (1 << (i + 1)) - 1
        low = (1 << i) - 1
        if me & full == full:
            got = yield ("recv", me - (1 << i))
            send = f(send, got)
        elif me & low == low:
            if me + (1 << i) < P:
                yield ("send", me + (1 << i), send)
                break
    for i in range(rounds, 0, -1):
        hi = (1 << i) - 1
        lo = (1 << (i - 1)) - 1
        if me & hi == hi:
            if me + (1 << (i - 1)) < P:
                yield ("send", me + (1 << (i - 1)), send)
        elif me & lo == lo:
            src = me - (1 << (i - 1))
            if src > 0:
                got = yield ("recv", src)
                send = f(send, got)
    return send, send


def _allreduce(me, P, send, f, ordered):
    """Reference src/comm/PeerToPeer.cpp:86-94."""
    if ordered:
        res, send = yield from _reduce_ltr(me, P, send, 0, f)
        res = yield from _bcast(me, P, res, 0)
        return res, send
    return (yield from _allreduce_no_order(me, P, send, f))


# ------------------------------------------------------------------------------------------------
# Public entry points: P peers' buckets in, each peer's (recvbuf, sendbuf-after-call) out.
# ------------------------------------------------------------------------------------------------
def _ltr(commutative: bool, associative: bool) -> bool:
    # reference include/Communicator.h:92,116 and src/comm/PeerToPeer.cpp:36,87,133
    return not (commutative and associative)


def reduce(xs: Sequence, f: Callable, root: int = 0, commutative: bool = True, associative: bool = True):
    P = len(xs)
    ordered = _ltr(commutative, associative)
    alg = _reduce_ltr if ordered else _reduce_no_order
    out = _run([alg(p, P, _copy(xs[p]), root, f) for p in range(P)])
    return out[root][0], [o[1] for o in out]


def allreduce(xs: Sequence, f: Callable, commutative: bool = True, associative: bool = True):
    P = len(xs)
    out = _run([_allreduce(p, P, _copy(xs[p]), f, _ltr(commutative, associative)) for p in range(P)])
    return [o[0] for o in out], [o[1] for o in out]


def scan(xs: Sequence, f: Callable, commutative: bool = True, associative: bool = True):
    P = len(xs)
    alg = _scan_ltr if _ltr(commutative, associative) else _scan_no_order
    out = _run([alg(p, P, _copy(xs[p]), f) for p in range(P)])
    return [o[0] for o in out], [o[1] for o in out]


def bcast(xs: Sequence, root: int):
    P = len(xs)
    return _run([_bcast(p, P, _copy(xs[p]), root) for p in range(P)])


def gather(xs: Sequence, root: int):
    P = len(xs)
    return _run([_gather(p, P, _copy(xs[p]), root) for p in range(P)])[root]


def symbols(P: int) -> List[str]:
    return [f"x{p}" for p in range(P)]


def expr(kind: str, P: int, rank: int = 0, root: int = 0, ordered: bool = False) -> str:
    """Symbolic expression peer `rank` (or the root) ends with — the reference's bracketing."""
    flags = dict(commutative=not ordered, associative=not ordered)
    if kind == "allreduce":
        return allreduce(symbols(P), sym_combine, **flags)[0][rank]
    if kind == "reduce":
        return reduce(symbols(P), sym_combine, root=root, **flags)[0]
    if kind == "scan":
        return scan(symbols(P), sym_combine, **flags)[0][rank]
    raise ValueError(kind)


def pairwise(op: str, a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """One reference combine f.f(a, b) with a built-in op (include/Communicator.h:180-189)."""
    return OPS[op](a, b)
