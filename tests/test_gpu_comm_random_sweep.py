"""Seeded random sweep over the C-ABI communicator (LOCAL transport, ranks as threads on the one GPU):
random rank count, collective, order (commutative or left-to-right), op, dtype and bucket length — the
shard grid, its zero padding, the all-to-all, the fused (or blocked) shard program and the gather /
all-to-all back — every rank's result bit-exact against the oracle's simulation of the reference
collective. Since round 5 also the host-ingress allreduce (fmi_comm_allreduce_host: page-locked or pageable
host buckets, a random chunk giving 1-12 chunks, through the device's shared copy streams, two or three chunk
slots deep). Deterministic: the case list is a function of the seed."""
import os

import numpy as np
import pytest

import fmi_amd
from fmi_amd import Bucket, PinnedArray
from fmi_amd.comm import Path
from oracle import fmi_oracle as orc
from tests.test_gpu_comm import run_ranks
from tests.test_gpu_parity import ALL_DTYPES, OPNAME, OPS, assert_bit_equal, inputs

pytestmark = pytest.mark.gpu


def _seeds(default):
    """FMI_SWEEP_SEEDS=a:b runs seeds a..b-1 instead (long soak runs); the default suite runs two."""
    spec = os.environ.get("FMI_SWEEP_SEEDS")
    if not spec:
        return default
    lo, hi = (int(v) for v in spec.split(":"))
    return list(range(lo, hi))

CASES = 48


def _cases(seed):
    rng = np.random.default_rng(seed)
    for k in range(CASES):
        N = int(rng.choice([1, 2, 3, 4, 5, 7, 8, 11, 16, 19]))
        kind = str(rng.choice(["allreduce", "allreduce_direct", "allreduce_host", "reduce", "reduce_sendbuf", "scan"]))
        ordered = bool(rng.integers(0, 2))
        op = OPS[int(rng.integers(0, 4))]
        dtype = ALL_DTYPES[int(rng.integers(0, len(ALL_DTYPES)))]
        n = int(rng.choice([1, 5, 64, 255, 1000, 4099, 65536 + 7]))
        root = int(rng.integers(0, N))
        chunk = max(1, n // int(rng.integers(1, 13)))  # allreduce_host: 1-12 chunks (rounded by the library)
        yield k, N, kind, ordered, op, dtype, n, root, chunk


@pytest.mark.parametrize("seed", _seeds([11, 12]))
def test_random_comm_cases(device, seed):
    done = 0
    for k, N, kind, ordered, op, dtype, n, root, chunk in _cases(seed):
        xs = [inputs(dtype, n, r, seed=500 * seed + k) for r in range(N)]

        def body(c, r):
            s, out = Bucket.from_numpy(xs[r]), Bucket(n, dtype)
            if kind == "allreduce":
                c.allreduce(op, s, out, ordered=ordered)
            elif kind == "allreduce_direct":
                w = c.window(n, dtype)
                w.upload(xs[r])
                c.allreduce(op, w, out, ordered=ordered, path=Path.DIRECT)
                fmi_amd.sync()
                got = out.numpy()
                c.window_free(w)
                return got
            elif kind == "allreduce_host":  # even ranks page-locked buckets, odd ranks pageable
                if r % 2 == 0:
                    hs, ho = PinnedArray(n, dtype), PinnedArray(n, dtype)
                    hs.array[:] = xs[r]
                    c.allreduce_host(op, hs.array, ho.array, ordered=ordered, chunk=chunk)
                    got = ho.array.copy()
                    hs.free()
                    ho.free()
                    return got
                got = np.zeros(n, dtype)
                c.allreduce_host(op, xs[r].copy(), got, ordered=ordered, chunk=chunk)
                return got
            elif kind == "reduce":
                c.reduce(op, s, out if r == root else None, root, ordered=ordered)
            elif kind == "reduce_sendbuf":  # every sendbuf as the reference leaves it (PeerToPeer.cpp:72)
                c.reduce(op, s, out if r == root else None, root, ordered=ordered, sendbuf_partials=True)
                fmi_amd.sync()
                return out.numpy(), s.numpy()
            else:
                c.scan(op, s, out, ordered=ordered)
            fmi_amd.sync()
            return out.numpy()

        res = run_ranks(N, body)
        fn = orc.OPS[OPNAME[op]]
        what = f"case {k}: N={N} {kind} ordered={ordered} {op.name} {np.dtype(dtype).name} n={n}"
        with np.errstate(all="ignore"):
            if kind.startswith("allreduce"):
                want, _ = orc.allreduce(xs, fn, commutative=not ordered, associative=not ordered)
                for r in range(N):
                    assert_bit_equal(res[r], want[r], f"{what} rank {r}")
            elif kind == "reduce":
                want, _ = orc.reduce(xs, fn, root=root, commutative=not ordered, associative=not ordered)
                assert_bit_equal(res[root], want, f"{what} root {root}")
            elif kind == "reduce_sendbuf":
                want, sends = orc.reduce(xs, fn, root=root, commutative=not ordered, associative=not ordered)
                assert_bit_equal(res[root][0], want, f"{what} root {root}")
                for r in range(N):
                    assert_bit_equal(res[r][1], sends[r], f"{what} sendbuf of rank {r}")
            else:
                want, _ = orc.scan(xs, fn, commutative=not ordered, associative=not ordered)
                for r in range(N):
                    assert_bit_equal(res[r], want[r], f"{what} rank {r}")
        done += 1
    print(f"seed {seed}: {done} cases bit-exact")
    assert done == CASES
