"""Seeded random sweep over the P-way entry points: random P (1..70 mostly, and 130 / 257 / 333 — no peer
cap — so single fused kernels, one-pass blocked kernels, fused 16-peer block launches over two and three
levels, ragged last blocks, and the 8/16-bit pairwise-pass programs over run-time-sized schedules), algorithm, op, dtype, bucket
length and element offset (aligned and unaligned views), every result bit-exact against the oracle's
simulation of the reference collective. Deterministic: the case list is a function of the seed."""
import os

import numpy as np
import pytest

import fmi_amd
from fmi_amd import Alg, Bucket
from oracle import fmi_oracle as orc
from tests.test_gpu_parity import ALL_DTYPES, OPNAME, OPS, assert_bit_equal, inputs

pytestmark = pytest.mark.gpu


def _seeds(default):
    """FMI_SWEEP_SEEDS=a:b runs seeds a..b-1 instead (long soak runs); the default suite runs two."""
    spec = os.environ.get("FMI_SWEEP_SEEDS")
    if not spec:
        return default
    lo, hi = (int(v) for v in spec.split(":"))
    return list(range(lo, hi))

CASES = 160


def _cases(seed):
    rng = np.random.default_rng(seed)
    for k in range(CASES):
        P = int(rng.choice([1, 2, 3, 5, 8, 13, 16, 17, 23, 31, 32, 33, 40, 47, 64, 70, 130, 257, 333]))
        alg = Alg(int(rng.integers(0, 5)))
        op = OPS[int(rng.integers(0, 4))]
        dtype = ALL_DTYPES[int(rng.integers(0, len(ALL_DTYPES)))]
        n = int(rng.choice([1, 3, 4, 15, 16, 17, 255, 1024, 1031, 4099]))
        off = int(rng.choice([0, 0, 0, 1, 3, 4]))
        rank = int(rng.integers(0, P))
        yield k, P, alg, op, dtype, n, off, rank


@pytest.mark.parametrize("seed", _seeds([1, 2]))
def test_random_p_way_cases(device, seed):
    done = 0
    for k, P, alg, op, dtype, n, off, rank in _cases(seed):
        xs = [inputs(dtype, n + off, p, seed=1000 * seed + k) for p in range(P)]
        big = [Bucket.from_numpy(x) for x in xs]
        ins = [b.view(off, n) for b in big]
        ys = [x[off:] for x in xs]
        fn = orc.OPS[OPNAME[op]]
        what = f"case {k}: P={P} {alg.name} {op.name} {np.dtype(dtype).name} n={n} off={off} rank={rank}"
        with np.errstate(all="ignore"):
            if alg in (Alg.SCAN, Alg.SCAN_LTR):
                ordered = alg == Alg.SCAN_LTR
                want, _ = orc.scan(ys, fn, commutative=not ordered, associative=not ordered)
                outs = [Bucket(n, dtype) for _ in range(P)]
                fmi_amd.scan_peers(op, alg, outs, ins)
                for p in range(P):
                    assert_bit_equal(outs[p].numpy(), want[p], f"{what} peer {p}")
                done += 1
                continue
            out = Bucket(n, dtype)
            fmi_amd.reduce_tree(op, alg, out, ins, rank=rank)
            if alg == Alg.ALLREDUCE:
                want, _ = orc.allreduce(ys, fn)
                want = want[rank]
            elif alg == Alg.REDUCE:
                want, _ = orc.reduce(ys, fn, root=rank)
            else:
                want, _ = orc.reduce(ys, fn, root=0, commutative=False, associative=False)
            assert_bit_equal(out.numpy(), want, what)
            done += 1
    print(f"seed {seed}: {done} cases bit-exact")
    assert done == CASES
