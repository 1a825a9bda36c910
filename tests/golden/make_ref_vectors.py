"""Generates the reference's own float outputs as fixtures (run in the build container, where /root/reference
exists and oracle/_ref/libfmi_ref.so is built by `make -C oracle`):

  tests/golden/ref_vectors.npz  inputs + the REFERENCE's results (src/comm/PeerToPeer.cpp compiled unmodified,
                                run by oracle/ref_harness.cpp) for float allreduce / reduce / scan, commutative
                                and left-to-right, every rank / several roots, with each peer's sendbuf after
                                the call.
  tests/golden/ref_expr.json    the reference's exact bracketing (symbolic run) for P = 1 .. 20, every rank
                                (reduce: every root), commutative and left-to-right.

These pin the float evaluation order that the reference's integer-only tests cannot. The GPU
parity tests (tests/test_gpu_ref_vectors.py) compare the HIP path against them directly; tests/test_ref_pinning.py
checks the oracle restatement against them and, where the library is built, that they still equal a live run.

Usage: python tests/golden/make_ref_vectors.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import fmi_oracle as orc  # noqa: E402
from oracle import fmi_ref as ref  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
PEERS = list(range(1, 10)) + [12, 13, 16, 17, 24, 31, 32, 33, 48, 64]
N = 19  # 16 + a 3-element tail (vector kernels' ragged end); element 0..7 carry edge values
CASES = [(np.float32, op) for op in ("sum", "prod", "max", "min")] + [(np.float64, "sum"), (np.float64, "max")]
# round 4: the rest of f64 and the integer types, at fewer peer counts (integer results do not depend on the
# bracketing, so these pin the element semantics: wrapping sum / prod, std::max / std::min on the extremes)
EXTRA_CASES = [(np.float64, "prod"), (np.float64, "min")] + [(dt, op) for dt in (np.int32, np.int64)
                                                             for op in ("sum", "prod", "max", "min")]
EXTRA_PEERS = [1, 2, 3, 5, 8, 13, 17, 33]
EXPR_PEERS = range(1, 21)


def fixture_inputs(dtype, P, seed):
    """Peer p: the synthetic bucket scaled by 2^((7p mod 13) - 6) (exact), so that sums of peers of different
    magnitudes round differently under different bracketings; elements 0..7 carry the edge values (signed
    zeros, infinities, NaN, subnormals, the largest finite) rotated by peer, which decide max / min order."""
    if np.issubdtype(dtype, np.integer):  # integers: the full-range synthetic bucket plus the extremes
        ii = np.iinfo(dtype)
        edge = np.array([ii.min, ii.max, 0, -1, 1, ii.min + 1, ii.max - 1, 2], dtype=dtype)
        xs = []
        for p in range(P):
            x = orc.synthetic(dtype, N, seed=seed, peer=p)
            x[:8] = np.roll(edge, p)
            xs.append(x)
        return np.stack(xs)
    fi = np.finfo(dtype)
    edge = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, fi.tiny / 4, -fi.max, fi.smallest_subnormal], dtype=dtype)
    xs = []
    for p in range(P):
        x = orc.synthetic(dtype, N, seed=seed, peer=p) * dtype(2.0 ** ((7 * p) % 13 - 6))
        x[:8] = np.roll(edge, p)
        xs.append(x.astype(dtype))
    return np.stack(xs)


def roots_of(P):
    return sorted({0, 1 % P, P // 2, P - 1})


def main():
    if not ref.available():
        raise SystemExit(f"{ref.LIB_PATH} missing: make -C oracle (needs /root/reference)")
    out = {}
    with np.errstate(all="ignore"):
        for dtype, op, peers in [(d, o, PEERS) for d, o in CASES] + [(d, o, EXTRA_PEERS) for d, o in EXTRA_CASES]:
            dn = np.dtype(dtype).name
            for P in peers:
                if dtype == np.float64 and P > 33:
                    continue
                xs = fixture_inputs(dtype, P, seed=1000 + P)
                key = f"{dn}/{op}/P{P}"
                out[f"{key}/in"] = xs
                r, s, _ = ref.run("allreduce", op, xs)
                out[f"{key}/allreduce/recv"], out[f"{key}/allreduce/send"] = r, s
                r, _, _ = ref.run("allreduce", op, xs, ordered=True)
                out[f"{key}/allreduce_ltr/recv"] = r
                r, s, _ = ref.run("scan", op, xs)
                out[f"{key}/scan/recv"], out[f"{key}/scan/send"] = r, s
                r, _, _ = ref.run("scan", op, xs, ordered=True)
                out[f"{key}/scan_ltr/recv"] = r
                for root in roots_of(P):
                    r, s, _ = ref.run("reduce", op, xs, root=root)
                    out[f"{key}/reduce/root{root}/recv"], out[f"{key}/reduce/root{root}/send"] = r[root], s
                    r, _, _ = ref.run("reduce", op, xs, root=root, ordered=True)
                    out[f"{key}/reduce_ltr/root{root}/recv"] = r[root]
    np.savez_compressed(os.path.join(HERE, "ref_vectors.npz"), **out)
    exprs = {"generator": "tests/golden/make_ref_vectors.py (oracle/_ref: reference src/comm/PeerToPeer.cpp)",
             "convention": "x<p> = peer p's bucket; (a+b) = f.f(a, b), a = the left operand (overwritten)",
             "allreduce": {}, "allreduce_ltr": {}, "reduce": {}, "reduce_ltr": {}, "scan": {}, "scan_ltr": {}}
    for P in EXPR_PEERS:
        for kind in ("allreduce", "reduce", "scan"):
            for ordered in (False, True):
                exprs[kind + ("_ltr" if ordered else "")][str(P)] = ref.exprs(kind, P, ordered=ordered)
    with open(os.path.join(HERE, "ref_expr.json"), "w") as f:
        json.dump(exprs, f, indent=0, sort_keys=True)
        f.write("\n")
    print(f"wrote {len(out)} arrays and {sum(len(v) for k, v in exprs.items() if isinstance(v, dict))} "
          f"expression lists")


if __name__ == "__main__":
    main()
