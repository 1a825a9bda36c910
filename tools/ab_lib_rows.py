"""A/B of two builds of libfmi_dev.so on the same box, interleaved: each round runs one child process per
library that times the same P-way rows (tools/bench_configs.py helpers), so box-to-box variation cancels.

    python tools/ab_lib_rows.py --lib-a build/ab_old/libfmi_dev.so --lib-b fmi_amd/lib/libfmi_dev.so
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
sys.path.insert(0, {root!r})
import fmi_amd._lib as L
L.LIB_PATH = {lib!r}
import numpy as np, fmi_amd
from fmi_amd import Alg, Bucket, Op
sys.path.insert(0, {tools!r})
from bench_configs import timed, MIB, PEAK
import json
fmi_amd.init(0)
for P, op in ((16, Op.SUM), (16, Op.MAX), (8, Op.MIN), (24, Op.MAX)):
    n = 1024 * MIB // 4 // P
    ins = [Bucket(n, np.float32).fill_synthetic(7, p) for p in range(P)]
    out = Bucket(n, np.float32)
    med, mn = timed(lambda k: fmi_amd.reduce_tree(op, Alg.ALLREDUCE, out, ins, rank=5), 15, 1)
    gbs = (P + 1) * n * 4 / (med * 1e-3) / 1e9
    print(json.dumps(dict(lib={tag!r}, row=f"allreduce {{op.name.lower()}} f32 P={{P}} rank 5", median_us=round(med * 1e3, 2),
                          frac_of_peak=round(gbs / PEAK, 4))), flush=True)
    del ins, out
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib-a", required=True)
    ap.add_argument("--lib-b", required=True)
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    for r in range(args.rounds):
        for tag, lib in (("a", args.lib_a), ("b", args.lib_b)):
            code = CHILD.format(root=ROOT, lib=os.path.abspath(lib), tools=os.path.join(ROOT, "tools"), tag=tag)
            out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                sys.stderr.write(out.stderr[-3000:])
                raise SystemExit(out.returncode)
            for line in out.stdout.splitlines():
                d = json.loads(line)
                d["round"] = r
                print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
