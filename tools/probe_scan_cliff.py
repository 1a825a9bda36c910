"""Probe of the many-peer, small-bucket scan regime: scan / scan_ltr time against P and bucket
size, no-re-use protocol. `--short` runs only scan_ltr P = 64 and 256 at 4 MiB; `--carved` runs those two with every bucket a view into
one allocation per role (inputs, each output set) against separate allocations.

    python tools/probe_scan_cliff.py [--short]
"""
import json, os, sys, numpy as np
_here = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(_here)); sys.path.insert(0, _here)
import fmi_amd
from fmi_amd import Alg, Bucket, Op
from bench_configs import timed_fresh
MIB = 1 << 20
fmi_amd.init(0)
CASES = [(Alg.SCAN_LTR, 128, 4), (Alg.SCAN_LTR, 160, 4), (Alg.SCAN_LTR, 192, 4), (Alg.SCAN_LTR, 256, 4),
           (Alg.SCAN_LTR, 256, 1), (Alg.SCAN_LTR, 256, 16), (Alg.SCAN, 128, 4), (Alg.SCAN, 256, 4),
                    (Alg.SCAN_LTR, 64, 4), (Alg.SCAN_LTR, 128, 8)]
CARVED = "--carved" in sys.argv
if "--short" in sys.argv or CARVED:
    CASES = [(Alg.SCAN_LTR, 64, 4), (Alg.SCAN_LTR, 256, 4)]
for carved in ((False, True) if CARVED else (False,)):
  for alg, P, mib in CASES:
    n = mib * MIB // 4
    sets = 2
    if carved:
        big_in = Bucket(P * n, np.float32)
        ins = [big_in.view(p * n, n).fill_synthetic(7, p) for p in range(P)]
        big_out = [Bucket(P * n, np.float32) for _ in range(sets)]
        outs = [[b.view(p * n, n) for p in range(P)] for b in big_out]
    else:
        ins = [Bucket(n, np.float32).fill_synthetic(7, p) for p in range(P)]
        outs = [[Bucket(n, np.float32) for _ in range(P)] for _ in range(sets)]
    med, mn = timed_fresh(lambda k: fmi_amd.scan_peers(Op.SUM, alg, outs[k], ins), 4, sets, reps=3)
    frac = 2 * P * n * 4 / (med * 1e-3) / 8e12
    print(json.dumps({"alg": alg.name, "P": P, "mib": mib, "carved": carved, "us": round(med * 1e3, 1),
                      "frac": round(frac, 4)}), flush=True)
    if carved:
        for b in [big_in] + big_out:
            b.free()
    else:
        for b in ins + [x for o in outs for x in o]:
            b.free()
