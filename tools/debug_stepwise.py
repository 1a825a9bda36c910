"""Debug: run the stepwise (P > 16) allreduce for several ranks/ops repeatedly and report mismatches."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import fmi_amd  # noqa: E402
from fmi_amd import Alg, Bucket, Op  # noqa: E402
from oracle import fmi_oracle as orc  # noqa: E402

fmi_amd.init(0)
P, n = 17, 1027
xs = [orc.synthetic(np.float32, n, 7, p) for p in range(P)]
ins = [Bucket.from_numpy(x) for x in xs]
for op, name in ((Op.SUM, "sum"), (Op.MIN, "min"), (Op.MAX, "max")):
    want, _ = orc.allreduce(xs, orc.OPS[name])
    for trial in range(3):
        for rank in (0, 8, 16):
            out = Bucket(n, np.float32)
            fmi_amd.reduce_tree(op, Alg.ALLREDUCE, out, ins, rank=rank)
            got = out.numpy()
            bad = np.count_nonzero(got.view(np.uint32) != want[rank].view(np.uint32))
            sync_out = Bucket(n, np.float32)
            fmi_amd.sync()
            fmi_amd.reduce_tree(op, Alg.ALLREDUCE, sync_out, ins, rank=rank)
            fmi_amd.sync()
            bad2 = np.count_nonzero(sync_out.numpy().view(np.uint32) != want[rank].view(np.uint32))
            print(name, trial, rank, "mismatch", bad, "after-sync", bad2, flush=True)
