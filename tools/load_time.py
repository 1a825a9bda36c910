"""Load time of libfmi_dev.so on a GPU box: import + fmi_dev_init, first pairwise launch, first fused tree.
FMI_DEV_LIB=<path> selects another build (used to compare the compressed and uncompressed code objects)."""
import sys, time
sys.path.insert(0, ".")
t0 = time.time()
import numpy as np
import fmi_amd
from fmi_amd import Alg, Bucket, Op
fmi_amd.init(0)
t1 = time.time()
a, b = Bucket(1 << 20, np.float32), Bucket(1 << 20, np.float32)
fmi_amd.reduce_pair(Op.SUM, a, b); fmi_amd.sync()
t2 = time.time()
ins = [Bucket(4099, np.float32) for _ in range(8)]
fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, ins[0], ins); fmi_amd.sync()
t3 = time.time()
print(f"{fmi_amd.LIB_PATH}: import+init {t1-t0:.3f} s, first pair {t2-t1:.3f} s, first tree {t3-t2:.3f} s")
