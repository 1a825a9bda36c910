"""HIP graphs through the C-ABI (fmi_graph_*): a recorded sequence of bucket combines replays with the same
results as the direct launches, against the oracle; a call that cannot be captured fails loudly (the stream
is then replaced, as HIP leaves an invalidated capture's stream unusable)."""
import numpy as np
import pytest

import fmi_amd
from fmi_amd import Alg, Bucket, Graph, Op, Stream
from oracle import fmi_oracle as orc
from tests.test_gpu_parity import OPNAME, assert_bit_equal, inputs

pytestmark = pytest.mark.gpu


def test_graph_replays_combines_and_p_way_kernels(device):
    s = Stream()
    n = (1 << 18) + 5  # 1 MiB of f32 and a ragged tail
    K = 24
    a = [inputs(np.float32, n, 2 * k, seed=61) for k in range(K)]
    b = [inputs(np.float32, n, 2 * k + 1, seed=61) for k in range(K)]
    da, db = [Bucket.from_numpy(x) for x in a], [Bucket.from_numpy(x) for x in b]
    peers = [inputs(np.int64, n, p, seed=62) for p in range(8)]
    dp = [Bucket.from_numpy(x) for x in peers]
    tree_out = Bucket(n, np.int64)
    scan_out = [Bucket(n, np.int64) for _ in range(4)]

    def record():
        for k in range(K):
            fmi_amd.reduce_pair(Op.SUM, da[k], db[k], stream=s)
        fmi_amd.reduce_tree(Op.MAX, Alg.ALLREDUCE, tree_out, dp, stream=s)
        fmi_amd.scan_peers(Op.SUM, Alg.SCAN, scan_out, dp[:4], stream=s)

    g = Graph.capture(s, record)
    s.sync()
    for k in range(K):  # recorded, not run
        assert_bit_equal(da[k].numpy(), a[k], f"bucket {k} untouched by the capture")
    with np.errstate(all="ignore"):
        once = [orc.pairwise("sum", a[k], b[k]) for k in range(K)]
        twice = [orc.pairwise("sum", once[k], b[k]) for k in range(K)]
        want_tree, _ = orc.allreduce(peers, orc.op_max)
        want_scan, _ = orc.scan(peers[:4], orc.op_sum)
    g.launch(s)
    s.sync()
    for k in range(K):
        assert_bit_equal(da[k].numpy(), once[k], f"replay 1, bucket {k}")
    assert_bit_equal(tree_out.numpy(), want_tree[0], "replayed fused tree")
    for r in range(4):
        assert_bit_equal(scan_out[r].numpy(), want_scan[r], f"replayed fused scan, peer {r}")
    g.launch(s)  # in-place combines accumulate: the graph recomputes from the buckets as they are now
    s.sync()
    for k in range(K):
        assert_bit_equal(da[k].numpy(), twice[k], f"replay 2, bucket {k}")
    g.destroy()
    s.destroy()


def test_graph_capture_of_a_synchronising_call_fails_loudly(device):
    s = Stream()
    x, y = Bucket.from_numpy(np.ones(4096, np.float32)), Bucket.from_numpy(np.ones(4096, np.float32))

    def record():
        fmi_amd.reduce_pair(Op.SUM, x, y, stream=s)
        s.sync()  # a host synchronisation cannot be recorded

    with pytest.raises(fmi_amd.FmiError):
        Graph.capture(s, record)
    s.destroy()  # HIP leaves a stream whose capture was invalidated unusable: replace it (include/fmi_dev.h)
    s = Stream()
    assert np.all(x.numpy() == 1.0)  # nothing recorded ran
    fmi_amd.reduce_pair(Op.SUM, x, y, stream=s)
    s.sync()
    assert np.all(x.numpy() == 2.0)
    g = Graph.capture(s, lambda: fmi_amd.reduce_pair(Op.SUM, x, y, stream=s))  # capture works again
    g.launch(s)
    s.sync()
    assert np.all(x.numpy() == 3.0)
    g.destroy()
    with pytest.raises(fmi_amd.FmiError):  # the library's own (null) stream is not capturable by callers
        fmi_amd._lib.call("fmi_graph_capture_begin", None)
    s.destroy()


def test_graph_replays_device_copies(device):
    """fmi_dev_d2d_async inside a graph: the copy kernel (aligned device buckets of >= 256 KiB, whose pointer
    check runs at capture time) and the runtime copy (small or unaligned) are both recorded and replayed."""
    s = Stream()
    big = 1 << 20  # floats: 4 MiB, the copy_tile kernel
    a, b = Bucket.from_numpy(np.arange(big, dtype=np.float32)), Bucket(big, np.float32)
    c, d = Bucket.from_numpy(np.arange(100, dtype=np.float32)), Bucket(100, np.float32)

    def record():
        b.copy_from(a, stream=s)
        d.copy_from(c, stream=s)

    g = Graph.capture(s, record)
    for k in (1, 2):
        a.upload(np.arange(big, dtype=np.float32) * k)
        c.upload(np.arange(100, dtype=np.float32) * k)
        g.launch(s)
        s.sync()
        assert np.array_equal(b.numpy(), np.arange(big, dtype=np.float32) * k)
        assert np.array_equal(d.numpy(), np.arange(100, dtype=np.float32) * k)
    g.destroy()
    s.destroy()
    for x in (a, b, c, d):
        x.free()


def test_graph_capture_of_an_arena_call_is_refused(device):
    """A call that needs the library's scratch arena (here an unaligned 4-peer reduce_tree, which runs the
    program as pairwise passes through arena temps) is refused while its stream is capturing: the arena's
    ordering event would be recorded inside the graph and its replays would race later direct calls
    (include/fmi_dev.h). FMI_ERR_UNSUPPORTED, and the stream works afterwards."""
    from fmi_amd import Alg

    s = Stream()
    n = 4099
    base = [Bucket.from_numpy(np.full(n + 1, p + 1, np.float32)) for p in range(4)]
    ins = [b.view(1, n) for b in base]  # 4-byte offset: not 16-B aligned
    out = Bucket(n, np.float32)
    with pytest.raises(fmi_amd.FmiError, match="FMI_ERR_UNSUPPORTED.*graph"):
        Graph.capture(s, lambda: fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, out, ins, stream=s))
    s.destroy()
    s = Stream()
    fmi_amd.reduce_tree(Op.SUM, Alg.ALLREDUCE, out, ins, stream=s)
    s.sync()
    assert np.all(out.numpy() == 10.0)
    s.destroy()


@pytest.mark.parametrize("dtype", [np.float32, np.int64, np.uint8, np.float64], ids=lambda d: np.dtype(d).name)
def test_pair_batch_matches_separate_combines(device, dtype):
    """fmi_dev_reduce_pair_batch: many buckets of mixed sizes (empty, below one 16-B lane group, ragged,
    several tiles) and more descriptors than one launch takes (64), every op, against the oracle; an
    unaligned bucket in the batch takes its own launch."""
    sizes = [0, 1, 3, 17, 4099, 65536 + 7, 1 << 18, 5] * 12  # 96 descriptors
    for op in (Op.SUM, Op.PROD, Op.MAX, Op.MIN):
        a = [inputs(dtype, n, 2 * k, seed=71) for k, n in enumerate(sizes)]
        b = [inputs(dtype, n, 2 * k + 1, seed=71) for k, n in enumerate(sizes)]
        da = [Bucket.from_numpy(x) for x in a]
        db = [Bucket.from_numpy(x) for x in b]
        pairs = list(zip(da, db))
        big = Bucket.from_numpy(np.concatenate([a[6], a[6][:1]]))  # an unaligned view as one more inout
        unaligned = big.view(1, sizes[6])
        ua = big.numpy()[1:].copy()
        pairs.append((unaligned, db[6]))
        fmi_amd.reduce_pair_batch(op, pairs)
        fmi_amd.sync()
        with np.errstate(all="ignore"):
            for k in range(len(sizes)):
                assert_bit_equal(da[k].numpy(), orc.pairwise(OPNAME[op], a[k], b[k]), f"{op.name} descriptor {k}")
            assert_bit_equal(unaligned.numpy(), orc.pairwise(OPNAME[op], ua, b[6]), f"{op.name} unaligned")


def test_pair_batch_rejects_overlap_and_is_graph_capturable(device):
    x = Bucket.from_numpy(np.ones(8192, np.float32))
    y = Bucket.from_numpy(np.ones(8192, np.float32))
    with pytest.raises(fmi_amd.FmiError):  # two descriptors writing the same bytes
        fmi_amd.reduce_pair_batch(Op.SUM, [(x.view(0, 4096), y.view(0, 4096)), (x.view(1024, 4096), y.view(0, 4096))])
    with pytest.raises(fmi_amd.FmiError):  # one reads what another writes
        fmi_amd.reduce_pair_batch(Op.SUM, [(x.view(0, 4096), y.view(0, 4096)), (y.view(0, 4096), x.view(0, 4096))])
    s = Stream()
    g = Graph.capture(s, lambda: fmi_amd.reduce_pair_batch(Op.SUM, [(x.view(0, 4096), y.view(0, 4096)),
                                                                      (x.view(4096, 4096), y.view(4096, 4096))],
                                                           stream=s))
    g.launch(s)
    g.launch(s)
    s.sync()
    assert np.all(x.numpy() == 3.0)
    g.destroy()
    s.destroy()
